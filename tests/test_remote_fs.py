"""s3:// (SigV4), azure:// (SharedKey) and http:// backends against in-process
mock servers that verify request signatures: streams, ranged reads larger and
smaller than the read-ahead block, multipart / block-list uploads, paginated
listings, and sharded InputSplit + parser over remote files."""
import os

import numpy as np
import pytest

import mock_remote
from dmlc_core_amd import _dmlc, data, io

pytestmark = pytest.mark.skipif(not os.path.exists("/usr/lib/x86_64-linux-gnu/libcurl.so.4"),
                                reason="libcurl not installed")


@pytest.fixture(scope="module")
def s3():
    srv = mock_remote.serve(mock_remote.S3Handler)
    os.environ.update({"S3_ENDPOINT": f"http://127.0.0.1:{srv.server_address[1]}",
                       "S3_ACCESS_KEY_ID": "AKIDTEST", "S3_SECRET_ACCESS_KEY": "secret",
                       "S3_REGION": "us-east-1", "DMLC_S3_WRITE_BUFFER_MB": "5"})
    yield mock_remote.S3Handler
    srv.shutdown()


@pytest.fixture(scope="module")
def azure():
    srv = mock_remote.serve(mock_remote.AzureHandler)
    os.environ.update({"AZURE_STORAGE_ENDPOINT": f"http://127.0.0.1:{srv.server_address[1]}",
                       "AZURE_STORAGE_ACCOUNT": mock_remote.AzureHandler.account,
                       "AZURE_STORAGE_ACCESS_KEY": mock_remote.AzureHandler.key})
    yield mock_remote.AzureHandler
    srv.shutdown()


def _blob(n, seed=0):
    return np.random.default_rng(seed).integers(0, 256, n, dtype=np.uint8).tobytes()


def _read_all(uri, chunk=1 << 20):
    s = io.Stream(uri, "r")
    out = bytearray()
    while True:
        b = s.read(chunk)
        if not b:
            return bytes(out)
        out += b


def test_s3_write_read_roundtrip_multipart(s3):
    payload = _blob(12 * (1 << 20) + 12345)  # > 2 parts of 5 MiB
    w = io.Stream("s3://bk1/dir/obj.bin", "w")
    for i in range(0, len(payload), 3 << 20):
        w.write(payload[i:i + (3 << 20)])
    w.close()
    assert s3.store["bk1/dir/obj.bin"] == payload
    assert _read_all("s3://bk1/dir/obj.bin", chunk=64 << 20) == payload  # direct-to-buffer path
    assert _read_all("s3://bk1/dir/obj.bin", chunk=4096) == payload      # read-ahead path


def test_s3_small_put_and_listing_pagination(s3):
    for i in range(5):
        w = io.Stream(f"s3://bk2/data/part-{i}.txt", "w")
        w.write(f"{i} 1:{i}\n".encode() * (i + 1))
        w.close()
    w = io.Stream("s3://bk2/data/sub/x.txt", "w")
    w.write(b"0 1:1\n")
    w.close()
    # a text InputSplit over the "directory" lists every object (pages of 2)
    split_recs = []
    for part in range(3):
        split_recs += [r.rstrip(b"\x00\n") for r in io.iter_records("s3://bk2/data", part, 3, "text")]
    expect = [f"{i} 1:{i}".encode() for i in range(5) for _ in range(i + 1)]
    assert split_recs == expect  # sub/ is a directory and is not descended into


def test_s3_parser_matches_local(s3, tmp_path):
    local = tmp_path / "s.libsvm"
    data.write_synthetic(str(local), 0, 3000, seed=3)
    raw = local.read_bytes()
    w = io.Stream("s3://bk3/train.libsvm", "w")
    w.write(raw)
    w.close()
    for nparts in (1, 2):
        for part in range(nparts):
            a = list(data.iter_blocks("s3://bk3/train.libsvm", part, nparts, type="libsvm"))
            b = list(data.iter_blocks(str(local), part, nparts, type="libsvm"))
            import pyref
            ca, cb = pyref.concat_blocks(a), pyref.concat_blocks(b)
            np.testing.assert_array_equal(ca["index"], cb["index"])
            np.testing.assert_array_equal(ca["value"], cb["value"])


def test_s3_parallel_ranged_partition_reads(s3, tmp_path):
    """The GPU ring's host stage (ShardReader) splits each remote chunk into
    parallel ranged GETs without a HEAD per piece; bytes must equal the local
    parallel-pread result for every partitioning."""
    local_dir = tmp_path / "d"
    local_dir.mkdir()
    for i in range(2):
        f = local_dir / f"part-{i}.libsvm"
        data.write_synthetic(str(f), i * 30000, (i + 1) * 30000, seed=5)
        w = io.Stream(f"s3://bk4/ds/part-{i}.libsvm", "w")
        w.write(f.read_bytes())
        w.close()
    for nparts in (1, 3):
        for part in range(nparts):
            h0 = s3.heads
            remote = _dmlc.read_partition("s3://bk4/ds", part, nparts, "text", 4, 12 << 20)
            h1 = s3.heads
            small = _dmlc.read_partition("s3://bk4/ds", part, nparts, "text", 4, 2 << 20)
            # HEADs come from split setup only: 6x more pieces, same count
            assert s3.heads - h1 == h1 - h0
            assert b"".join(small) == b"".join(remote)
            loc = _dmlc.read_partition(str(local_dir), part, nparts, "text", 4, 12 << 20)
            assert b"".join(remote) == b"".join(loc)
            assert all(c.endswith(b"\n") for c in remote)


def test_http_fault_is_retried(s3):
    """An injected transient GET failure (DMLC_FAULT_INJECT=http:1) goes
    through the ranged-read retry loop; the data still arrives intact."""
    payload = _blob(3 << 20, seed=7)
    w = io.Stream("s3://bk5/f.bin", "w")
    w.write(payload)
    w.close()
    _dmlc.fault_configure("http:1")
    try:
        assert _read_all("s3://bk5/f.bin", chunk=1 << 20) == payload
        assert _dmlc.fault_count("http") >= 2  # the failed pass + the retry
    finally:
        _dmlc.fault_configure("")


def test_s3_bad_signature_rejected(s3):
    os.environ["S3_SECRET_ACCESS_KEY"] = "wrong"
    try:
        with pytest.raises(Exception):
            io.Stream("s3://bk-wrong/x", "r")
    finally:
        os.environ["S3_SECRET_ACCESS_KEY"] = "secret"


def test_azure_roundtrip_blocks_and_listing(azure):
    big = _blob((64 << 20) + 1000, seed=1)  # > one 64 MiB block -> Put Block List
    w = io.Stream("azure://cont/big/blob.bin", "w")
    w.write(big)
    w.close()
    assert azure.store["cont/big/blob.bin"] == big
    assert _read_all("azure://cont/big/blob.bin", chunk=16 << 20) == big
    for i in range(4):
        w = io.Stream(f"azure://cont/txt/p{i}", "w")
        w.write(f"line{i}\n".encode())
        w.close()
    recs = [r.rstrip(b"\x00\n") for p in range(2) for r in io.iter_records("azure://cont/txt", p, 2, "text")]
    assert recs == [f"line{i}".encode() for i in range(4)]


def test_http_ranged_reads():
    srv = mock_remote.serve(mock_remote.PlainHandler)
    try:
        payload = _blob(3 << 20, seed=2)
        mock_remote.PlainHandler.store["/files/a.bin"] = payload
        url = f"http://127.0.0.1:{srv.server_address[1]}/files/a.bin"
        assert _read_all(url, chunk=1000) == payload
        mock_remote.PlainHandler.store["/files/t.txt"] = b"a\nbb\nccc\n"
        url = f"http://127.0.0.1:{srv.server_address[1]}/files/t.txt"
        assert [r.rstrip(b"\x00\n") for r in io.iter_records(url, 0, 1, "text")] == [b"a", b"bb", b"ccc"]
    finally:
        srv.shutdown()


def test_http_native_receive_and_libcurl_fallback():
    """Ranged GETs into caller memory are received natively (the body recv()ed
    straight into the destination, no libcurl buffer); a response the native
    path does not take (chunked transfer encoding) goes to libcurl and the
    bytes are the same."""
    srv = mock_remote.serve(mock_remote.PlainHandler)
    try:
        payload = _blob((3 << 20) + 777, seed=4)
        mock_remote.PlainHandler.store["/files/n.bin"] = payload
        url = f"http://127.0.0.1:{srv.server_address[1]}/files/n.bin"
        s0 = _dmlc.http_stats()
        assert _read_all(url, chunk=1 << 20) == payload
        s1 = _dmlc.http_stats()
        if os.environ.get("DMLC_HTTP_NATIVE", "1") != "0":
            assert s1["native_gets"] - s0["native_gets"] >= 4
        assert s1["native_fallbacks"] == s0["native_fallbacks"]
        mock_remote.PlainHandler.chunked = True
        assert _read_all(url, chunk=1 << 20) == payload
        s2 = _dmlc.http_stats()
        assert s2["native_gets"] == s1["native_gets"]
        if os.environ.get("DMLC_HTTP_NATIVE", "1") != "0":
            assert s2["native_fallbacks"] - s1["native_fallbacks"] >= 4
    finally:
        mock_remote.PlainHandler.chunked = False
        srv.shutdown()


@pytest.mark.skipif(os.environ.get("DMLC_HTTP_NATIVE", "1") == "0", reason="native path off")
def test_http_native_path_respects_proxy_env(monkeypatch):
    """A host libcurl would reach through http_proxy never takes the native
    receive (it only talks to origin servers); no_proxy brings it back.  The
    mock server is its own forward proxy, so the proxied reads still return
    the bytes."""
    srv = mock_remote.serve(mock_remote.PlainHandler)
    port = srv.server_address[1]
    try:
        payload = _blob((2 << 20) + 5, seed=6)
        mock_remote.PlainHandler.store["/files/p.bin"] = payload
        url = f"http://127.0.0.1:{port}/files/p.bin"
        monkeypatch.setenv("http_proxy", f"http://127.0.0.1:{port}")
        monkeypatch.delenv("no_proxy", raising=False)
        monkeypatch.delenv("NO_PROXY", raising=False)
        s0, p0 = _dmlc.http_stats(), mock_remote.PlainHandler.proxied
        assert _read_all(url, chunk=1 << 20) == payload
        s1 = _dmlc.http_stats()
        assert s1["native_gets"] == s0["native_gets"]
        assert mock_remote.PlainHandler.proxied - p0 >= 3
        for np_ in ("127.0.0.1", "localhost, 127.0.0.1:9", "*"):
            monkeypatch.setenv("no_proxy", np_)
            assert _read_all(url, chunk=1 << 20) == payload
            s2 = _dmlc.http_stats()
            assert s2["native_gets"] - s1["native_gets"] >= 3, np_
            s1 = s2
    finally:
        srv.shutdown()


def test_http_unreachable_host_falls_back_once():
    """A direct connect that fails marks the authority: the request goes to
    libcurl (which fails the same way here) and later requests skip the
    native connect."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()  # nothing listens on this port: connect is refused at once
    with pytest.raises(_dmlc.DMLCError):
        _read_all(f"http://127.0.0.1:{port}/x.bin", chunk=1 << 20)


def test_hdfs_fails_loudly_without_libhdfs():
    with pytest.raises(_dmlc.DMLCError, match="libhdfs"):
        io.Stream("hdfs://namenode:8020/x", "r")


@pytest.fixture()
def webhdfs():
    mock_remote.WebHdfsHandler.store = {}
    mock_remote.WebHdfsHandler.namenode_bodies = 0
    mock_remote.WebHdfsHandler.batch = True
    srv = mock_remote.serve(mock_remote.WebHdfsHandler)
    os.environ["HADOOP_USER_NAME"] = "dmlc"
    os.environ["DMLC_WEBHDFS_WRITE_BUFFER_MB"] = "1"
    yield mock_remote.WebHdfsHandler, f"127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()
    for k in ("HADOOP_USER_NAME", "DMLC_WEBHDFS_WRITE_BUFFER_MB", "DMLC_WEBHDFS_ENDPOINT",
              "DMLC_HDFS_BACKEND"):
        os.environ.pop(k, None)


def test_webhdfs_create_append_open_roundtrip(webhdfs):
    """Writes CREATE with the first 1 MiB block and APPEND the rest, each via
    the namenode's 307 to the datanode (no data ever sent to the namenode);
    reads are ranged OPENs, through both the direct and the read-ahead path."""
    h, addr = webhdfs
    payload = _blob((3 << 20) + 4321, seed=11)
    w = io.Stream(f"webhdfs://{addr}/user/dmlc/blob.bin", "w")
    for i in range(0, len(payload), 700_000):
        w.write(payload[i:i + 700_000])
    w.close()
    assert h.store["/user/dmlc/blob.bin"] == payload
    assert h.namenode_bodies == 0
    assert h.users == {"dmlc"}
    assert _read_all(f"webhdfs://{addr}/user/dmlc/blob.bin", chunk=16 << 20) == payload
    assert _read_all(f"webhdfs://{addr}/user/dmlc/blob.bin", chunk=5000) == payload
    # "a" mode appends to an existing file
    a = io.Stream(f"webhdfs://{addr}/user/dmlc/blob.bin", "a")
    a.write(b"tail")
    a.close()
    assert h.store["/user/dmlc/blob.bin"] == payload + b"tail"
    # an empty "w" stream still creates the file
    io.Stream(f"webhdfs://{addr}/user/dmlc/empty", "w").close()
    assert h.store["/user/dmlc/empty"] == b""


@pytest.mark.parametrize("batch", [True, False])
def test_webhdfs_listing_and_sharded_parser(webhdfs, tmp_path, batch):
    """A directory of 5 LibSVM parts (+ a subdirectory, not descended into) is
    listed in pages of 2 (LISTSTATUS_BATCH / startAfter) or, on an older
    namenode, with one LISTSTATUS; sharded parsing equals the local files."""
    h, addr = webhdfs
    h.batch = batch
    local = tmp_path / "d"
    local.mkdir()
    for i in range(5):
        f = local / f"part-{i}.libsvm"
        data.write_synthetic(str(f), i * 400, (i + 1) * 400, seed=21)
        h.store[f"/data/train/part-{i}.libsvm"] = f.read_bytes()
    h.store["/data/train/sub/x.libsvm"] = b"1 1:1\n"
    import pyref
    for nparts in (1, 3):
        for part in range(nparts):
            a = pyref.concat_blocks(list(data.iter_blocks(f"webhdfs://{addr}/data/train", part, nparts,
                                                          type="libsvm")))
            b = pyref.concat_blocks(list(data.iter_blocks(str(local), part, nparts, type="libsvm")))
            np.testing.assert_array_equal(a["index"], b["index"])
            np.testing.assert_array_equal(a["value"], b["value"])
            np.testing.assert_array_equal(a["offset"], b["offset"])


def test_hdfs_routes_to_webhdfs_without_libhdfs(webhdfs):
    h, addr = webhdfs
    h.store["/x/y.txt"] = b"a\nbb\nccc\n"
    os.environ["DMLC_WEBHDFS_ENDPOINT"] = f"http://{addr}"
    # a namenode address not seen before, so a fresh hdfs:// instance is made
    recs = [r.rstrip(b"\x00\n") for r in io.iter_records("hdfs://nn-web:8020/x/y.txt", 0, 1, "text")]
    assert recs == [b"a", b"bb", b"ccc"]


def test_webhdfs_missing_file_reports_remote_exception(webhdfs):
    _, addr = webhdfs
    with pytest.raises(_dmlc.DMLCError, match="FileNotFoundException"):
        io.Stream(f"webhdfs://{addr}/nope", "r")


def test_hdfs_through_libhdfs_abi(tmp_path):
    """hdfs:// over the dlopen'ed libhdfs C API, using a stand-in libhdfs.so
    (tests/fake_libhdfs.c: the hdfs.h functions over a local directory, short
    reads and one EINTR): write (short writes looped), append, read back,
    GetPathInfo sizes, and a sharded parse of a directory equal to local."""
    import subprocess
    import sys
    lib = tmp_path / "hadoop" / "lib" / "native"
    lib.mkdir(parents=True)
    src = os.path.join(os.path.dirname(__file__), "fake_libhdfs.c")
    subprocess.check_call(["gcc", "-O1", "-shared", "-fPIC", "-o", str(lib / "libhdfs.so"), src])
    root = tmp_path / "root"
    (root / "data").mkdir(parents=True)
    for i in range(3):
        data.write_synthetic(str(root / "data" / f"part-{i}.libsvm"), i * 500, (i + 1) * 500, seed=4)
    code = f"""
import numpy as np, pyref
from dmlc_core_amd import data, io
blob = bytes(range(256)) * 40
w = io.Stream("hdfs://nn:8020/out/blob.bin", "w"); w.write(blob); w.close()
a = io.Stream("hdfs://nn:8020/out/blob.bin", "a"); a.write(b"tail"); a.close()
s = io.Stream("hdfs://nn:8020/out/blob.bin", "r")
got = b""
while True:
    b = s.read(3000)
    if not b:
        break
    got += b
assert got == blob + b"tail", len(got)
for nparts in (1, 2):
    for part in range(nparts):
        x = pyref.concat_blocks(list(data.iter_blocks("hdfs://nn:8020/data", part, nparts, type="libsvm")))
        y = pyref.concat_blocks(list(data.iter_blocks({str(root / 'data')!r}, part, nparts, type="libsvm")))
        for k in ("offset", "index", "value", "label"):
            np.testing.assert_array_equal(x[k], y[k])
print("ok")
"""
    env = dict(os.environ, HADOOP_HOME=str(tmp_path / "hadoop"), FAKE_HDFS_ROOT=str(root),
               PYTHONPATH=os.pathsep.join([os.path.dirname(__file__),
                                           os.path.dirname(os.path.dirname(__file__))]))
    env.pop("DMLC_WEBHDFS_ENDPOINT", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]
    assert (root / "out" / "blob.bin").read_bytes() == bytes(range(256)) * 40 + b"tail"


_HTTPS_CLIENT = r'''
import json, os, sys
sys.path.insert(0, os.environ["TESTS_DIR"])
import numpy as np
import mock_remote
from dmlc_core_amd import _dmlc, io

crt, key = sys.argv[1], sys.argv[2]

def read_all(uri, chunk=1 << 20):
    s = io.Stream(uri, "r")
    out = bytearray()
    while True:
        b = s.read(chunk)
        if not b:
            return bytes(out)
        out += b

res = {}
payload = np.random.default_rng(11).integers(0, 256, (3 << 20) + 333, dtype=np.uint8).tobytes()
srv = mock_remote.serve_tls(mock_remote.PlainHandler, crt, key)
mock_remote.PlainHandler.store["/files/t.bin"] = payload
s0 = _dmlc.http_stats()
res["https_equal"] = read_all(f"https://127.0.0.1:{srv.server_address[1]}/files/t.bin") == payload
s1 = _dmlc.http_stats()
res["https_native"] = s1["native_gets"] - s0["native_gets"]
res["https_fallbacks"] = s1["native_fallbacks"] - s0["native_fallbacks"]
s3 = mock_remote.serve_tls(mock_remote.S3Handler, crt, key)
os.environ.update({"S3_ENDPOINT": f"https://127.0.0.1:{s3.server_address[1]}",
                   "S3_ACCESS_KEY_ID": "AKIDTEST", "S3_SECRET_ACCESS_KEY": "secret",
                   "S3_REGION": "us-east-1", "S3_VERIFY_SSL": "0"})
w = io.Stream("s3://tls/obj.bin", "w")
w.write(payload)
w.close()
s2 = _dmlc.http_stats()
res["s3_equal"] = read_all("s3://tls/obj.bin") == payload
s3s = _dmlc.http_stats()
res["s3_native"] = s3s["native_gets"] - s2["native_gets"]
res["s3_fallbacks"] = s3s["native_fallbacks"] - s2["native_fallbacks"]
print(json.dumps(res))
'''


@pytest.mark.skipif(os.environ.get("DMLC_HTTP_NATIVE", "1") == "0", reason="native path off")
def test_https_native_receive_into_caller_memory(tmp_path):
    """https GETs take the native receive too (OpenSSL 3 by dlopen, SSL_read
    into the destination): with verification against the trust store that
    CURL_CA_BUNDLE / SSL_CERT_FILE name (the test's self-signed certificate,
    for libcurl's HEAD and the native GETs alike) and with
    S3_VERIFY_SSL=0; the bytes equal what was served or written.  A fresh
    process: the trust store is read once per process."""
    import shutil
    import subprocess
    import sys
    if shutil.which("openssl") is None:
        pytest.skip("no openssl CLI to make a test certificate")
    crt, key = str(tmp_path / "c.pem"), str(tmp_path / "k.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-keyout", key,
                    "-out", crt, "-days", "2", "-subj", "/CN=127.0.0.1",
                    "-addext", "subjectAltName=IP:127.0.0.1"], check=True, capture_output=True)
    env = dict(os.environ, SSL_CERT_FILE=crt, CURL_CA_BUNDLE=crt, TESTS_DIR=os.path.dirname(__file__))
    for k in ("http_proxy", "https_proxy", "HTTPS_PROXY", "all_proxy", "ALL_PROXY"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, "-c", _HTTPS_CLIENT, crt, key], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    import json
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["https_equal"] and r["s3_equal"], r
    assert r["https_native"] >= 3 and r["https_fallbacks"] == 0, r
    assert r["s3_native"] >= 3 and r["s3_fallbacks"] == 0, r
