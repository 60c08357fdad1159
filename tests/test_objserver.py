"""tools/dmlc_objserver (the sendfile loopback S3 / HTTP server used for the
config-4 throughput runs) against the native S3 and HTTP readers: listing with
pagination and prefixes, HEAD sizes, ranged GETs, sharded text splits."""
import os
import subprocess

import pytest

from dmlc_core_amd import io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "dmlc_objserver")

pytestmark = pytest.mark.skipif(not os.path.exists("/usr/lib/x86_64-linux-gnu/libcurl.so.4"),
                                reason="libcurl not installed")


@pytest.fixture(scope="module")
def server(tmp_path_factory):
    if not os.path.exists(BIN):
        subprocess.run(["make", "-C", ROOT, "build/dmlc_objserver"], check=True,
                       stdout=subprocess.DEVNULL)
    root = tmp_path_factory.mktemp("objroot")
    bk = root / "bk"
    (bk / "many").mkdir(parents=True)
    for i in range(1003):  # > one ListObjectsV2 page
        (bk / "many" / f"f{i:05d}.txt").write_text(f"{i}\n")
    (bk / "text").mkdir()
    lines = [f"line {i} " + "x" * (i % 97) for i in range(20000)]
    for k in range(3):
        (bk / "text" / f"part-{k}.txt").write_text("\n".join(lines[k::3]) + "\n")
    proc = subprocess.Popen([BIN, "--root", str(root)], stdout=subprocess.PIPE, text=True)
    port = int(proc.stdout.readline().split()[1])
    env = {"S3_ENDPOINT": f"http://127.0.0.1:{port}", "S3_ACCESS_KEY_ID": "x",
           "S3_SECRET_ACCESS_KEY": "y", "S3_REGION": "us-east-1"}
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    yield port, root, lines
    proc.kill()
    proc.wait()
    for k, v in old.items():
        if v is None:
            os.environ.pop(k, None)
        else:
            os.environ[k] = v


def test_listing_paginates_and_sizes(server):
    _port, _root, _ = server
    recs = list(io.iter_records("s3://bk/many/", 0, 1, "text"))
    # text records keep their line end ('\0' in place of the last EOL byte, as
    # the reference LineSplitter does)
    assert sorted(int(r.rstrip(b"\0\r\n")) for r in recs) == list(range(1003))


@pytest.mark.parametrize("nparts", [1, 4])
def test_sharded_text_split_over_s3_and_http(server, nparts):
    port, root, lines = server
    want = sorted(lines)
    got = []
    for p in range(nparts):
        got += [r.rstrip(b"\0\r\n").decode()
                for r in io.iter_records("s3://bk/text/", p, nparts, "text")]
    assert sorted(got) == want
    one = [r.rstrip(b"\0\r\n").decode()
           for r in io.iter_records(f"http://127.0.0.1:{port}/bk/text/part-1.txt", 0, 1, "text")]
    assert one == lines[1::3]


def test_ranged_reads_match_file(server):
    _port, root, _ = server
    s = io.Stream("s3://bk/text/part-2.txt", "r")
    data = s.read(1 << 30)
    assert data == (root / "bk" / "text" / "part-2.txt").read_bytes()


def test_range_edge_cases(server):
    """suffix ranges return the last N bytes (as S3); a reversed range is 416"""
    import http.client
    port, root, _ = server
    body = (root / "bk" / "text" / "part-1.txt").read_bytes()

    def get(rng):
        c = http.client.HTTPConnection("127.0.0.1", port, timeout=10)
        c.request("GET", "/bk/text/part-1.txt", headers={"Range": rng})
        r = c.getresponse()
        out = (r.status, r.getheader("Content-Length"), r.read())
        c.close()
        return out

    st, ln, data = get("bytes=-500")
    assert st == 206 and data == body[-500:] and int(ln) == 500
    st, _, data = get("bytes=-%d" % (len(body) + 10))
    assert st == 206 and data == body
    st, _, data = get("bytes=10-19")
    assert st == 206 and data == body[10:20]
    st, _, _ = get("bytes=100-50")
    assert st == 416
