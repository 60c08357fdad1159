"""K7 GPU RecordIO decode vs the CPU RecordIOReader (bit-identical payloads,
same order): injected aligned/unaligned magic words, multi-part records,
empty records, sharding into 1..7 parts, tiny chunks, zero-copy on/off."""
import os
import random

import numpy as np
import pytest

from dmlc_core_amd import io

pytestmark = pytest.mark.gpu

MAGIC = (0xCED7230A).to_bytes(4, "little")


def _records(n, seed, max_len=700):
    rng = random.Random(seed)
    recs = []
    for i in range(n):
        ln = rng.choice([0, 1, 3, 4, 5, 8, rng.randint(0, max_len)])
        b = bytearray(rng.getrandbits(8) for _ in range(ln))
        # aligned magic words force multi-part records; unaligned ones must survive
        for k in range(0, ln - 3, 4):
            if rng.random() < 0.03:
                b[k:k + 4] = MAGIC
        if ln > 9 and rng.random() < 0.1:
            b[5:9] = MAGIC
        recs.append(bytes(b))
    return recs


def _write(path, recs):
    w = io.RecordIOWriter(str(path))
    for r in recs:
        w.write(r)
    exc = w.except_counter()
    w.close()
    return exc


def _cpu(path, part, nparts):
    return list(io.iter_records(str(path), part, nparts, "recordio"))


@pytest.mark.parametrize("zero_copy", [0, 1])
@pytest.mark.parametrize("chunk_kb", [4, 64, 1024])
def test_gpu_recordio_equals_cpu(tmp_path, zero_copy, chunk_kb):
    p = tmp_path / "a.rec"
    recs = _records(3000, 1)
    assert _write(p, recs) > 0  # some records were split into parts
    for nparts in (1, 3, 7):
        got = []
        for part in range(nparts):
            r = io.GPURecordIO(str(p), part, nparts, chunk_bytes=chunk_kb * 1024,
                               zero_copy=zero_copy)
            r.read_all()
            off, data = r.resident_to_host()
            mine = io.split_records(off, data)
            assert mine == _cpu(p, part, nparts)
            got += mine
            assert r.stats()["zero_copy"] == bool(zero_copy)
        assert got == recs


def test_gpu_recordio_streaming_and_torch(tmp_path):
    p = tmp_path / "s.rec"
    recs = _records(2000, 2, max_len=300)
    _write(p, recs)
    r = io.GPURecordIO(str(p), chunk_bytes=16 * 1024)
    for _ in range(2):
        got = []
        for off, data in r.iter_host():
            got += io.split_records(off, data)
        assert got == recs
        r.before_first()
    batch = r.read_all()
    t = io.GPURecordIO.to_torch(batch)
    assert t["data"].device.type == "cuda" and t["size"] == len(recs)
    off = t["offset"].cpu().numpy().astype(np.int64)
    assert off[-1] == sum(len(x) for x in recs)
    assert bytes(t["data"].cpu().numpy()[off[5]:off[6]].tobytes()) == recs[5]


def test_gpu_recordio_multi_file(tmp_path):
    d = tmp_path / "parts"
    d.mkdir()
    allrecs = []
    for i in range(3):
        recs = _records(500, 10 + i)
        _write(d / f"p{i}.rec", recs)
        allrecs += recs
    for nparts in (1, 2, 5):
        got = []
        for part in range(nparts):
            r = io.GPURecordIO(str(d), part, nparts, chunk_bytes=8192)
            r.read_all()
            got += io.split_records(*r.resident_to_host())
        assert got == allrecs


def _write_indexed(path, idx, recs):
    w = io.RecordIOWriter(str(path))
    with open(idx, "w") as f:
        for k, r in enumerate(recs):
            f.write(f"{k}\t{w.tell()}\n")
            w.write(r)
    w.close()


def _cpu_indexed_epochs(path, idx, part, nparts, shuffle, seed, epochs):
    s = io.InputSplit(str(path), part, nparts, "indexed_recordio", index_uri=str(idx),
                      shuffle=shuffle, seed=seed, batch_size=7)
    out = []
    for e in range(epochs):
        if e:
            s.before_first()
        ep = []
        while True:
            r = s.next_record()
            if r is None:
                break
            ep.append(r)
        out.append(ep)
    return out


@pytest.mark.parametrize("shuffle", [False, True])
def test_gpu_indexed_recordio_epoch_order_matches_cpu(tmp_path, shuffle):
    """Shuffled epochs on the GPU (shard resident in HBM, batches gathered on
    the device) visit records in exactly the CPU IndexedRecordIOSplitter's
    mt19937(111 + seed) order, epoch after epoch."""
    p, idx = tmp_path / "i.rec", tmp_path / "i.idx"
    recs = _records(1500, 5, max_len=400)
    _write_indexed(p, idx, recs)
    for nparts in (1, 3):
        for part in range(nparts):
            cpu = _cpu_indexed_epochs(p, idx, part, nparts, shuffle, 7, 3)
            r = io.GPURecordIO(str(p), part, nparts, index=str(idx), shuffle=int(shuffle), seed=7,
                               chunk_bytes=32 * 1024)
            for e in range(3):
                if e:
                    r.before_first()
                r.read_all()
                got = io.split_records(*r.resident_to_host())
                assert got == cpu[e], (part, e)
            if shuffle and len(cpu[0]) > 2:
                assert cpu[0] != cpu[1]  # a new order every epoch
            # streaming batches follow the same order
            r.before_first()
            streamed = []
            for off, data in r.iter_host():
                streamed += io.split_records(off, data)
            assert streamed == cpu_next_epoch(p, idx, part, nparts, shuffle, 7, 4)


def cpu_next_epoch(p, idx, part, nparts, shuffle, seed, epoch_count):
    return _cpu_indexed_epochs(p, idx, part, nparts, shuffle, seed, epoch_count)[-1]


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_gpu_recordio_hbm_cache_replay(tmp_path, zero_copy):
    """hbm_cache: the first epoch leaves the shard resident; later epochs decode
    from HBM (merged chunks) and equal the CPU reader."""
    p = tmp_path / "h.rec"
    recs = _records(2500, 9)
    _write(p, recs)
    r = io.GPURecordIO(str(p), 0, 1, chunk_bytes=16 * 1024, hbm_cache=1, zero_copy=zero_copy,
                       device_slots=4)
    # a streaming first epoch fills the cache; its batch sizes are the contract
    first = [len(data) for _, data in r.iter_host()]
    for e in range(3):
        r.before_first()
        r.read_all()
        assert io.split_records(*r.resident_to_host()) == recs, e
    assert r.stats()["replayed_chunks"] > 0

    # streaming from the cache too, with the first epoch's batch sizes (the
    # resident read_all merges cached chunks; Next() must not)
    r.before_first()
    got, sizes = [], []
    for off, data in r.iter_host():
        sizes.append(len(data))
        got += io.split_records(off, data)
    assert got == recs
    assert sizes == first


@pytest.mark.parametrize("replay_mb", [0.03, 0.1])
def test_gpu_recordio_replay_prelaunched_counts(tmp_path, replay_mb):
    """read_all over the HBM cache runs the next piece's count + scan on a
    second stream beside the current fill: many small merged pieces, epochs
    with a streaming pass in between, every epoch equal to the CPU reader."""
    p = tmp_path / "q.rec"
    recs = _records(3000, 11)
    _write(p, recs)
    r = io.GPURecordIO(str(p), 0, 1, chunk_bytes=16 * 1024, hbm_cache=1, device_slots=3,
                       replay_chunk_mb=replay_mb)
    for e in range(4):
        if e:
            r.before_first()
        r.read_all()
        assert io.split_records(*r.resident_to_host()) == recs, e
        if e == 1:
            r.before_first()
            assert next(r.iter_host(), None) is not None  # a partial streaming pass
    assert r.stats()["replayed_chunks"] > 4


def test_gpu_recordio_rejects_corrupt_chain(tmp_path):
    p = tmp_path / "c.rec"
    recs = [b"x" * 40, bytes(MAGIC) * 3 + b"tail!", b"y" * 12]
    _write(p, recs)
    raw = bytearray(open(p, "rb").read())
    # flip the cflag of the first continuation part to "whole record"
    pos = raw.find(MAGIC, 48)
    while pos >= 0 and ((int.from_bytes(raw[pos + 4:pos + 8], "little") >> 29) not in (2, 3)):
        pos = raw.find(MAGIC, pos + 4)
    assert pos > 0
    lrec = int.from_bytes(raw[pos + 4:pos + 8], "little") & ((1 << 29) - 1)
    raw[pos + 4:pos + 8] = lrec.to_bytes(4, "little")
    open(p, "wb").write(bytes(raw))
    r = io.GPURecordIO(str(p), zero_copy=0)
    with pytest.raises(Exception, match="malformed record"):
        r.read_all()


def test_gpu_recordio_one_pass_overflow_rerun(tmp_path):
    """one_pass=1 after a streamed first epoch: the first read_all finds no
    resident output yet, its piece overflows, grows the output and runs again"""
    p = tmp_path / "v.rec"
    recs = _records(2500, 17)
    _write(p, recs)
    r = io.GPURecordIO(str(p), 0, 1, chunk_bytes=16 * 1024, hbm_cache=1, one_pass=1)
    assert sum(1 for _ in r.iter_host()) > 1  # epoch 1 streams, fills the cache
    for _ in range(2):
        r.before_first()
        r.read_all()
        assert io.split_records(*r.resident_to_host()) == recs
    assert r.stats()["one_pass_chunks"] > 0 and r.stats()["one_pass_reruns"] >= 1


@pytest.mark.parametrize("replay_mb", [0.05, 1])
def test_gpu_recordio_one_pass_replay(tmp_path, replay_mb):
    """read_all over the HBM cache decodes each merged piece in one launch
    (R1 inside the fill, look-back, payload copied from the LDS-staged tile):
    multi-part records, escaped magic words, empty and tiny records, records
    straddling tiles -- every epoch equals the CPU reader and the counted
    path (one_pass=0)"""
    p = tmp_path / "o.rec"
    recs = _records(4000, 13, max_len=3000)
    _write(p, recs)
    outs = {}
    for one in (1, 0):
        r = io.GPURecordIO(str(p), 0, 1, chunk_bytes=16 * 1024, hbm_cache=1,
                           replay_chunk_mb=replay_mb, one_pass=one)
        for e in range(3):
            if e:
                r.before_first()
            r.read_all()
            got = io.split_records(*r.resident_to_host())
            assert got == recs, (one, e)
        outs[one] = r.stats()
    assert outs[1]["one_pass_chunks"] > 0 and outs[0]["one_pass_chunks"] == 0


@pytest.mark.parametrize("max_len", [700, 20000])
@pytest.mark.parametrize("chunk_kb", [4, 64, 1024])
def test_gpu_recordio_chain_count_equals_cpu(tmp_path, max_len, chunk_kb):
    """R1c (counts from part headers alone, chain_count=1) decodes every
    shard exactly like the CPU reader: multi-part records, escaped magic
    words, empty / tiny records, records longer than a tile (tiles without a
    header)."""
    p = tmp_path / "h.rec"
    recs = _records(1500, 19, max_len=max_len)
    _write(p, recs)
    for nparts in (1, 3):
        got = []
        for part in range(nparts):
            r = io.GPURecordIO(str(p), part, nparts, chunk_bytes=chunk_kb * 1024, chain_count=1)
            r.read_all()
            mine = io.split_records(*r.resident_to_host())
            assert mine == _cpu(p, part, nparts)
            assert r.stats()["chain_counts"] > 0
            got += mine
        assert got == recs


def test_gpu_recordio_chain_count_multi_tile_lanes(tmp_path):
    """R1c with several consecutive tiles per lane (the layout of large
    pieces; forced here by DMLC_REC_CHAIN_TILES=3 in a subprocess, since the
    setting is read once): the chain runs on across a lane's tiles, the
    counts binned per tile equal R1's -- every shard equals the CPU reader."""
    import json
    import subprocess
    import sys
    p = tmp_path / "m.rec"
    recs = _records(2500, 23, max_len=9000)
    _write(p, recs)
    code = (
        "import json, sys\n"
        "from dmlc_core_amd import io\n"
        "out = []\n"
        "for part in range(2):\n"
        "    r = io.GPURecordIO(sys.argv[1], part, 2, chunk_bytes=256 * 1024, chain_count=1)\n"
        "    r.read_all()\n"
        "    out.append([x.hex() for x in io.split_records(*r.resident_to_host())])\n"
        "    assert r.stats()['chain_counts'] > 0\n"
        "print(json.dumps(out))\n")
    env = dict(os.environ, DMLC_REC_CHAIN_TILES="3")
    res = subprocess.run([sys.executable, "-c", code, str(p)], capture_output=True, text=True,
                         env=env, timeout=120)
    assert res.returncode == 0, res.stderr[-3000:]
    got = json.loads(res.stdout.strip().splitlines()[-1])
    for part in range(2):
        assert [bytes.fromhex(x) for x in got[part]] == _cpu(p, part, 2)


def test_gpu_recordio_chain_count_auto_on_replay(tmp_path):
    """chain_count auto: the first chunk uses R1, later ones (records of
    >= 128 B on average) R1c, including the prelaunched replay counts"""
    p = tmp_path / "a.rec"
    rng = random.Random(3)
    recs = [bytes(rng.getrandbits(8) for _ in range(rng.randint(200, 900))) for _ in range(3000)]
    _write(p, recs)
    r = io.GPURecordIO(str(p), 0, 1, chunk_bytes=64 * 1024, hbm_cache=1, replay_chunk_mb=0.2)
    for e in range(3):
        if e:
            r.before_first()
        r.read_all()
        assert io.split_records(*r.resident_to_host()) == recs, e
    assert r.stats()["chain_counts"] > 0


def test_gpu_recordio_chain_count_rejects_unescaped_header(tmp_path):
    """A payload holding an unescaped part header that ends exactly where the
    payload ends (a writer that skipped the escaping): the chain count and
    the fill see different headers, and the tile check turns that into an
    error instead of a silently different record list."""
    p = tmp_path / "u.rec"
    recs = [b"a" * 24, b"x" * 64, b"b" * 20]
    _write(p, recs)
    raw = bytearray(open(p, "rb").read())
    pos = raw.find(b"x" * 64)
    assert pos > 0 and pos % 4 == 0
    raw[pos:pos + 4] = MAGIC
    raw[pos + 4:pos + 8] = (56).to_bytes(4, "little")  # a whole record of 56 bytes
    open(p, "wb").write(bytes(raw))
    r = io.GPURecordIO(str(p), zero_copy=0, chain_count=1)
    with pytest.raises(Exception, match="malformed record"):
        r.read_all()
