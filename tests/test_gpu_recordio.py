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
