"""Python-level coverage of reference InputSplit behaviours (the exact orders
are pinned against std::mt19937 oracles in tests/cpp/unittest_split_behaviors.cc):

* ``stdin`` as a URI reads a single unsplittable stream (reference
  src/io.cc:95-97 -> SingleFileSplit, src/io/single_file_split.h);
* ``num_shuffle_parts`` (InputSplitShuffle): every epoch visits each record of
  the shard exactly once, in an order that changes between epochs and is
  reproducible for a fixed seed;
* ``uri#cache``: the cache file is written during the first pass and replayed.
"""
import os

import subprocess
import sys

import numpy as np

from dmlc_core_amd import io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _records(split):
    out = []
    while True:
        r = split.next_record()
        if r is None:
            return out
        out.append(r.rstrip(b"\r\n\0"))


def test_stdin_single_file_split():
    lines = [f"row {i} {'z' * (i % 17)}" for i in range(5000)]
    code = ("import sys; sys.path.insert(0, %r)\n"
            "from dmlc_core_amd import io\n"
            "s = io.InputSplit('stdin', 0, 1, 'text')\n"
            "n = 0\n"
            "while True:\n"
            "    r = s.next_record()\n"
            "    if r is None: break\n"
            "    sys.stdout.buffer.write(r.rstrip(b'\\r\\n\\0') + b'\\n'); n += 1\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], input=("\n".join(lines) + "\n").encode(),
                       capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr.decode()[-2000:]
    assert p.stdout.decode().splitlines() == lines


def test_shuffle_parts_cover_shard_and_reorder(tmp_path):
    path = str(tmp_path / "l.txt")
    lines = [f"line-{i}".encode() for i in range(4000)]
    with open(path, "wb") as f:
        f.write(b"\n".join(lines) + b"\n")
    for nparts in (1, 2):
        union = []
        for part in range(nparts):
            plain = _records(io.InputSplit(path, part, nparts, "text"))
            s = io.InputSplit(path, part, nparts, "text", num_shuffle_parts=6, seed=9)
            e0 = _records(s)
            s.before_first()
            e1 = _records(s)
            assert sorted(e0) == sorted(plain) == sorted(e1)
            assert e0 != plain or e1 != plain  # sub-shards visited out of order
            again = _records(io.InputSplit(path, part, nparts, "text", num_shuffle_parts=6, seed=9))
            assert again == e0  # same seed -> same order
            union += e0
        assert sorted(union) == sorted(lines)


def test_cache_file_written_and_replayed(tmp_path):
    path = str(tmp_path / "c.txt")
    with open(path, "w") as f:
        f.write("".join(f"{i} {i * i}\n" for i in range(3000)))
    cache = str(tmp_path / "c.cache")
    s = io.InputSplit(path + "#" + cache, 0, 1, "text")
    e0 = _records(s)
    s.before_first()
    e1 = _records(s)
    assert e0 == e1 == _records(io.InputSplit(path, 0, 1, "text"))
    assert os.path.getsize(cache) > os.path.getsize(path)


def test_partition_reader_grows_for_a_record_longer_than_its_buffer(tmp_path):
    """io.PartitionReader (the pinned-ring ShardReader) grows its buffer for a
    line longer than chunk_bytes instead of failing; every byte arrives once."""
    path = str(tmp_path / "g.txt")
    lines = [b"short %d" % i for i in range(300)]
    lines.insert(150, b"x" * (5 * 4096 + 7))
    with open(path, "wb") as f:
        f.write(b"\n".join(lines) + b"\n")
    r = io.PartitionReader(path, 0, 1, "text", nthread=2, chunk_bytes=4096)
    chunks = []
    while True:
        c = r.next()
        if c is None:
            break
        chunks.append(c)
    assert b"".join(chunks).split(b"\n")[:-1] == lines
    assert max(len(c) for c in chunks) > 4096


def test_shuffle_parts_order_matches_input_split_shuffle(tmp_path):
    """_dmlc.shuffle_parts_order (used by the GPU ShuffledGPUParser) is the
    visiting order of InputSplitShuffle: the split's records in epochs 0 and 1
    are the sub-shards' records concatenated in that order."""
    from dmlc_core_amd import _dmlc, io
    d = tmp_path / "sh"
    d.mkdir()
    for i in range(3):
        (d / f"p{i}.txt").write_text("".join(f"{i}-{k}\n" for k in range(400)))
    uri = str(d)
    for part, nparts, k, seed in ((0, 1, 4, 3), (1, 2, 3, 0)):
        split = io.InputSplit(uri, part, nparts, "text", num_shuffle_parts=k, seed=seed)
        for epoch in range(2):
            if epoch:
                split.before_first()
            got = []
            while True:
                r = split.next_record()
                if r is None:
                    break
                got.append(r.rstrip(b"\0\r\n"))
            order = _dmlc.shuffle_parts_order(part, nparts, k, seed, epoch)
            assert sorted(order) == list(range(k))
            want = []
            for sub in order:
                want += [r.rstrip(b"\0\r\n") for r in io.iter_records(uri, part * k + sub, nparts * k)]
            assert got == want, (part, epoch, order)


def test_recordio_mapped_chunks_multi_file_multi_part_two_epochs(tmp_path, monkeypatch):
    """With DMLC_SPLIT_MMAP=1, RecordIO splits over local files read chunks
    as views of a file mapping (no copy out of the page cache).  Records that contain the magic
    word (multi-part, compacted in place on extraction), several files, and a
    second epoch (the copy-on-write mapping is dropped at BeforeFirst) give
    the records written -- the same as the buffered (default) path."""
    import struct
    from dmlc_core_amd import io
    magic = struct.pack("<I", 0xCED7230A)
    rng = np.random.default_rng(3)
    recs = []
    for f in range(3):
        w = io.RecordIOWriter(str(tmp_path / f"r{f}.rec"))
        for i in range(700):
            n = int(rng.integers(0, 3000))
            body = bytearray(rng.integers(0, 256, size=n, dtype=np.uint8).tobytes())
            if i % 7 == 0 and n >= 8:
                body[(n // 2) & ~3:((n // 2) & ~3) + 4] = magic  # a multi-part record
            w.write(bytes(body))
            recs.append(bytes(body))
        w.close()
    uri = str(tmp_path / r"r\d\.rec")
    monkeypatch.setenv("DMLC_SPLIT_MMAP", "1")
    got = []
    for part in range(3):
        s = io.InputSplit(uri, part, 3, "recordio")
        for epoch in range(2):
            out = []
            while True:
                r = s.next_record()
                if r is None:
                    break
                out.append(bytes(r))
            if epoch == 0:
                got += out
                first = out
            else:
                assert out == first
            s.before_first()
    assert got == recs
    monkeypatch.setenv("DMLC_SPLIT_MMAP", "0")
    buffered = [bytes(r) for p in range(3) for r in io.iter_records(uri, p, 3, "recordio")]
    assert buffered == recs
