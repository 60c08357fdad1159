"""Mid-epoch resume: the host reader's cursor is a record
boundary in partition-byte space; a new reader seeked to it continues with
exactly the remaining bytes, across file boundaries and shards."""
import pytest

from dmlc_core_amd import data, io


@pytest.fixture
def ds(tmp_path):
    d = tmp_path / "ds"
    d.mkdir()
    for i in range(3):
        data.write_synthetic(str(d / f"p{i}.libsvm"), i * 4000, (i + 1) * 4000, seed=2)
    # one file without a trailing newline: the reader inserts a separator
    (d / "p3.libsvm").write_bytes(b"1 3:1.5 7:2\n0 2:1")
    return str(d)


def _all(r):
    out = []
    while True:
        c = r.next()
        if c is None:
            return out
        out.append(c)


@pytest.mark.parametrize("nparts", [1, 3])
def test_partition_reader_seek_resumes_exactly(ds, nparts):
    for part in range(nparts):
        full = _all(io.PartitionReader(ds, part, nparts, "text", 2, 256 << 10))
        assert b"".join(full) == b"".join(io.read_partition(ds, part, nparts, "text", 2, 256 << 10))
        for k in range(len(full) + 1):
            r = io.PartitionReader(ds, part, nparts, "text", 2, 256 << 10)
            head = [r.next() for _ in range(k)]
            cur = r.tell()
            r2 = io.PartitionReader(ds, part, nparts, "text", 2, 100 << 10)  # other chunking
            r2.seek(cur)
            rest = _all(r2)
            assert b"".join(head) + b"".join(rest) == b"".join(full), (part, k)
        assert r.tell() == r.partition_bytes() or k < len(full)


def test_cursor_is_record_boundary(ds):
    r = io.PartitionReader(ds, 0, 1, "text", 2, 64 << 10)
    r.next()
    cur = r.tell()
    r2 = io.PartitionReader(ds, 0, 1, "text", 2, 64 << 10)
    r2.seek(cur)
    first = r2.next()
    assert first[:1] in (b"0", b"1")  # starts with a label, i.e. a whole line
