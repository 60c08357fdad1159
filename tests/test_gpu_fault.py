"""Fault injection through the GPU pipeline: a failing reader fill (pinned
ring, reader thread), H2D copy, or chunk parse surfaces as dmlc::Error in
Python; the parser tears down cleanly (streams drained, slots recycled) and a
fresh parser over the same data is bit-exact with the CPU parser."""
import numpy as np
import pytest

import pyref
from dmlc_core_amd import _dmlc, data, io

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def disarm():
    yield
    _dmlc.fault_configure("")


def _cpu(p):
    return pyref.concat_blocks(list(data.iter_blocks(p, 0, 1, type="libsvm")))


@pytest.mark.parametrize("point,zero_copy", [("read", 0), ("read", 1), ("h2d", 0), ("h2d", 1),
                                             ("parse", 0)])
def test_gpu_parser_fault_then_recovery(tmp_path, point, zero_copy):
    p = str(tmp_path / "f.libsvm")
    data.write_synthetic(p, 0, 30000, seed=5)
    _dmlc.fault_configure(f"{point}:3")
    g = data.GPUParser(p, chunk_bytes=1 << 20, zero_copy=zero_copy, read_threads=2)
    with pytest.raises(_dmlc.DMLCError, match=f'injected fault at "{point}"'):
        g.parse_all()
    del g
    _dmlc.fault_configure("")
    h = data.GPUParser(p, chunk_bytes=1 << 20, zero_copy=zero_copy).parse_all().to_host()
    c = _cpu(p)
    for k in ("label", "offset", "index", "value"):
        np.testing.assert_array_equal(h[k], c[k], err_msg=k)


def test_gpu_recordio_fault(tmp_path):
    f = str(tmp_path / "r.rec")
    data.write_synthetic(f, 0, 20000, format="recordio", seed=3, record_bytes=256)
    _dmlc.fault_configure("recordio:2")
    r = io.GPURecordIO(f, chunk_bytes=1 << 20)
    with pytest.raises(_dmlc.DMLCError, match='injected fault at "recordio"'):
        r.read_all()
    del r
    _dmlc.fault_configure("")
    r = io.GPURecordIO(f, chunk_bytes=1 << 20)
    assert r.read_all()["size"] == 20000


@pytest.mark.parametrize("zero_copy", [0, 1])
def test_gpu_parse_failure_keeps_resume_cursor(tmp_path, zero_copy):
    """A chunk that fails mid-parse is not delivered: tell() still points at
    its start, so seeking there on the same parser replays it exactly."""
    p = str(tmp_path / "c.libsvm")
    data.write_synthetic(p, 0, 30000, seed=6)
    g = data.GPUParser(p, chunk_bytes=1 << 20, zero_copy=zero_copy, read_threads=2)
    blocks = []
    assert g.next()
    blocks.append(g.value_to_host())
    before = g.tell()
    _dmlc.fault_configure("parse_fill:1")
    with pytest.raises(_dmlc.DMLCError, match='injected fault at "parse_fill"'):
        g.next()
    _dmlc.fault_configure("")
    assert g.tell() == before
    g.seek(before)
    while g.next():
        blocks.append(g.value_to_host())
    got = pyref.concat_blocks(blocks)
    c = _cpu(p)
    for k in ("label", "offset", "index", "value"):
        np.testing.assert_array_equal(got[k], c[k], err_msg=k)
