"""Deterministic fault injection (DMLC_FAULT_INJECT, include/dmlc/fault.h):
the k-th pass through a pipeline stage fails with dmlc::Error, the error
reaches Python across the reader threads, and the runtime is usable again
afterwards (reference: throwing producers in
test/unittest/unittest_threaditer_exc_handling.cc:20-50, here per stage)."""
import os
import subprocess
import sys

import pytest

from dmlc_core_amd import _dmlc, data

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(autouse=True)
def disarm():
    yield
    _dmlc.fault_configure("")


def _file(tmp_path, rows=20000):
    p = str(tmp_path / "f.libsvm")
    data.write_synthetic(p, 0, rows, seed=1)
    return p


def test_read_fault_fires_on_kth_fill_then_recovers(tmp_path):
    p = _file(tmp_path)
    good = _dmlc.read_partition(p, 0, 1, "text", 2, 1 << 20)
    assert len(good) > 3
    _dmlc.fault_configure("read:3")
    with pytest.raises(_dmlc.DMLCError, match='injected fault at "read"'):
        _dmlc.read_partition(p, 0, 1, "text", 2, 1 << 20)
    assert _dmlc.fault_count("read") == 3
    _dmlc.fault_configure("")
    assert _dmlc.read_partition(p, 0, 1, "text", 2, 1 << 20) == good


def test_tracker_connect_fault():
    _dmlc.fault_configure("tracker:1")
    c = _dmlc.TrackerClient("127.0.0.1", 1, "x", -1, -1, 1.0)
    with pytest.raises(_dmlc.DMLCError, match='injected fault at "tracker"'):
        c.start()


def test_env_variable_arms_faults(tmp_path):
    p = _file(tmp_path, 2000)
    code = (f"import sys; sys.path.insert(0, {ROOT!r}); from dmlc_core_amd import _dmlc; "
            f"_dmlc.read_partition({p!r}, 0, 1, 'text', 2, 1 << 20)")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=dict(os.environ, DMLC_FAULT_INJECT="read:1"))
    assert r.returncode != 0 and 'injected fault at "read"' in r.stderr
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                       env=dict(os.environ, DMLC_FAULT_INJECT="h2d:1"))
    assert r.returncode == 0, r.stderr  # other stages are unaffected


def test_bad_spec_rejected():
    with pytest.raises(_dmlc.DMLCError, match="bad count"):
        _dmlc.fault_configure("read:0")
