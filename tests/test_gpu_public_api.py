"""The reference's public factories reach the MI355X path with `?device=gpu`
(Parser<I>::Create / RowBlockIter<I>::Create, reference include/dmlc/data.h:
246-311): device-resident blocks, to_host blocks and the whole-shard
DeviceRowIter are value-identical to the CPU parser (native C++ check in
tools/dmlc_gpu_api_check.cc, plus the Python bindings)."""
import os
import subprocess

import numpy as np
import pytest

import pyref
from dmlc_core_amd import data

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "dmlc_gpu_api_check")


@pytest.mark.parametrize("fmt,nparts,args", [("libsvm", 1, "chunk_bytes=65536"),
                                             ("libsvm", 3, "chunk_bytes=40960"),
                                             ("libfm", 2, "chunk_bytes=65536"),
                                             ("csv", 2, "chunk_bytes=65536")])
def test_native_public_api_device_gpu(tmp_path, fmt, nparts, args):
    assert os.path.exists(EXE), "build with `make tools`"
    p = str(tmp_path / f"d.{fmt}")
    data.write_synthetic(p, 0, 6000, format=fmt, seed=4)
    uri = p + ("?label_column=0" if fmt == "csv" else "")
    r = subprocess.run([EXE, uri, fmt, str(nparts), args], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert r.stdout.strip().endswith("OK")


def test_python_parser_device_gpu_matches_cpu(tmp_path):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 5000, format="libsvm", seed=8, weight_every=3)
    cpu = pyref.concat_blocks(list(data.iter_blocks(p, type="libsvm")))
    gpu = pyref.concat_blocks(list(data.iter_blocks(p + "?device=gpu&chunk_bytes=65536",
                                                    type="libsvm")))
    for k in ("label", "weight", "offset", "index", "value"):
        np.testing.assert_array_equal(gpu[k], cpu[k], err_msg=k)
    it = data.RowBlockIter(p + "?device=gpu")
    assert it.num_col() == data.RowBlockIter(p).num_col()


def test_device_row_iter_empty_partition_matches_cpu(tmp_path):
    """An empty shard behaves as the reference BasicRowIter's
    (src/data/basic_row_iter.h:35-48): Next() yields one (empty) block and
    NumCol() is max_index + 1."""
    p = str(tmp_path / "two.libsvm")
    with open(p, "w") as f:
        f.write("1 3:1 7:2\n0 2:5\n")
    for part in range(8):
        cpu = data.RowBlockIter(p, part, 8, "libsvm")
        gpu = data.RowBlockIter(p + "?device=gpu", part, 8, "libsvm")
        assert gpu.num_col() == cpu.num_col(), part
        n_cpu = n_gpu = 0
        while cpu.next():
            n_cpu += 1
        while gpu.next():
            n_gpu += 1
        assert n_gpu == n_cpu == 1, (part, n_gpu, n_cpu)
