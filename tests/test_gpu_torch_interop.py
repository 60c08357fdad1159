"""PyTorch interop: device CSR -> torch.sparse_csr_tensor,
and the streaming GPUBlockDataset, checked against the CPU parser."""
import numpy as np
import pytest
import torch

import pyref
from dmlc_core_amd import data

pytestmark = pytest.mark.gpu


def _cpu(path):
    return pyref.concat_blocks(list(data.iter_blocks(path)))


def test_sparse_csr_tensor_matches_cpu(tmp_path):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 3000, seed=4)
    csr = data.GPUParser(p, chunk_bytes=64 * 1024).parse_all()
    t = data.csr_to_torch(csr)
    sp = data.to_sparse_csr(t, num_cols=int(csr.max_index) + 1)
    c = _cpu(p)
    w = torch.randn(sp.shape[1], 1, dtype=torch.float32, device="cuda")
    y = (sp @ w).squeeze(1).cpu().numpy()
    wn = w.squeeze(1).cpu().numpy()
    off = c["offset"].astype(np.int64)
    ref = np.array([np.dot(c["value"][off[r]:off[r + 1]], wn[c["index"][off[r]:off[r + 1]]])
                    for r in range(len(off) - 1)], dtype=np.float64)
    np.testing.assert_allclose(y, ref, rtol=1e-4, atol=1e-4)


def test_gpu_block_dataset_streams_every_row(tmp_path):
    p = str(tmp_path / "s.libsvm")
    data.write_synthetic(p, 0, 5000, seed=5)
    ds = data.GPUBlockDataset(p, chunk_bytes=128 * 1024, epochs=2)
    labels, nblocks = [], 0
    for blk in ds:
        labels.append(blk["label"].cpu().numpy())
        sp = data.to_sparse_csr(blk)
        assert sp.shape[0] == blk["label"].numel()
        nblocks += 1
    c = _cpu(p)
    got = np.concatenate(labels)
    assert nblocks > 4
    np.testing.assert_array_equal(got, np.concatenate([c["label"], c["label"]]))
