"""End-to-end demonstrator on one MI355X: GPU parse -> SpMV logistic
regression -> (world-1) gradient reducer -> SGD; the loss must fall."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_train_sparse_logreg_example():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "DMLC_TRACKER_URI"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "train_sparse_logreg.py"),
                        "--rows", "50000", "--epochs", "3", "--batch-rows", "8192"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    losses = out["loss_per_epoch"]
    assert out["rows"] == 50000
    assert losses[-1] < losses[0]


def test_train_hashed_fm_example():
    """Config 5 end to end: LibFM -> fused hash -> fp8 batch -> HashedFM on the
    MFMA kernels -> Adam; the loss must fall."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "DMLC_TRACKER_URI"):
        env.pop(k, None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "train_hashed_fm.py"),
                        "--rows", "40000", "--dim", "512", "--epochs", "3", "--batch-rows", "8192"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert out["gemm"] == "hip_mfma_bf16" and out["rows_rank0"] == 40000
    losses = out["loss_per_epoch"]
    assert losses[-1] < losses[0], losses
