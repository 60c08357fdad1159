"""Models consuming the ingestion runtime.

The reference (dmlc-core) ships no model; its consumers (XGBoost, linear
learners in ps-lite/rabit) train on RowBlocks.  These demonstrators close the
loop on MI355X: device CSR from the GPU parser -> HIP SpMV -> loss ->
gradient all-reduced over RCCL.
"""
from __future__ import annotations

import torch

from ..ops import csr_spmv, hashed_dense

__all__ = ["SparseLogReg", "HashedFM"]


class SparseLogReg(torch.nn.Module):
    """Sparse logistic regression: p(y=1|x) = sigmoid(x . w + b)."""

    def __init__(self, num_features: int):
        super().__init__()
        self.num_features = int(num_features)
        self.weight = torch.nn.Parameter(torch.zeros(self.num_features, dtype=torch.float32))
        self.bias = torch.nn.Parameter(torch.zeros(1, dtype=torch.float32))

    def forward(self, csr) -> torch.Tensor:
        return csr_spmv(csr, self.weight, self.bias)

    def loss(self, csr) -> torch.Tensor:
        logits = self.forward(csr)
        label = csr["label"].float()
        w = csr.get("weight")
        return torch.nn.functional.binary_cross_entropy_with_logits(
            logits, label, weight=w, reduction="mean")


class HashedFM(torch.nn.Module):
    """Factorisation-machine-style model on hashed fp8 features (K9 output).

    x = hashed_dense(csr, dim) in OCP fp8 e4m3 -> bf16 -> linear + pairwise
    interaction through a rank-k projection (matmul on MFMA via hipBLASLt).
    """

    def __init__(self, dim: int = 1024, rank: int = 16, seed: int = 0):
        super().__init__()
        self.dim, self.seed = int(dim), int(seed)
        self.linear = torch.nn.Linear(dim, 1)
        self.v = torch.nn.Parameter(torch.randn(dim, rank) * 0.01)

    def forward(self, csr) -> torch.Tensor:
        x = hashed_dense(csr, self.dim, seed=self.seed, fp8=True).to(torch.bfloat16)
        lin = self.linear(x.float()).squeeze(-1)
        xv = x.float() @ self.v
        x2v2 = (x.float() ** 2) @ (self.v ** 2)
        inter = 0.5 * (xv ** 2 - x2v2).sum(-1)
        return lin + inter
