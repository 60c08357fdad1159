"""Models consuming the ingestion runtime.

The reference (dmlc-core) ships no model; its consumers (XGBoost, linear
learners in ps-lite/rabit) train on RowBlocks.  These demonstrators close the
loop on MI355X: device CSR from the GPU parser -> HIP SpMV -> loss ->
gradient all-reduced over RCCL.
"""
from __future__ import annotations

import torch

from ..ops import csr_spmv, hashed_dense

__all__ = ["SparseLogReg", "HashedFM", "fp8_gemm_available"]


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


class _FP8Linear(torch.autograd.Function):
    """y = x8 @ w with x8 OCP fp8 e4m3 (scale sx) and w quantised to fp8 per
    tensor, on the MFMA fp8 path (torch._scaled_mm -> hipBLASLt); the weight
    gradient is computed in bf16 (fp8 forward / bf16 backward)."""

    @staticmethod
    def forward(ctx, x8, sx, w):
        amax = w.detach().abs().max().clamp(min=1e-12).float()
        sw = (amax / 448.0).reshape(())
        w8 = (w.detach() / sw).to(torch.float8_e4m3fn)
        y = torch._scaled_mm(x8, w8.t().contiguous().t(), scale_a=sx, scale_b=sw,
                             out_dtype=torch.float32)
        ctx.save_for_backward(x8, sx)
        return y

    @staticmethod
    def backward(ctx, gy):
        x8, sx = ctx.saved_tensors
        xb = x8.to(torch.bfloat16) * sx.to(torch.bfloat16)
        gw = (xb.t() @ gy.to(torch.bfloat16)).float()
        return None, None, gw


def fp8_gemm_available(device=None) -> bool:
    """True when torch._scaled_mm runs OCP fp8 e4m3 GEMMs on this device."""
    if not torch.cuda.is_available():
        return False
    try:
        a = torch.zeros(16, 16, device=device or "cuda").to(torch.float8_e4m3fn)
        one = torch.ones((), device=a.device)
        torch._scaled_mm(a, a.t().contiguous().t(), scale_a=one, scale_b=one,
                         out_dtype=torch.float32)
        return True
    except (RuntimeError, NotImplementedError, TypeError):
        return False


class HashedFM(torch.nn.Module):
    """Factorisation machine on hashed fp8 features (BASELINE config 5).

    Input: the ``[rows, dim]`` float8_e4m3fn batch of
    ``GPUParser.parse_all_hashed`` (fused tokenize -> hash -> fp8 kernel) or of
    :func:`~dmlc_core_amd.ops.hashed_dense`, with its quantisation ``scale``.
    ``y = b + x.w + 1/2 sum_f ((x V)_f^2 - (x^2 V^2)_f)``: the linear term and
    ``x V`` share ONE fp8 GEMM on the MFMA fp8 path (``torch._scaled_mm`` ->
    hipBLASLt, ``[w | V]`` quantised per tensor, N padded to 16); the
    ``x^2 V^2`` term is a bf16 GEMM.  Where the fp8 GEMM is unavailable the
    first term falls back to bf16 (``self.gemm`` tells which ran).
    """

    def __init__(self, dim: int = 1024, rank: int = 16, seed: int = 0):
        super().__init__()
        if dim % 16 != 0:
            raise ValueError("dim must be a multiple of 16 (fp8 GEMM tiles)")
        self.dim, self.rank, self.seed = int(dim), int(rank), int(seed)
        self.bias = torch.nn.Parameter(torch.zeros(1))
        self.w = torch.nn.Parameter(torch.zeros(dim, 1))
        self.v = torch.nn.Parameter(torch.randn(dim, rank) * 0.01)
        self.gemm = None

    def forward(self, x8: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        sx = torch.tensor(1.0 / scale, dtype=torch.float32, device=x8.device)
        wv = torch.cat([self.w, self.v], dim=1)
        n = wv.shape[1]
        pad = (-n) % 16
        wvp = torch.nn.functional.pad(wv, (0, pad))
        if self.gemm is None:
            self.gemm = "fp8" if fp8_gemm_available(x8.device) else "bf16"
        if self.gemm == "fp8":
            y = _FP8Linear.apply(x8, sx, wvp)[:, :n]
        else:
            xb = x8.to(torch.bfloat16) * sx.to(torch.bfloat16)
            y = (xb @ wvp.to(torch.bfloat16)).float()[:, :n]
        lin = y[:, 0] + self.bias
        xv = y[:, 1:]
        x2 = (x8.to(torch.float32) * sx) ** 2
        x2v2 = (x2.to(torch.bfloat16) @ (self.v ** 2).to(torch.bfloat16)).float()
        return lin + 0.5 * (xv ** 2 - x2v2).sum(-1)

    @staticmethod
    def reference(x: torch.Tensor, w, v, bias) -> torch.Tensor:
        """fp32 reference of the same model on dequantised features."""
        xv = x @ v
        return bias + (x @ w).squeeze(-1) + 0.5 * (xv ** 2 - (x ** 2) @ (v ** 2)).sum(-1)
