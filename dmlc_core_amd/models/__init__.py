"""Models consuming the ingestion runtime.

The reference (dmlc-core) ships no model; its consumers (XGBoost, linear
learners in ps-lite/rabit) train on RowBlocks.  These demonstrators close the
loop on MI355X: device CSR from the GPU parser -> HIP SpMV -> loss ->
gradient all-reduced over RCCL.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..ops import csr_spmv, hashed_dense

__all__ = ["SparseLogReg", "HashedFM"]


class SparseLogReg(torch.nn.Module):
    """Sparse logistic regression: p(y=1|x) = sigmoid(x . w + b)."""

    def __init__(self, num_features: int, grad: str = "auto"):
        super().__init__()
        self.num_features = int(num_features)
        self.grad = grad  # X^T g: "auto" / "transpose" (cached inverted index) / "atomic"
        self.weight = torch.nn.Parameter(torch.zeros(self.num_features, dtype=torch.float32))
        self.bias = torch.nn.Parameter(torch.zeros(1, dtype=torch.float32))

    def forward(self, csr) -> torch.Tensor:
        return csr_spmv(csr, self.weight, self.bias, grad=self.grad)

    def loss(self, csr) -> torch.Tensor:
        logits = self.forward(csr)
        label = csr["label"].float()
        w = csr.get("weight")
        return torch.nn.functional.binary_cross_entropy_with_logits(
            logits, label, weight=w, reduction="mean")


class _HashedFMFunction(torch.autograd.Function):
    """HashedFM forward / backward as two HIP kernels over the fp8 batch
    (src/gpu/fm_kernels.hip): F1 reads the batch once and writes y and xV,
    F2 reads it once more and writes per-block partials of G^T X and
    (X^2)^T g, F3/F4 sum them and form dw, dV; no fp32 / bf16 copy of the
    batch exists."""

    @staticmethod
    def forward(ctx, x8, sx: float, w, v, bias):
        rows, dim = x8.shape
        dev = x8.device
        # F0: [w | V]^T in bf16 and q = rowsum(V^2), one kernel
        wf = w.detach().float().contiguous()
        vf = v.detach().float().contiguous()
        wt = torch.empty((v.shape[1] + 1, dim), dtype=torch.bfloat16, device=dev)
        q = torch.empty(dim, dtype=torch.float32, device=dev)
        _dmlc().fm_prep(wf.data_ptr(), vf.data_ptr(), dim, wt.data_ptr(), q.data_ptr(), _stream())
        b = bias.detach().float().contiguous()
        y = torch.empty(rows, dtype=torch.float32, device=dev)
        xv = torch.empty((rows, v.shape[1]), dtype=torch.float32, device=dev)
        _dmlc().fm_forward(x8.data_ptr(), rows, dim, wt.data_ptr(), q.data_ptr(), b.data_ptr(),
                           float(sx), y.data_ptr(), xv.data_ptr(), _num_cus(dev), _stream())
        ctx.save_for_backward(x8, xv, v.detach())
        ctx.sx = float(sx)
        return y

    @staticmethod
    def backward(ctx, gy):
        x8, xv, v = ctx.saved_tensors
        rows, dim = x8.shape
        g = gy.detach().float().contiguous()
        nblk = max(1, min(2 * _num_cus(x8.device), (rows + 31) // 32))
        part = torch.empty((nblk, v.shape[1] + 2, dim), dtype=torch.float32, device=x8.device)
        _dmlc().fm_backward(x8.data_ptr(), rows, dim, g.data_ptr(), xv.data_ptr(), nblk,
                            part.data_ptr(), _stream())
        # F3 + F4: partials summed and turned into dw, dV on the device
        vf = v.float().contiguous()
        z = torch.empty((v.shape[1] + 2, dim), dtype=torch.float32, device=x8.device)
        gw = torch.empty((dim, 1), dtype=torch.float32, device=x8.device)
        gv = torch.empty((dim, v.shape[1]), dtype=torch.float32, device=x8.device)
        _dmlc().fm_reduce_grads(part.data_ptr(), nblk, dim, vf.data_ptr(), ctx.sx, z.data_ptr(),
                                gw.data_ptr(), gv.data_ptr(), _stream())
        return None, None, gw.to(v.dtype), gv.to(v.dtype), g.sum().reshape(1)


_FM_LOSSES = {"logistic": 0, "squared": 1}


class _HashedFMLossFunction(torch.autograd.Function):
    """Forward + loss + backward of one HashedFM step as one HIP kernel over
    the fp8 batch (F5 k_fm_fused, src/gpu/fm_kernels.hip), then F3/F4 for dw,
    dV.  The gradients exist after forward; backward scales them by the
    incoming gradient of the (scalar) loss."""

    @staticmethod
    def forward(ctx, x8, label, weight, sx: float, kind: int, y, w, v, bias):
        rows, dim = x8.shape
        dev = x8.device
        rank = v.shape[1]
        wf = w.detach().float().contiguous()
        vf = v.detach().float().contiguous()
        wt = torch.empty((rank + 1, dim), dtype=torch.bfloat16, device=dev)
        q = torch.empty(dim, dtype=torch.float32, device=dev)
        ext = _dmlc()
        ext.fm_prep(wf.data_ptr(), vf.data_ptr(), dim, wt.data_ptr(), q.data_ptr(), _stream())
        b = bias.detach().float().contiguous()
        lab = label.detach().to(device=dev, dtype=torch.float32).contiguous()
        wgt = None if weight is None else weight.detach().to(device=dev,
                                                             dtype=torch.float32).contiguous()
        if lab.numel() != rows or (wgt is not None and wgt.numel() != rows):
            raise ValueError("label / weight must have one value per row")
        # one workgroup per CU: eight waves of 248 VGPRs fill a CU
        nblk = max(1, min(_num_cus(dev), (rows + 31) // 32))
        part = torch.empty((nblk, rank + 2, dim), dtype=torch.float32, device=dev)
        lpart = torch.empty((nblk, 2), dtype=torch.float32, device=dev)
        ext.fm_fused(x8.data_ptr(), rows, dim, wt.data_ptr(), q.data_ptr(), b.data_ptr(), float(sx),
                     lab.data_ptr(), 0 if wgt is None else wgt.data_ptr(), int(kind), 1.0 / rows,
                     nblk, y.data_ptr(), part.data_ptr(), lpart.data_ptr(), _stream())
        z = torch.empty((rank + 2, dim), dtype=torch.float32, device=dev)
        gw = torch.empty((dim, 1), dtype=torch.float32, device=dev)
        gv = torch.empty((dim, rank), dtype=torch.float32, device=dev)
        ext.fm_reduce_grads(part.data_ptr(), nblk, dim, vf.data_ptr(), float(sx), z.data_ptr(),
                            gw.data_ptr(), gv.data_ptr(), _stream())
        sums = lpart.sum(0)
        ctx.save_for_backward(gw, gv, sums[1:2].clone())
        ctx.dtypes = (w.dtype, v.dtype, bias.dtype)
        return sums[0] / rows

    @staticmethod
    def backward(ctx, gl):
        gw, gv, gb = ctx.saved_tensors
        tw, tv, tb = ctx.dtypes
        return (None, None, None, None, None, None, (gw * gl).to(tw), (gv * gl).to(tv),
                (gb * gl).to(tb))


def _dmlc():
    from .. import _dmlc as ext
    return ext


def _stream() -> int:
    return int(torch.cuda.current_stream().cuda_stream)


_CUS = {}


def _num_cus(dev) -> int:
    i = dev.index if dev.index is not None else torch.cuda.current_device()
    if i not in _CUS:
        _CUS[i] = torch.cuda.get_device_properties(i).multi_processor_count
    return _CUS[i]


class HashedFM(torch.nn.Module):
    """Factorisation machine on hashed fp8 features (BASELINE config 5).

    Input: the ``[rows, dim]`` float8_e4m3fn batch of
    ``GPUParser.parse_all_hashed`` (fused tokenize -> hash -> fp8 kernel) or of
    :func:`~dmlc_core_amd.ops.hashed_dense`, with its quantisation ``scale``.
    ``y = b + x.w + 1/2 sum_f ((x V)_f^2 - (x^2 V^2)_f)``; the last term is
    ``x^2 . q`` with ``q = rowsum(V^2)``.  On a GPU (rank 16, dim a multiple of
    128) forward and backward are the bf16-MFMA kernels of
    ``src/gpu/fm_kernels.hip``, each reading the fp8 batch once; elsewhere the
    fp32 formula runs on the dequantised batch (``self.gemm`` tells which).
    """

    def __init__(self, dim: int = 1024, rank: int = 16, seed: int = 0):
        super().__init__()
        if dim % 16 != 0:
            raise ValueError("dim must be a multiple of 16")
        self.dim, self.rank, self.seed = int(dim), int(rank), int(seed)
        self.bias = torch.nn.Parameter(torch.zeros(1))
        self.w = torch.nn.Parameter(torch.zeros(dim, 1))
        self.v = torch.nn.Parameter(torch.randn(dim, rank) * 0.01)
        self.gemm = None
        self.last_logits = None

    def _native(self, x8: torch.Tensor) -> bool:
        return (x8.is_cuda and x8.dtype == torch.float8_e4m3fn and self.rank == 16
                and self.dim % 128 == 0 and self.dim <= 2048)

    def loss(self, x8: torch.Tensor, label: torch.Tensor, scale: float = 1.0,
             loss: str = "logistic", weight: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Mean training loss of the batch: ``"logistic"`` (binary cross
        entropy on the logits, labels in [0, 1]) or ``"squared"``, optionally
        row-weighted (``mean(weight * loss)``, as torch's
        ``binary_cross_entropy_with_logits(weight=...)``).

        On a GPU with dim 128 / 256 / 512 / 1024 this is one fused pass over
        the fp8 batch (``k_fm_fused``: forward, loss, dloss/dy and the
        backward products per 32-row tile, the batch read once per step
        instead of twice); its backward only scales the gradients it already
        holds.  Elsewhere: ``forward`` then the torch loss.  The logits of the
        last call are kept in ``self.last_logits``."""
        if loss not in _FM_LOSSES:
            raise ValueError(f"loss must be one of {sorted(_FM_LOSSES)}, got {loss!r}")
        if self._native(x8) and self.dim in (128, 256, 512, 1024) and x8.shape[0] > 0:
            self.gemm = "hip_mfma_bf16_fused"
            y = torch.empty(x8.shape[0], dtype=torch.float32, device=x8.device)
            out = _HashedFMLossFunction.apply(x8.contiguous(), label, weight, 1.0 / scale,
                                              _FM_LOSSES[loss], y, self.w, self.v, self.bias)
            self.last_logits = y
            return out
        y = self.forward(x8, scale)
        self.last_logits = y.detach()
        lab = label.to(y.dtype)
        if loss == "logistic":
            return torch.nn.functional.binary_cross_entropy_with_logits(y, lab, weight=weight)
        err = (y - lab) ** 2
        return (err * weight).mean() if weight is not None else err.mean()

    def forward(self, x8: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        if self._native(x8):
            self.gemm = "hip_mfma_bf16"
            return _HashedFMFunction.apply(x8.contiguous(), 1.0 / scale, self.w, self.v, self.bias)
        self.gemm = "torch_fp32"
        return self.reference(x8.float() / scale, self.w, self.v, self.bias)
    @staticmethod
    def reference(x: torch.Tensor, w, v, bias) -> torch.Tensor:
        """fp32 reference of the same model on dequantised features."""
        xv = x @ v
        return bias + (x @ w).squeeze(-1) + 0.5 * (xv ** 2 - (x ** 2) @ (v ** 2)).sum(-1)
