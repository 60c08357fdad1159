"""HIP (gfx950) kernels exposed as PyTorch operations on device CSR data.

Every op launches a hand-written CDNA4 kernel from ``libdmlc.so`` on the
current torch stream (src/gpu/feature_kernels.hip).  There is no PyTorch
fallback: on a machine without the extension or a GPU these functions raise.

CSR arguments are the dict returned by :func:`dmlc_core_amd.data.csr_to_torch`
(``offset`` int64/uint64 [rows+1], ``index`` int32/uint32 or 64-bit [nnz],
optional ``value`` float32 [nnz], optional ``field``).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from .. import _dmlc

__all__ = ["spmv", "spmv_t", "hashed_dense", "SpMVFunction", "csr_spmv", "transpose",
           "release_workspace"]

# persistent transpose scratch per (device, stream), grow-only: a rebuild (a
# further shard, a refreshed batch) allocates no multi-GB scratch again
_WORKSPACE: Dict = {}


def _workspace(nbytes: int, dev) -> torch.Tensor:
    key = (dev.index, _stream())
    ws = _WORKSPACE.get(key)
    if ws is None or ws.numel() < nbytes:
        _WORKSPACE.pop(key, None)  # free the smaller one first
        ws = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        _WORKSPACE[key] = ws
    return ws


def release_workspace() -> None:
    """Free the persistent scratch of :func:`transpose` (it is kept between
    calls so that later builds allocate only their outputs)."""
    _WORKSPACE.clear()


def _ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def _index64(csr: Dict) -> bool:
    return csr["index"].element_size() == 8


def _paired(csr: Dict) -> bool:
    """index / value are the interleaved (int32 index, float32 value) pair
    views :func:`transpose` returns: value's storage is index's shifted by one
    4-byte word, both with stride 2"""
    idx, val = csr["index"], csr.get("value")
    return (val is not None and idx.element_size() == 4 and idx.dim() == 1 and val.dim() == 1
            and idx.stride(0) == 2 and val.stride(0) == 2 and idx.numel() == val.numel()
            and val.data_ptr() == idx.data_ptr() + 4 and idx.data_ptr() % 8 == 0)


def _check(csr: Dict, pairs: bool = False):
    """device CSR arrays the kernels can take: contiguous, or (``pairs``: the
    SpMV) the interleaved pair views of a transpose"""
    if pairs and _paired(csr) and csr["offset"].is_cuda and csr["offset"].is_contiguous():
        return
    for k in ("offset", "index"):
        t = csr[k]
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError(f"csr[{k!r}] must be a contiguous device tensor")
    if csr.get("value") is not None and csr["value"].dtype != torch.float32:
        raise ValueError("csr['value'] must be float32")
    if csr.get("value") is not None and not csr["value"].is_contiguous():
        raise ValueError("csr['value'] must be contiguous")


def _unpair(csr: Dict) -> Dict:
    """a transpose's interleaved (index, value) pair views as separate
    contiguous arrays, for the kernels that take only contiguous CSR arrays
    (any other dict is returned as it is)"""
    if not _paired(csr):
        return csr
    out = dict(csr)
    out["index"], out["value"] = csr["index"].contiguous(), csr["value"].contiguous()
    out.pop("pairs", None)
    return out


def _stream() -> int:
    return int(torch.cuda.current_stream().cuda_stream)


def spmv(csr: Dict, w: torch.Tensor, bias: float = 0.0) -> torch.Tensor:
    """y[r] = sum_j value[j] * w[index[j]] + bias  (K11, 16 lanes per row).
    Takes contiguous arrays or a transpose's interleaved (index, value) pairs."""
    _check(csr, pairs=True)
    assert w.dtype == torch.float32 and w.is_cuda and w.is_contiguous()
    nrows = csr["offset"].numel() - 1
    y = torch.empty(nrows, dtype=torch.float32, device=w.device)
    _dmlc.spmv(_ptr(csr["offset"]), _ptr(csr["index"]), _ptr(csr.get("value")), nrows, _ptr(w),
               float(bias), _ptr(y), _stream(), _index64(csr))
    return y


def spmv_t(csr: Dict, d: torch.Tensor, num_features: int) -> torch.Tensor:
    """g[index[j]] += value[j] * d[row(j)]  (transposed K11, f32 atomics).
    A transpose's pair views are unpaired into contiguous copies first."""
    csr = _unpair(csr)
    _check(csr)
    assert d.dtype == torch.float32 and d.is_cuda and d.is_contiguous()
    g = torch.zeros(num_features, dtype=torch.float32, device=d.device)
    nrows = csr["offset"].numel() - 1
    _dmlc.spmv_t(_ptr(csr["offset"]), _ptr(csr["index"]), _ptr(csr.get("value")), nrows, _ptr(d),
                 _ptr(g), _stream(), _index64(csr))
    return g


def hashed_dense(csr: Dict, dim: int, seed: int = 0, fp8: bool = True,
                 scale: float = 1.0) -> torch.Tensor:
    """K9: signed feature hashing of every row into ``dim`` buckets.

    Returns float8_e4m3fn [rows, dim] (gfx950 OCP fp8, hardware conversion)
    when ``fp8`` else float32.  LibFM fields are folded into the hash key.
    """
    csr = _unpair(csr)
    _check(csr)
    nrows = csr["offset"].numel() - 1
    dev = csr["index"].device
    if fp8:
        out = torch.empty((nrows, dim), dtype=torch.uint8, device=dev)
    else:
        out = torch.empty((nrows, dim), dtype=torch.float32, device=dev)
    _dmlc.hashed_dense(_ptr(csr["offset"]), _ptr(csr["index"]), _ptr(csr.get("value")),
                       _ptr(csr.get("field")), nrows, int(dim), float(scale), int(seed) & 0xFFFFFFFF,
                       _ptr(out), bool(fp8), _stream(), _index64(csr))
    if fp8:
        return out.view(torch.float8_e4m3fn)
    return out


def transpose(csr: Dict, num_features: int, out: Optional[Dict] = None) -> Dict:
    """The CSR's transpose (CSC / inverted index) on the device, as a
    CSR-shaped dict whose rows are the features: ``offset`` int64
    [num_features + 1], ``index`` int32 row ids (ascending within every
    column), ``value`` (or None).  With values, ``index`` and ``value`` are
    the two columns of one interleaved [nnz, 2] buffer (``pairs``: int32 row,
    float32 bits), so each is a stride-2 view: the column scatter writes one
    8-byte pair per entry instead of a 4-byte store into each of two arrays,
    and :func:`spmv` reads the pairs directly (``.contiguous()`` gives
    separate copies).

    Built by the hand-written stable two-level counting sort of
    src/gpu/transpose_kernels.hip (bucket histogram -> scan -> stable bucket
    scatter -> per-bucket column histogram -> scan -> stable column scatter;
    ballot ranks, no atomics on the ordering), it turns the gradient X^T d into
    a gather SpMV (K11 over the transpose): every output is summed on chip and
    written once, instead of one memory-side f32 atomic per nonzero, which
    runs ~17x below the contiguous atomic rate when 64 lanes hit 64 different
    rows (MI355X_MICROARCH.md, Global float atomics).  Feature ids must be
    < num_features <= ``_dmlc.csr_transpose_max_features()`` (2^28: up to
    2^22 columns a two-level sort, above it three levels); an id outside
    raises.

    The sort's scratch (~10 bytes per entry) is a persistent per-device,
    per-stream workspace (:func:`release_workspace` frees it).  ``out``: a
    previous result of the same shape to overwrite instead of allocating
    the outputs (its ``index`` / ``value`` need at least nnz entries).  The
    input may itself be a transpose (its pair views are unpaired first)."""
    csr = _unpair(csr)
    _check(csr)
    offset, index, value = csr["offset"], csr["index"], csr.get("value")
    nrows, dev = offset.numel() - 1, index.device
    if num_features <= 0 or num_features > _dmlc.csr_transpose_max_features():
        raise ValueError(f"transpose: num_features must be in (0, "
                         f"{_dmlc.csr_transpose_max_features()}], got {num_features}")
    off = offset.view(torch.int64) if offset.dtype != torch.int64 else offset
    # the rows may be a slice of a larger CSR: entries [off[0], off[-1]) of index / value
    # (one device read for both ends)
    lo, hi = (int(v) for v in off[[0, -1]].tolist()) if nrows > 0 else (0, 0)
    nnz = hi - lo
    pairs = None
    if out is not None:
        col_ptr, rows, vals = out["offset"], out["index"], out.get("value")
        if (col_ptr.numel() != num_features + 1 or rows.numel() < nnz
                or (value is not None and (vals is None or vals.numel() < nnz))):
            raise ValueError("transpose: out= does not fit this CSR")
        if value is None:
            vals = None
        elif _paired(out):
            pairs = out.get("pairs")
        elif not (rows.is_contiguous() and vals.is_contiguous()):
            raise ValueError("transpose: out= index / value must be contiguous or a transpose's pairs")
    else:
        col_ptr = torch.empty(num_features + 1, dtype=torch.int64, device=dev)
        if value is not None:
            pairs = torch.empty((max(nnz, 1), 2), dtype=torch.int32, device=dev)
            rows, vals = pairs[:, 0], pairs.view(torch.float32)[:, 1]
        else:
            rows = torch.empty(max(nnz, 1), dtype=torch.int32, device=dev)
            vals = None
    scratch = _workspace(_dmlc.csr_transpose_scratch_bytes(nnz, num_features), dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _dmlc.csr_transpose(_ptr(offset), nrows, lo, nnz, _ptr(index), _ptr(value), int(num_features),
                        _ptr(col_ptr), _ptr(rows), _ptr(vals), _ptr(scratch), _ptr(err), _stream(),
                        _index64(csr))
    if int(err.item()) != 0:
        raise ValueError(f"transpose: a feature id is >= num_features ({num_features})")
    res = {"offset": col_ptr, "index": rows[:nnz],
           "value": vals[:nnz] if vals is not None else None}
    if pairs is not None:
        res["pairs"] = pairs
    return res


def _source_key(csr: Dict, num_features: int):
    """identity of the tensors a cached transpose was built from: storage,
    size and in-place version of offset / index / value"""
    def one(t):
        return None if t is None else (int(t.data_ptr()), t.numel(), t._version)
    return (num_features, one(csr["offset"]), one(csr["index"]), one(csr.get("value")))


def _whole(csr: Dict) -> bool:
    """the dict is a whole CSR (its row pointer is a complete tensor of its
    own, as csr_to_torch returns), not a row slice of a larger one -- decided
    from the tensor's storage, without reading device memory"""
    off = csr["offset"]
    return off.storage_offset() == 0 and \
        off.numel() * off.element_size() == off.untyped_storage().nbytes()


class SpMVFunction(torch.autograd.Function):
    """Autograd wrapper: forward = spmv, backward d/dw = X^T g -- a gather
    SpMV over the transpose cached in ``csr['transpose']``, or the f32-atomic
    spmv_t.  ``grad``: "transpose" builds the transpose on the first backward;
    "auto" builds it on the first backward of a whole CSR (it is reused every
    epoch) and on the second backward through the same dict otherwise (a
    batch made per step -- e.g. a row slice -- keeps the atomic form, which
    costs less than one transpose); "atomic" never builds it."""

    @staticmethod
    def forward(ctx, w, bias, csr_tuple, holder, grad):
        offset, index, value = csr_tuple
        ctx.csr = {"offset": offset, "index": index, "value": value}
        ctx.holder, ctx.grad = holder, grad
        ctx.num_features = w.numel()
        return spmv(ctx.csr, w, 0.0) + bias

    @staticmethod
    def backward(ctx, grad_out):
        grad_out = grad_out.contiguous().float()
        key = _source_key(ctx.csr, ctx.num_features)
        t = ctx.holder.get("transpose")
        if t is not None and ctx.holder.get("_transpose_key") != key:
            t = None  # the dict now holds other tensors (or they were written in place)
        if t is None and ctx.grad != "atomic":
            uses = ctx.holder.get("_backward_calls", 0) + 1
            if ctx.holder.get("_calls_key") != key:
                uses = 1
            ctx.holder["_backward_calls"] = uses
            ctx.holder["_calls_key"] = key
            # auto: only feature spaces the counting-sort transpose takes
            # (<= 2^28 columns); wider models keep the atomic scatter, which
            # has no column limit.  "transpose" asked for it: transpose() raises
            fits = ctx.num_features <= _dmlc.csr_transpose_max_features()
            if ctx.grad == "transpose" or (fits and (uses >= 2 or _whole(ctx.csr))):
                t = transpose(ctx.csr, ctx.num_features)
                ctx.holder["transpose"] = t
                ctx.holder["_transpose_key"] = key
        if t is not None and ctx.grad != "atomic":
            gw = spmv(t, grad_out, 0.0)
        else:
            gw = spmv_t(ctx.csr, grad_out, ctx.num_features)
        gb = grad_out.sum().reshape(1)
        return gw, gb, None, None, None


def csr_spmv(csr: Dict, w: torch.Tensor, bias: torch.Tensor, grad: str = "auto") -> torch.Tensor:
    """Differentiable y = X w + b for a device CSR batch.  X^T g runs as a
    gather SpMV over the CSR's transpose cached in ``csr['transpose']`` (one
    hand-written counting-sort transpose; ~16x faster than atomics on a
    10 M x 1 M batch) or as an
    f32-atomic scatter: grad="auto" (the default) builds the transpose on the
    first backward of a whole CSR and once a row-slice dict is seen a second
    time (only up to ``_dmlc.csr_transpose_max_features()`` = 2^28 columns;
    wider models stay on the atomic form), "transpose" at once, "atomic"
    never."""
    if grad not in ("auto", "transpose", "atomic"):
        raise ValueError(f"grad must be 'auto', 'transpose' or 'atomic', got {grad!r}")
    return SpMVFunction.apply(w, bias, (csr["offset"], csr["index"], csr.get("value")), csr, grad)
