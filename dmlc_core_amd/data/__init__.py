"""Parsers and row-block iterators.

CPU path (reference parity, include/dmlc/data.h): :class:`Parser`,
:class:`RowBlockIter` return host CSR blocks as numpy arrays.

GPU path (MI355X): :class:`GPUParser` streams a shard through the pinned ring
into HIP kernels and keeps the CSR resident in HBM; :func:`csr_to_torch`
exposes it to PyTorch zero-copy (DLPack, device = the HIP device).
"""
from __future__ import annotations

from typing import Dict, Iterator, Optional

from .. import _dmlc

__all__ = ["Parser", "RowBlockIter", "GPUParser", "ShuffledGPUParser", "DeviceCSR", "csr_to_torch",
           "iter_blocks", "write_synthetic", "to_sparse_csr", "GPUBlockDataset", "PageCache",
           "write_page_cache"]

write_synthetic = _dmlc.write_synthetic


def _host_blocks_uri(uri: str) -> str:
    """``?device=gpu`` URIs tokenise on the MI355X; the numpy views returned by
    value() need host blocks, so ``to_host=1`` is added (device-resident blocks
    are served by GPUParser / DeviceCSR instead)."""
    q = uri.split("#", 1)[0]
    if "?" not in q:
        return uri
    args = dict(kv.split("=", 1) for kv in q.split("?", 1)[1].split("&") if "=" in kv)
    if not args.get("device", "").startswith("gpu") or "to_host" in args:
        return uri
    head, _, tail = uri.partition("#")
    return head + "&to_host=1" + ("#" + tail if tail else "")


def Parser(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: N802,A002
           index64: bool = False):
    """Streaming parser (LibSVM / LibFM / CSV), reference Parser<I>::Create;
    ``?device=gpu`` selects the HIP tokeniser (blocks copied back to the host)."""
    cls = _dmlc.Parser64 if index64 else _dmlc.Parser
    return cls(_host_blocks_uri(uri), part, nparts, type)


def RowBlockIter(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: N802,A002
                 index64: bool = False):
    """In-memory (or ``#cache`` paged) iterator, reference RowBlockIter<I>::Create;
    ``?device=gpu`` parses the whole shard on the MI355X (DeviceRowIter), and
    with ``#cachefile`` loads / builds the same binary page file DiskRowIter uses."""
    cls = _dmlc.RowBlockIter64 if index64 else _dmlc.RowBlockIter
    return cls(_host_blocks_uri(uri), part, nparts, type)


def iter_blocks(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: A002
                index64: bool = False) -> Iterator[Dict]:
    """Yield host CSR blocks (dicts of numpy arrays) of one partition."""
    p = Parser(uri, part, nparts, type, index64)
    while p.next():
        yield p.value()


def DeviceCSR(index64: bool = False):  # noqa: N802
    """Empty HBM-resident CSR container."""
    return _dmlc.DeviceCSR64() if index64 else _dmlc.DeviceCSR()


def PageCache(path: str, device: int = -1, index64: bool = False):  # noqa: N802
    """Open a ``#cache`` page file (DiskRowIter's binary RowBlock pages) for
    zero-copy DMA into HBM: ``.load(csr)`` replaces a :func:`DeviceCSR`'s
    contents with every page (no parse).  None when the file does not exist."""
    cls = _dmlc.PageCache64 if index64 else _dmlc.PageCache
    return cls.open(path, device)


def write_page_cache(csr, path: str, page_mb: float = 64.0) -> int:
    """Write a DeviceCSR as ``#cache`` pages (the CPU DiskRowIter's format and
    64 MiB page rule: same bytes for the same shard).  Returns the page count."""
    cls = _dmlc.PageCache64 if isinstance(csr, _dmlc.DeviceCSR64) else _dmlc.PageCache
    return cls.write(csr, path, page_mb)


class GPUParser:
    """Text shard -> CSR in HBM on the current HIP device.

    Parameters mirror ``dmlc::gpu::DeviceParserConfig``: ``format`` (libsvm |
    libfm | csv), ``chunk_mb``, ``pinned_slots``, ``device_slots``,
    ``read_threads``, ``device``, and CSV ``label_column`` / ``weight_column`` /
    ``delimiter``.  URI ``?k=v`` arguments override them.
    """

    def __init__(self, uri: str, part: int = 0, nparts: int = 1, format: str = "libsvm",  # noqa: A002
                 index64: bool = False, **config):
        cfg = {"format": format}
        cfg.update({k: str(v) for k, v in config.items()})
        self.index64 = index64
        self._where = {"uri": uri, "part": part, "nparts": nparts, "format": format}
        cls = _dmlc.DeviceParser64 if index64 else _dmlc.DeviceParser
        self._p = cls(uri, part, nparts, cfg)

    def parse_all(self, out=None):
        """Parse the rest of the partition into ``out`` (a DeviceCSR, appended)."""
        if out is None:
            out = DeviceCSR(self.index64)
        self._p.parse_all(out)
        return out

    def parse_all_hashed(self, dim: int, seed: int = 0, fp8: bool = True, scale: float = 1.0,
                         strategy: str = "auto", out: Optional[Dict] = None):
        """Rest of the partition as a hashed dense batch (BASELINE config 5).
        Returns ``{"x": [rows, dim] float8_e4m3fn (or float32), "label": [rows]
        float32, "batch": handle}`` as torch tensors on the device.

        ``strategy``: ``"fused"`` (and ``"auto"``) tokenises, hashes and packs
        with ONE wave-per-tile kernel per chunk (no CSR in between; the tile
        parser's fast path when dim % 16 == 0, the exact per-line kernel
        otherwise); ``"csr"`` parses to a device CSR and runs
        :func:`dmlc_core_amd.ops.hashed_dense` (K9).  Both compute the same hash
        and the same fp8 bytes.

        ``out``: an earlier result of this call whose tensors are no longer
        used; its HBM buffers are refilled in place (no multi-GB allocation
        per epoch) and, when the shape is unchanged, ``out`` itself is
        returned (its ``x`` / ``label`` alias the new batch).  When the refill
        has to grow or reshape the batch, a new dict is returned; tensors of
        the earlier result keep their own (old, still valid) buffers, which
        are freed when the last of them goes -- each DLPack capsule owns the
        buffer it exports."""
        import torch
        import torch.utils.dlpack as tdl

        if strategy not in ("auto", "fused", "csr"):
            raise ValueError(f"strategy must be auto, fused or csr, not {strategy!r}")
        if strategy == "csr":
            from .. import ops

            t = csr_to_torch(self.parse_all())
            x = ops.hashed_dense(t, int(dim), seed=seed, fp8=fp8, scale=scale)
            return {"x": x, "label": t["label"].clone(), "batch": None}  # the CSR is released

        handle = out.get("batch") if isinstance(out, dict) else out
        if handle is not None and torch.cuda.is_available():
            # the refill must not overtake torch work still reading the old batch
            if getattr(self, "_ext_stream", None) is None:
                self._ext_stream = torch.cuda.ExternalStream(self._p.stream())
            self._ext_stream.wait_stream(torch.cuda.current_stream())
        d = self._p.parse_all_hashed(int(dim), float(scale), int(seed) & 0xFFFFFFFF, bool(fp8), handle)
        if isinstance(out, dict) and out.get("batch") is d["batch"] and "x" in out:
            # refilled in place with the same shape: the tensors already alias it
            x0 = out["x"]
            if (tuple(x0.shape) == (d["rows"], d["dim"]) and x0.data_ptr() == d["x_ptr"]
                    and out["label"].data_ptr() == d["label_ptr"]
                    and (x0.dtype == torch.float8_e4m3fn) == bool(fp8)):
                return out
        x = tdl.from_dlpack(d["x"]).view(d["rows"], d["dim"])
        if fp8:
            x = x.view(torch.float8_e4m3fn)
        return {"x": x, "label": tdl.from_dlpack(d["label"]), "batch": d["batch"]}

    def before_first(self):
        self._p.before_first()

    def tell(self) -> int:
        """Mid-epoch resume cursor: partition byte offset of the first record
        not yet delivered (a record boundary)."""
        return self._p.tell()

    def seek(self, cursor: int) -> None:
        """Continue from a :meth:`tell` cursor."""
        self._p.seek(int(cursor))

    def state_dict(self) -> Dict:
        """Checkpointable position (store it next to the model state)."""
        return dict(self._where, cursor=self.tell())

    def load_state_dict(self, state: Dict) -> None:
        for k in ("uri", "part", "nparts", "format"):
            if state[k] != self._where[k]:
                raise ValueError(f"state is for {k}={state[k]!r}, parser has {self._where[k]!r}")
        self.seek(state["cursor"])

    def next(self) -> bool:
        return self._p.next()

    def value_to_host(self) -> Dict:
        return self._p.value_to_host()

    def value_torch(self) -> Dict:
        """Zero-copy torch views of the last next() block (valid until next())."""
        import torch.utils.dlpack as tdl

        return {k: None if c is None else tdl.from_dlpack(c)
                for k, c in self._p.value_capsules().items()}

    def stream(self) -> int:
        return self._p.stream()

    def stats(self) -> Dict:
        return self._p.stats()

    @property
    def partition_bytes(self) -> int:
        return self._p.partition_bytes()


class ShuffledGPUParser(GPUParser):
    """GPU counterpart of ``InputSplitShuffle`` (reference
    ``include/dmlc/input_split_shuffle.h``), native: the rank's shard is cut
    into ``num_shuffle_parts`` sub-shards (partition ``part * K + i`` of
    ``nparts * K``) visited each epoch in the order the CPU split uses
    (``std::mt19937(666 + part + nparts + K + seed)``, reshuffled by
    ``before_first``).  ONE C++ DeviceParser pipeline serves every sub-shard
    (``?shuffle_parts=K&shuffle_seed=S``): its reader / zero-copy source is
    re-targeted per epoch, and with ``hbm_cache=1`` every sub-shard's chunks
    replay from HBM in each epoch's order.  Rows come out in the CPU split's
    record order; ``state_dict`` carries the epoch and the cursor.
    """

    def __init__(self, uri: str, part: int = 0, nparts: int = 1, num_shuffle_parts: int = 2,
                 shuffle_seed: int = 0, format: str = "libsvm", index64: bool = False,  # noqa: A002
                 **config):
        if num_shuffle_parts < 1:
            raise ValueError("num_shuffle_parts must be >= 1")
        self.k, self.seed = int(num_shuffle_parts), int(shuffle_seed)
        super().__init__(uri, part, nparts, format=format, index64=index64,
                         shuffle_parts=self.k, shuffle_seed=self.seed, **config)
        self._where.update(num_shuffle_parts=self.k, shuffle_seed=self.seed)

    @property
    def order(self):
        """sub-shard visiting order of the current epoch"""
        return list(self._p.visit_order())

    @property
    def epoch(self) -> int:
        return self._p.epoch()

    def state_dict(self) -> Dict:
        return dict(self._where, epoch=self.epoch, cursor=self.tell())

    def load_state_dict(self, state: Dict) -> None:
        for k in ("uri", "part", "nparts", "format", "num_shuffle_parts", "shuffle_seed"):
            if state[k] != self._where[k]:
                raise ValueError(f"state is for {k}={state[k]!r}, parser has {self._where[k]!r}")
        self._p.set_epoch(int(state["epoch"]))
        self.seek(state["cursor"])


def csr_to_torch(csr) -> Dict[str, Optional["object"]]:
    """Zero-copy torch tensors (on the HIP device) for every CSR array."""
    import torch.utils.dlpack as tdl

    out = {}
    for k, cap in csr.capsules().items():
        out[k] = None if cap is None else tdl.from_dlpack(cap)
    return out


def to_sparse_csr(t: Dict, num_cols: Optional[int] = None):
    """torch.sparse_csr_tensor view of a device CSR dict (``csr_to_torch`` /
    ``GPUParser.value_torch`` output).  Index arrays are widened to int64
    (torch's sparse CSR layout); values default to 1 for binary rows."""
    import torch

    offset = t["offset"]
    crow = (offset.view(torch.int64) if offset.dtype == torch.uint64 else offset).to(torch.int64)
    crow = crow - crow[0]
    idx = t["index"]
    if idx.dtype == torch.uint32:
        col = idx.view(torch.int32).to(torch.int64)  # indices < 2^31 in practice
    elif idx.dtype == torch.uint64:
        col = idx.view(torch.int64)
    else:
        col = idx.to(torch.int64)
    base = int(offset[0].item()) if offset.numel() else 0
    nnz = int(crow[-1].item()) if crow.numel() else 0
    col = col[base:base + nnz]
    val = t.get("value")
    val = torch.ones(nnz, dtype=torch.float32, device=col.device) if val is None else val[base:base + nnz]
    ncols = int(num_cols) if num_cols is not None else (int(col.max().item()) + 1 if nnz else 0)
    return torch.sparse_csr_tensor(crow, col, val, size=(crow.numel() - 1, ncols))


class GPUBlockDataset:
    """torch.utils.data-style iterable over GPU-parsed blocks of one shard.

    Each item is a dict of device tensors for one parsed chunk (offset,
    label, index, value, ...).  The tensors are views of the parser's buffers:
    consume (or clone) them before requesting the next item.  Use with
    ``DataLoader(ds, batch_size=None)`` or iterate directly.
    """

    def __init__(self, uri: str, part: int = 0, nparts: int = 1, format: str = "libsvm",  # noqa: A002
                 epochs: int = 1, **config):
        self.args = (uri, part, nparts, format, config)
        self.epochs = epochs

    def __iter__(self):
        uri, part, nparts, fmt, config = self.args
        p = GPUParser(uri, part, nparts, format=fmt, **config)
        for epoch in range(self.epochs):
            if epoch:
                p.before_first()
            while p.next():
                yield p.value_torch()
