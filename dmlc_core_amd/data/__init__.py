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

__all__ = ["Parser", "RowBlockIter", "GPUParser", "DeviceCSR", "csr_to_torch", "iter_blocks",
           "write_synthetic"]

write_synthetic = _dmlc.write_synthetic


def Parser(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: N802,A002
           index64: bool = False):
    """CPU streaming parser (LibSVM / LibFM / CSV), reference Parser<I>::Create."""
    cls = _dmlc.Parser64 if index64 else _dmlc.Parser
    return cls(uri, part, nparts, type)


def RowBlockIter(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: N802,A002
                 index64: bool = False):
    """CPU in-memory (or ``#cache`` paged) iterator, reference RowBlockIter<I>::Create."""
    cls = _dmlc.RowBlockIter64 if index64 else _dmlc.RowBlockIter
    return cls(uri, part, nparts, type)


def iter_blocks(uri: str, part: int = 0, nparts: int = 1, type: str = "auto",  # noqa: A002
                index64: bool = False) -> Iterator[Dict]:
    """Yield host CSR blocks (dicts of numpy arrays) of one partition."""
    p = Parser(uri, part, nparts, type, index64)
    while p.next():
        yield p.value()


def DeviceCSR(index64: bool = False):  # noqa: N802
    """Empty HBM-resident CSR container."""
    return _dmlc.DeviceCSR64() if index64 else _dmlc.DeviceCSR()


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
        cls = _dmlc.DeviceParser64 if index64 else _dmlc.DeviceParser
        self._p = cls(uri, part, nparts, cfg)

    def parse_all(self, out=None):
        """Parse the rest of the partition into ``out`` (a DeviceCSR, appended)."""
        if out is None:
            out = DeviceCSR(self.index64)
        self._p.parse_all(out)
        return out

    def before_first(self):
        self._p.before_first()

    def next(self) -> bool:
        return self._p.next()

    def value_to_host(self) -> Dict:
        return self._p.value_to_host()

    def stats(self) -> Dict:
        return self._p.stats()

    @property
    def partition_bytes(self) -> int:
        return self._p.partition_bytes()


def csr_to_torch(csr) -> Dict[str, Optional["object"]]:
    """Zero-copy torch tensors (on the HIP device) for every CSR array."""
    import torch.utils.dlpack as tdl

    out = {}
    for k, cap in csr.capsules().items():
        out[k] = None if cap is None else tdl.from_dlpack(cap)
    return out
