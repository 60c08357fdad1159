"""Streams, sharded InputSplits and RecordIO (native, see include/dmlc/io.h),
plus the GPU RecordIO reader (K7 kernels, include/dmlc/gpu/device_recordio.h)."""
from __future__ import annotations

from typing import Dict, Iterator, List, Tuple

from .._dmlc import (DeviceRecordIO, InputSplit, PartitionReader, RecordIOReader,  # noqa: F401
                     RecordIOWriter, Stream, read_partition)

__all__ = ["InputSplit", "RecordIOReader", "RecordIOWriter", "Stream", "iter_records",
           "GPURecordIO", "split_records", "PartitionReader", "read_partition"]


def iter_records(uri: str, part: int = 0, nparts: int = 1, type: str = "text"):  # noqa: A002
    """Yield every record (bytes) of one partition."""
    split = InputSplit(uri, part, nparts, type)
    while True:
        rec = split.next_record()
        if rec is None:
            return
        yield rec


def split_records(offsets, data: bytes) -> List[bytes]:
    """Byte-CSR (offsets, payload) -> list of record bytes."""
    return [data[int(offsets[i]):int(offsets[i + 1])] for i in range(len(offsets) - 1)]


class GPURecordIO:
    """RecordIO partition decoded on the MI355X.

    >>> r = GPURecordIO("data.rec", part, nparts, chunk_mb=64)
    >>> batch = r.read_all()            # whole shard resident in HBM
    >>> t = r.to_torch(batch)           # {"offset": int64? u64 tensor, "data": u8 tensor}

    Streaming: ``for offsets, data in r.iter_host(): ...`` (one chunk at a time).
    Config keys (also ``?k=v`` on the uri): chunk_mb, chunk_bytes, device,
    zero_copy, device_slots, pinned_slots, hbm_cache (epochs after the first
    decode from an HBM-resident copy), replay_chunk_mb, and for indexed
    RecordIO ``index=<index file>``, ``shuffle``, ``seed`` -- the epoch order of
    the CPU ``indexed_recordio`` InputSplit, gathered on the device.
    """

    def __init__(self, uri: str, part: int = 0, nparts: int = 1, **config):
        self._r = DeviceRecordIO(uri, part, nparts, {k: str(v) for k, v in config.items()})

    def read_all(self) -> Dict[str, object]:
        return self._r.read_all()

    def resident_to_host(self) -> Tuple[object, bytes]:
        return self._r.resident_to_host()

    def iter_host(self) -> Iterator[Tuple[object, bytes]]:
        while self._r.next():
            yield self._r.value_to_host()

    def before_first(self) -> None:
        self._r.before_first()

    def stats(self) -> Dict[str, object]:
        return self._r.stats()

    @property
    def partition_bytes(self) -> int:
        return self._r.partition_bytes()

    @staticmethod
    def to_torch(batch: Dict[str, object]) -> Dict[str, object]:
        import torch.utils.dlpack as tdl
        return {"offset": tdl.from_dlpack(batch["offset"]), "data": tdl.from_dlpack(batch["data"]),
                "size": batch["size"], "bytes": batch["bytes"]}
