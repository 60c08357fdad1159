"""Streams, sharded InputSplits and RecordIO (native, see include/dmlc/io.h)."""
from __future__ import annotations

from .._dmlc import InputSplit, RecordIOReader, RecordIOWriter, Stream  # noqa: F401

__all__ = ["InputSplit", "RecordIOReader", "RecordIOWriter", "Stream", "iter_records"]


def iter_records(uri: str, part: int = 0, nparts: int = 1, type: str = "text"):  # noqa: A002
    """Yield every record (bytes) of one partition."""
    split = InputSplit(uri, part, nparts, type)
    while True:
        rec = split.next_record()
        if rec is None:
            return
        yield rec
