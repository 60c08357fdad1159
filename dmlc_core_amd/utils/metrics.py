"""Structured per-stage metrics: JSON-lines records and their
reduction across ranks.

Every record is one JSON object per line::

    {"ts": 1760000000.123, "rank": 3, "world": 8, "stage": "ingest",
     "step": 12, "rows": 1250000, "bytes": 797000000, "wait_gpu_sec": 0.01, ...}

* :class:`MetricsLogger` appends records to ``path`` (or ``$DMLC_METRICS_FILE``;
  ``{rank}`` in the path is replaced, so every rank can own a file) -- the
  reference only printed MB/s lines (``src/data/basic_row_iter.h:72-81``).
* :func:`reduce_across_ranks` turns one numeric dict per rank into
  ``{key: {"sum", "min", "max", "mean"}}`` with three all-reduces (works on
  the gloo and nccl/RCCL backends; a single process returns its own values).
* :func:`parser_record` flattens ``GPUParser.stats()`` into a record.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional


def _rank_world():
    try:
        import torch.distributed as td
        if td.is_available() and td.is_initialized():
            return td.get_rank(), td.get_world_size()
    except ImportError:  # pragma: no cover - torch is always present here
        pass
    return int(os.environ.get("RANK", os.environ.get("DMLC_RANK", "0"))), int(
        os.environ.get("WORLD_SIZE", os.environ.get("DMLC_NUM_WORKER", "1")))


class MetricsLogger:
    """Append-only JSONL metrics sink; a no-op when no path is configured."""

    def __init__(self, path: Optional[str] = None):
        path = path if path is not None else os.environ.get("DMLC_METRICS_FILE")
        rank, self.world = _rank_world()
        self.rank = rank
        self.path = path.replace("{rank}", str(rank)) if path else None
        self._f = None
        if self.path:
            d = os.path.dirname(self.path)
            if d:
                os.makedirs(d, exist_ok=True)
            self._f = open(self.path, "a", buffering=1)

    @property
    def enabled(self) -> bool:
        return self._f is not None

    def log(self, stage: str, **fields) -> Dict:
        rec = {"ts": round(time.time(), 6), "rank": self.rank, "world": self.world,
               "stage": stage}
        rec.update(fields)
        if self._f is not None:
            self._f.write(json.dumps(rec, sort_keys=True) + "\n")
        return rec

    def close(self) -> None:
        if self._f is not None:
            self._f.close()
            self._f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def reduce_across_ranks(values: Dict[str, float], device=None) -> Dict[str, Dict[str, float]]:
    """Sum / min / max / mean of every numeric field over all ranks."""
    import torch

    keys = sorted(k for k, v in values.items() if isinstance(v, (int, float, bool)))
    vec = [float(values[k]) for k in keys]
    try:
        import torch.distributed as td
        dist_on = td.is_available() and td.is_initialized()
    except ImportError:  # pragma: no cover
        dist_on = False
    if not dist_on:
        return {k: {"sum": v, "min": v, "max": v, "mean": v} for k, v in zip(keys, vec)}
    if device is None:
        device = (torch.device("cuda", torch.cuda.current_device())
                  if td.get_backend() == "nccl" else torch.device("cpu"))
    s = torch.tensor(vec, dtype=torch.float64, device=device)
    lo, hi = s.clone(), s.clone()
    td.all_reduce(s, op=td.ReduceOp.SUM)
    td.all_reduce(lo, op=td.ReduceOp.MIN)
    td.all_reduce(hi, op=td.ReduceOp.MAX)
    n = td.get_world_size()
    return {k: {"sum": a, "min": b, "max": c, "mean": a / n}
            for k, a, b, c in zip(keys, s.tolist(), lo.tolist(), hi.tolist())}


def parser_record(stats: Dict) -> Dict[str, float]:
    """Numeric fields of ``GPUParser.stats()`` / ``GPURecordIO.stats()``."""
    return {k: (float(v) if not isinstance(v, bool) else int(v)) for k, v in stats.items()
            if isinstance(v, (int, float, bool))}
