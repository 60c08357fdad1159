"""Small utilities: logging with rank prefix, timing, environment helpers."""
from __future__ import annotations

import logging
import os
import time

_LOGGER = None


def get_logger(name: str = "dmlc") -> logging.Logger:
    """Logger whose lines carry ``[rank r]`` when RANK / DMLC_RANK is set."""
    global _LOGGER
    if _LOGGER is None:
        rank = os.environ.get("DMLC_RANK", os.environ.get("RANK", ""))
        prefix = f"[rank {rank}] " if rank else ""
        handler = logging.StreamHandler()
        handler.setFormatter(logging.Formatter(f"[%(asctime)s] {prefix}%(message)s", "%H:%M:%S"))
        _LOGGER = logging.getLogger(name)
        _LOGGER.addHandler(handler)
        _LOGGER.setLevel(os.environ.get("DMLC_LOG_LEVEL", "INFO"))
        _LOGGER.propagate = False
    return _LOGGER


def get_time() -> float:
    """Monotonic seconds (same clock as the C++ dmlc::GetTime)."""
    return time.perf_counter()


def get_env(key: str, default):
    """Typed environment lookup: unset or blank returns ``default`` (parity with
    dmlc::GetEnv, reference include/dmlc/parameter.h:1036-1050)."""
    val = os.environ.get(key)
    if val is None or val == "":
        return default
    if isinstance(default, bool):
        low = val.strip().lower()
        if low in ("1", "true"):
            return True
        if low in ("0", "false"):
            return False
        raise ValueError(f"invalid boolean for {key}: {val!r}")
    return type(default)(val)
