"""Distributed launch, rendezvous (dmlc tracker) and RCCL collectives.

* :mod:`.tracker` -- rendezvous server speaking the rabit protocol plus the
  ``rccl`` / ``barrier`` / ``heartbeat`` commands (reference
  `tracker/dmlc_tracker/tracker.py`).
* :mod:`.client` -- worker side of that protocol (Python twin of the C++
  ``dmlc::dist::TrackerClient``).
* :mod:`.launch` -- dmlc-submit backends: local, mpi, ssh, slurm, sge, yarn,
  mesos, kubernetes.
* :mod:`.dist` -- process-group bootstrap (one process per MI355X, RCCL),
  control collectives and the bucketed gradient all-reducer.

Only :mod:`.dist` needs torch; it (and the names it exports) load on first
use, so the tracker and the launchers run in processes that never load the
HIP runtime.
"""
from __future__ import annotations

import importlib

from . import client, tracker
from .client import TrackerClient, Topology
from .tracker import RabitTracker, PSTracker, TrackerError, get_host_ip, link_map, submit

_DIST_NAMES = ("GradAllReducer", "global_stats", "init", "finalize")


def __getattr__(name):
    if name == "dist":
        return importlib.import_module(__name__ + ".dist")
    if name in _DIST_NAMES:
        return getattr(importlib.import_module(__name__ + ".dist"), name)
    raise AttributeError(f"module {__name__!r} has no attribute {name!r}")


__all__ = ["client", "dist", "tracker", "TrackerClient", "Topology", "GradAllReducer",
           "global_stats", "init", "finalize", "RabitTracker", "PSTracker", "TrackerError",
           "get_host_ip", "link_map", "submit"]
