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
"""
from __future__ import annotations

from . import client, dist, tracker
from .client import TrackerClient, Topology
from .dist import GradAllReducer, global_stats, init, finalize
from .tracker import RabitTracker, PSTracker, TrackerError, get_host_ip, link_map, submit

__all__ = ["client", "dist", "tracker", "TrackerClient", "Topology", "GradAllReducer",
           "global_stats", "init", "finalize", "RabitTracker", "PSTracker", "TrackerError",
           "get_host_ip", "link_map", "submit"]
