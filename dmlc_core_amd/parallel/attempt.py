"""``python -m dmlc_core_amd.parallel.attempt``: print this launch's
DMLC_NUM_ATTEMPT, asked from the tracker by task id.

Launchers whose cluster relaunches a failed container on its own (YARN
services: ``restart_policy: ON_FAILURE``) cannot put an attempt counter into
the container's environment, as the reference ApplicationMaster does per
launch (``ApplicationMaster.java:446``).  The launch command runs this first:
the tracker counts the launches of every ``DMLC_TASK_ID``.  Without a tracker
(or an answer within the timeout) it prints 0, the first attempt.
"""
from __future__ import annotations

import os
import sys


def query(timeout: float = 10.0) -> int:
    from .client import TrackerClient
    task = os.environ.get("DMLC_TASK_ID")
    if task is None or "DMLC_TRACKER_URI" not in os.environ:
        return 0
    role = os.environ.get("DMLC_ROLE", "worker")
    try:
        return TrackerClient(jobid=f"attempt:{role}:{task}", timeout=timeout).attempt()
    except (OSError, ConnectionError, ValueError):
        return 0


def main() -> int:
    print(query())
    return 0


if __name__ == "__main__":
    sys.exit(main())
