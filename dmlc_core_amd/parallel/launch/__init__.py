"""Cluster launchers for `dmlc-submit` (reference `tracker/dmlc_tracker/*.py`).

Each backend exposes ``submit(args)`` that starts the tracker through
:func:`dmlc_core_amd.parallel.tracker.submit` and launches the processes.
Backends build their command lines through small pure functions so they can
be checked without the cluster software installed (``--dry-run``).
"""
BACKENDS = ("local", "mpi", "ssh", "slurm", "sge", "yarn", "mesos", "kubernetes")
