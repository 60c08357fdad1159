"""MPI backend: mpirun as a process launcher (reference
`tracker/dmlc_tracker/mpi.py:12-82`).  OpenMPI exports env with ``-x K``,
MPICH/Intel MPI with ``-env K V`` (the reference's ``--verion`` typo and
bytes/str compare are fixed, §7.4 #7).  With ``--gpus-per-node`` the worker
command is wrapped so every rank binds GPU ``OMPI_COMM_WORLD_LOCAL_RANK`` /
``MPI_LOCALRANKID``.
"""
from __future__ import annotations

import subprocess
import threading
from typing import Dict, List

from .. import tracker
from .opts import user_envs

LOCAL_RANK_SNIPPET = ('export DMLC_LOCAL_RANK=${OMPI_COMM_WORLD_LOCAL_RANK:-'
                      '${MPI_LOCALRANKID:-${PMI_LOCAL_RANK:-0}}}; '
                      'export LOCAL_RANK=$DMLC_LOCAL_RANK; ')


def detect_flavor() -> str:
    try:
        out = subprocess.run(["mpirun", "--version"], capture_output=True, text=True).stdout
    except OSError:
        return "none"
    return "openmpi" if "Open MPI" in out or "OpenRTE" in out else "mpich"


def build_command(flavor: str, nproc: int, role: str, envs: Dict[str, object], cmd: str,
                  host_file=None, gpus_per_node: int = 0) -> List[str]:
    env = {k: str(v) for k, v in envs.items()}
    env.update({"DMLC_ROLE": role, "DMLC_JOB_CLUSTER": "mpi"})
    argv = ["mpirun", "-n", str(nproc)]
    if host_file:
        argv += ["--hostfile" if flavor == "openmpi" else "-f", host_file]
    for k, v in sorted(env.items()):
        if flavor == "openmpi":
            argv += ["-x", f"{k}={v}"]
        else:
            argv += ["-env", k, v]
    body = (LOCAL_RANK_SNIPPET if gpus_per_node and role == "worker" else "") + cmd
    return argv + ["bash", "-c", body]


def submit(args):
    cmd = " ".join(args.command)
    flavor = detect_flavor() if not args.dry_run else "openmpi"

    def launch(nworker, nserver, envs):
        envs = dict(envs)
        envs.update(user_envs(args))
        jobs = [("worker", nworker)] + ([("server", nserver)] if nserver else [])
        cmds = [build_command(flavor, n, role, envs, cmd, args.host_file, args.gpus_per_node)
                for role, n in jobs]
        if args.dry_run:
            for c in cmds:
                print(" ".join(c))
            return
        threads = [threading.Thread(target=subprocess.check_call, args=(c,), daemon=True)
                   for c in cmds]
        for t in threads:
            t.start()
        for t in threads:
            t.join()

    if args.dry_run:
        launch(args.num_workers, args.num_servers, {"DMLC_NUM_WORKER": args.num_workers,
                                                    "DMLC_NUM_SERVER": args.num_servers})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch, host_ip=args.host_ip or "auto",
                   pscmd=cmd, timeout=args.timeout, heartbeat_timeout=args.heartbeat_timeout)
    return 0
