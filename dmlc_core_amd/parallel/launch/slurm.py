"""SLURM backend (reference `tracker/dmlc_tracker/slurm.py:20-65`): one srun
per role with ``--exclusive=user``; node counts default to task counts.
With ``--gpus-per-node`` it asks SLURM for that many GPUs per node
(``--gpus-per-node`` / ``--ntasks-per-node``) and every task binds
``SLURM_LOCALID``.
"""
from __future__ import annotations

import subprocess
import threading
from typing import Dict, List

from .. import tracker
from .opts import user_envs


def build_command(role: str, ntasks: int, nnodes: int, envs: Dict[str, object], cmd: str,
                  gpus_per_node: int = 0, jobname=None) -> List[str]:
    env = ",".join(["ALL"] + [f"{k}={v}" for k, v in sorted(envs.items())] +
                   [f"DMLC_ROLE={role}", "DMLC_JOB_CLUSTER=slurm"])
    argv = ["srun", "--share", "--exclusive=user", "-N", str(nnodes), "-n", str(ntasks),
            f"--export={env}"]
    if jobname:
        argv += ["-J", jobname]
    body = cmd
    if gpus_per_node and role == "worker":
        argv += [f"--gpus-per-node={gpus_per_node}", f"--ntasks-per-node={gpus_per_node}"]
        body = "export DMLC_LOCAL_RANK=$SLURM_LOCALID LOCAL_RANK=$SLURM_LOCALID; " + cmd
    return argv + ["bash", "-c", body]


def submit(args):
    cmd = " ".join(args.command)

    def launch(nworker, nserver, envs):
        envs = dict(envs)
        envs.update(user_envs(args))
        cmds = [build_command("worker", nworker, args.slurm_worker_nodes or
                              (max(1, -(-nworker // args.gpus_per_node)) if args.gpus_per_node
                               else nworker), envs, cmd, args.gpus_per_node, args.jobname)]
        if nserver:
            cmds.append(build_command("server", nserver, args.slurm_server_nodes or nserver,
                                      envs, cmd, 0, args.jobname))
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
