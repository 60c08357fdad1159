"""Sun Grid Engine backend (reference `tracker/dmlc_tracker/sge.py:9-48`):
writes a ``rundmlc.sh`` wrapper and submits an array job ``qsub -t 1-N``;
the container launcher maps SGE_TASK_ID to DMLC_TASK_ID / role.  The
reference's undefined ``args.logdir`` / ``args.vcores`` are replaced by
``--sge-log-dir`` and ``--worker-cores`` (§7.4 #7).
"""
from __future__ import annotations

import os
import subprocess
import sys
from typing import Dict, List

from .. import tracker
from .opts import user_envs


def write_runscript(path: str, cmd: str) -> str:
    with open(path, "w") as f:
        f.write("#!/bin/bash\n")
        f.write(f"{sys.executable} -m dmlc_core_amd.parallel.launch.container {cmd}\n")
    os.chmod(path, 0o755)
    return path


def build_command(args, envs: Dict[str, object], ntask: int, script: str) -> List[str]:
    env = ",".join(f"{k}={v}" for k, v in sorted(envs.items()))
    logdir = args.sge_log_dir or os.path.join(os.getcwd(), "sge-log")
    argv = ["qsub", "-cwd", "-t", f"1-{ntask}", "-S", "/bin/bash", "-q", args.queue,
            "-N", args.jobname or "dmlc", "-o", logdir, "-e", logdir,
            "-pe", "orte", str(args.worker_cores), "-v", env + ",DMLC_JOB_CLUSTER=sge"]
    return argv + [script]


def submit(args):
    cmd = " ".join(args.command)

    def launch(nworker, nserver, envs):
        envs = dict(envs)
        envs.update(user_envs(args))
        script = os.path.join(os.getcwd(), "rundmlc.sh")
        c = build_command(args, envs, nworker + nserver, script)
        if args.dry_run:
            print(" ".join(c))
            return
        write_runscript(script, cmd)
        os.makedirs(args.sge_log_dir or os.path.join(os.getcwd(), "sge-log"), exist_ok=True)
        subprocess.check_call(c)

    if args.dry_run:
        launch(args.num_workers, args.num_servers, {"DMLC_NUM_WORKER": args.num_workers,
                                                    "DMLC_NUM_SERVER": args.num_servers})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch, host_ip=args.host_ip or "auto",
                   pscmd=cmd, timeout=args.timeout, heartbeat_timeout=args.heartbeat_timeout)
    return 0
