"""Mesos backend (reference `tracker/dmlc_tracker/mesos.py:16-104`): uses
``pymesos.subprocess`` when importable, otherwise ``mesos-execute`` per task;
per-task cpus/mem and DMLC_WORKER_ID / DMLC_SERVER_ID.  Imported lazily so
dmlc-submit works without pymesos.
"""
from __future__ import annotations

import os
import subprocess
import threading
from typing import Dict, List

from .. import tracker
from .opts import user_envs


def build_command(master: str, name: str, role: str, tid: int, env: Dict[str, object],
                  cmd: str, cpus: int, mem_mb: int) -> List[str]:
    e = {k: str(v) for k, v in env.items()}
    e.update({"DMLC_ROLE": role, "DMLC_JOB_CLUSTER": "mesos",
              ("DMLC_WORKER_ID" if role == "worker" else "DMLC_SERVER_ID"): str(tid)})
    exports = "; ".join(f"export {k}={v}" for k, v in sorted(e.items()))
    return ["mesos-execute", f"--master={master}", f"--name={name}-{role}-{tid}",
            f"--resources=cpus:{cpus};mem:{mem_mb}", f"--command={exports}; {cmd}"]


def submit(args):
    master = args.mesos_master or os.environ.get("MESOS_MASTER", "")
    if not master and not args.dry_run:
        raise SystemExit("--mesos-master or MESOS_MASTER is required")
    cmd = " ".join(args.command)

    def launch(nworker, nserver, envs):
        envs = dict(envs)
        envs.update(user_envs(args))
        tasks = [("worker", i, args.worker_cores, args.worker_memory_mb) for i in range(nworker)]
        tasks += [("server", i, args.server_cores, args.server_memory_mb) for i in range(nserver)]
        cmds = [build_command(master, args.jobname or "dmlc", r, i, envs, cmd, c, m)
                for r, i, c, m in tasks]
        if args.dry_run:
            for c in cmds:
                print(" ".join(c))
            return
        try:
            import pymesos.subprocess  # noqa: F401  (optional dependency)
        except ImportError:
            pass
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
