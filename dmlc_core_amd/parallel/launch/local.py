"""Local backend: every task is a child process of this host
(reference `tracker/dmlc_tracker/local.py:12-72`).

Differences from the reference: ``DMLC_NUM_ATTEMPT`` is an integer retry
budget (the reference decrements a string, §7.4 #7); workers start before
servers consistently; with ``--gpus-per-node`` each worker gets
``DMLC_LOCAL_RANK`` (and ``LOCAL_RANK``) = its local index so it binds its
own MI355X; ``--torch-env`` also exports the torch.distributed rendezvous
(RANK = task index, MASTER_ADDR = 127.0.0.1) so the same processes can
build an RCCL process group.
"""
from __future__ import annotations

import logging
import os
import socket
import subprocess
import threading
from typing import Dict, List

from .. import tracker
from .opts import user_envs

logger = logging.getLogger("dmlc.submit.local")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def task_envs(args, envs: Dict[str, object], role: str, task_id: int, nworker: int,
              master_port: int) -> Dict[str, str]:
    env = {k: str(v) for k, v in envs.items()}
    env.update({"DMLC_TASK_ID": str(task_id), "DMLC_ROLE": role, "DMLC_JOB_CLUSTER": "local"})
    if role == "worker":
        # ranks sharing this host (per-host budgets, e.g. the zero-copy pin budget)
        env["DMLC_LOCAL_WORLD_SIZE"] = str(nworker)
        if args.gpus_per_node:
            local = task_id % args.gpus_per_node
            env["DMLC_LOCAL_RANK"] = str(local)
            env["LOCAL_RANK"] = str(local)
        if args.torch_env:
            env.update({"RANK": str(task_id), "WORLD_SIZE": str(nworker),
                        "LOCAL_WORLD_SIZE": str(args.gpus_per_node or nworker),
                        "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(master_port)})
            env.setdefault("LOCAL_RANK", str(task_id))
    env.update(user_envs(args))
    return env


def run_task(cmd: str, env: Dict[str, str], results: List[int], slot: int) -> None:
    full = os.environ.copy()
    full.update(env)
    attempts = int(full.get("DMLC_NUM_ATTEMPT", "0"))
    while True:
        ret = subprocess.call(cmd, shell=True, env=full)
        if ret == 0:
            break
        if attempts <= 0:
            logger.error("task %s exited with %d", env.get("DMLC_TASK_ID"), ret)
            break
        attempts -= 1
        full["DMLC_NUM_ATTEMPT"] = str(attempts)
        logger.warning("task %s failed (%d), %d attempt(s) left", env.get("DMLC_TASK_ID"),
                       ret, attempts)
    results[slot] = ret


def submit(args):
    cmd = " ".join(args.command)
    master_port = _free_port()
    failures: List[int] = []

    def launch(nworker: int, nserver: int, envs: Dict[str, object]) -> None:
        plan = [("worker", i) for i in range(nworker)] + [("server", i) for i in range(nserver)]
        if args.dry_run:
            for role, i in plan:
                e = task_envs(args, envs, role, i, nworker, master_port)
                print(" ".join(f"{k}={v}" for k, v in sorted(e.items())), cmd)
            return
        results = [0] * len(plan)
        threads = []
        for slot, (role, i) in enumerate(plan):
            e = task_envs(args, envs, role, i, nworker, master_port)
            t = threading.Thread(target=run_task, args=(cmd, e, results, slot), daemon=True)
            t.start()
            threads.append(t)
        for t in threads:
            t.join()
        failures.extend(r for r in results if r != 0)

    if args.dry_run:
        launch(args.num_workers, args.num_servers,
               {"DMLC_NUM_WORKER": args.num_workers, "DMLC_NUM_SERVER": args.num_servers,
                "DMLC_TRACKER_URI": "<tracker>", "DMLC_TRACKER_PORT": "<port>"})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch,
                   host_ip=args.host_ip or "127.0.0.1", pscmd=cmd, timeout=args.timeout,
                   heartbeat_timeout=args.heartbeat_timeout)
    if failures:
        raise SystemExit(f"{len(failures)} task(s) failed")
    return 0
