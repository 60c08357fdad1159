"""SSH backend (reference `tracker/dmlc_tracker/ssh.py:13-86`): hosts from
``--host-file`` (``ip[:port]`` per line), optional rsync of the working
directory to ``--sync-dst-dir``, round-robin task placement, forwarded
OMP/LD_LIBRARY_PATH/AWS/DMLC_INTERFACE env.  Workers are placed before
servers (the reference did servers first, §7.4 #7), and it is wired into
the dispatch (the reference accepted ``--cluster ssh`` but never ran it).
With ``--gpus-per-node``, DMLC_LOCAL_RANK = index of the task on its host.
"""
from __future__ import annotations

import os
import shlex
import subprocess
import threading
from typing import Dict, List, Tuple

from .. import tracker
from .opts import user_envs

FORWARD = ("OMP_NUM_THREADS", "KMP_AFFINITY", "LD_LIBRARY_PATH", "AWS_ACCESS_KEY_ID",
           "AWS_SECRET_ACCESS_KEY", "AWS_SESSION_TOKEN", "DMLC_INTERFACE",
           "HSA_ENABLE_IPC_MODE_LEGACY", "NCCL_SOCKET_IFNAME", "RCCL_MSCCL_ENABLE")


def read_hosts(path: str) -> List[Tuple[str, int]]:
    hosts = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            host, _, port = line.partition(":")
            hosts.append((host, int(port) if port else 22))
    if not hosts:
        raise SystemExit(f"no hosts in {path}")
    return hosts


def plan_tasks(hosts, nworker: int, nserver: int, gpus_per_node: int = 0):
    """[(host, port, role, task_id, local_index)] with round-robin placement."""
    plan, per_host = [], {}
    roles = [("worker", i) for i in range(nworker)] + [("server", i) for i in range(nserver)]
    for k, (role, tid) in enumerate(roles):
        host, port = hosts[k % len(hosts)]
        local = per_host.get(host, 0)
        per_host[host] = local + 1
        plan.append((host, port, role, tid, local))
    return plan


def build_command(host: str, port: int, env: Dict[str, str], cmd: str, workdir: str) -> List[str]:
    exports = " ".join(f"export {k}={shlex.quote(v)};" for k, v in sorted(env.items()))
    remote = f"{exports} cd {shlex.quote(workdir)}; {cmd}"
    return ["ssh", "-o", "StrictHostKeyChecking=no", host, "-p", str(port), remote]


def submit(args):
    if args.host_file is None:
        raise SystemExit("--host-file is required for --cluster ssh")
    hosts = read_hosts(args.host_file)
    cmd = " ".join(args.command)
    workdir = args.sync_dst_dir or os.getcwd()

    def launch(nworker, nserver, envs):
        base = {k: str(v) for k, v in envs.items()}
        base.update({k: os.environ[k] for k in FORWARD if k in os.environ})
        base.update(user_envs(args))
        if args.sync_dst_dir and not args.dry_run:
            for host, port in sorted(set(hosts)):
                subprocess.check_call(["rsync", "-az", "--rsh", f"ssh -o StrictHostKeyChecking=no -p {port}",
                                       os.getcwd() + "/", f"{host}:{args.sync_dst_dir}"])
        cmds = []
        for host, port, role, tid, local in plan_tasks(hosts, nworker, nserver, args.gpus_per_node):
            env = dict(base, DMLC_ROLE=role, DMLC_TASK_ID=str(tid), DMLC_JOB_CLUSTER="ssh")
            if args.gpus_per_node and role == "worker":
                env["DMLC_LOCAL_RANK"] = env["LOCAL_RANK"] = str(local % args.gpus_per_node)
            cmds.append(build_command(host, port, env, cmd, workdir))
        if args.dry_run:
            for c in cmds:
                print(" ".join(shlex.quote(x) for x in c))
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
