"""Command-line options of dmlc-submit (reference `tracker/dmlc_tracker/opts.py:60-178`).

Same flags as the reference plus MI355X-specific ones: ``--gpus-per-node``
(one process per GPU, bound by local index), ``--torch-env`` (export
RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* for torch.distributed over RCCL),
``--timeout`` / ``--heartbeat-timeout`` for the tracker, ``--dry-run``.
"""
from __future__ import annotations

import argparse
import os

from . import BACKENDS


def get_memory_mb(mem_str: str) -> int:
    """'4g' -> 4096, '512m' -> 512, '2048' -> 2048 (MB)."""
    s = str(mem_str).strip().lower()
    if s.endswith("g"):
        return int(float(s[:-1]) * 1024)
    if s.endswith("m"):
        return int(float(s[:-1]))
    return int(s)


def get_cache_file_set(args):
    """Files referenced in the command that should ship with the job
    (reference opts.py:8-40): every existing local path among the command
    tokens when --auto-file-cache is on, plus --files.  The command is
    rewritten to refer to the shipped basename."""
    fset = set(args.files)
    cmds = []
    for tok in args.command:
        if args.auto_file_cache and os.path.exists(tok) and os.path.isfile(tok):
            fset.add(tok)
            cmds.append("./" + os.path.basename(tok))
        else:
            cmds.append(tok)
    return fset, " ".join(cmds)


def _bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="DMLC job submission (MI355X build)", allow_abbrev=False)
    p.add_argument("--cluster", type=str, choices=BACKENDS,
                   help="cluster backend; defaults to ${DMLC_SUBMIT_CLUSTER}")
    p.add_argument("--num-workers", required=True, type=int)
    p.add_argument("--worker-cores", default=1, type=int)
    p.add_argument("--worker-memory", default="1g", type=str)
    p.add_argument("--num-servers", default=0, type=int)
    p.add_argument("--server-cores", default=1, type=int)
    p.add_argument("--server-memory", default="1g", type=str)
    p.add_argument("--jobname", default=None, type=str)
    p.add_argument("--queue", default="default", type=str)
    p.add_argument("--log-level", default="INFO", choices=["INFO", "DEBUG"])
    p.add_argument("--log-file", default=None, type=str)
    p.add_argument("--host-ip", default=None, type=str)
    p.add_argument("--hdfs-tempdir", default="/tmp", type=str)
    p.add_argument("--host-file", default=None, type=str)
    p.add_argument("--sge-log-dir", default=None, type=str)
    p.add_argument("--auto-file-cache", default=True, type=_bool)
    p.add_argument("--files", default=[], action="append")
    p.add_argument("--archives", default=[], action="append")
    p.add_argument("--env", default=[], action="append",
                   help="KEY=VALUE exported to every task (repeatable)")
    p.add_argument("--yarn-app-classpath", type=str, default=None)
    p.add_argument("--mesos-master", type=str, default=None)
    p.add_argument("--ship-libcxx", default=None, type=str)
    p.add_argument("--sync-dst-dir", type=str, default=None)
    p.add_argument("--slurm-worker-nodes", default=None, type=int)
    p.add_argument("--slurm-server-nodes", default=None, type=int)
    p.add_argument("--kube-namespace", default="default", type=str)
    p.add_argument("--kube-worker-image", default="rocm/pytorch", type=str)
    p.add_argument("--kube-server-image", default="rocm/pytorch", type=str)
    p.add_argument("--kube-worker-template", default=None, type=str)
    p.add_argument("--kube-server-template", default=None, type=str)
    p.add_argument("--kube-pod-per-rank", default=False, type=_bool,
                   help="kubernetes + --gpus-per-node: one pod (1 GPU) per rank instead of "
                        "one pod per node running --gpus-per-node ranks")
    # MI355X additions
    p.add_argument("--gpus-per-node", default=0, type=int,
                   help="bind one process per GPU (DMLC_LOCAL_RANK = local index)")
    p.add_argument("--torch-env", default=False, type=_bool,
                   help="export RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT")
    p.add_argument("--timeout", default=None, type=float, help="tracker job timeout (s)")
    p.add_argument("--heartbeat-timeout", default=None, type=float)
    p.add_argument("--dry-run", action="store_true", help="print the launch commands only")
    # everything from the first positional token on is the task's command,
    # verbatim (its own --options included), as with the reference's
    # parse_known_args + `command += unknown` (tracker/dmlc_tracker/opts.py:142-166)
    p.add_argument("command", nargs=argparse.REMAINDER, help="command to run on every task")
    return p


def get_opts(argv=None):
    args, unknown = build_parser().parse_known_args(argv)
    args.command = list(args.command) + unknown
    if not args.command:
        raise SystemExit("dmlc-submit: no command given")
    if args.cluster is None:
        args.cluster = os.environ.get("DMLC_SUBMIT_CLUSTER")
        if args.cluster is None:
            raise SystemExit("--cluster is not set and DMLC_SUBMIT_CLUSTER is empty")
    args.worker_memory_mb = get_memory_mb(args.worker_memory)
    args.server_memory_mb = get_memory_mb(args.server_memory)
    return args


def user_envs(args) -> dict:
    out = {}
    for kv in args.env:
        k, _, v = kv.partition("=")
        if not k:
            raise SystemExit(f"--env expects KEY=VALUE, got {kv!r}")
        out[k] = v
    return out
