"""YARN backend, client side (reference `tracker/dmlc_tracker/yarn.py:16-129`).

Builds the ``hadoop jar dmlc-yarn.jar org.apache.hadoop.yarn.dmlc.Client``
invocation with the resource env (DMLC_WORKER_CORES/MEMORY_MB, ...) and the
shipped files/archives.  The ApplicationMaster jar is not bundled with this
MI355X build (YARN is rarely the scheduler of GPU nodes); point
``--yarn-app-dir`` at a directory holding ``dmlc-yarn.jar``.
"""
from __future__ import annotations

import os
import subprocess
from typing import Dict, List

from .. import tracker
from .opts import get_cache_file_set, user_envs


def hadoop_version() -> List[int]:
    out = subprocess.run(["hadoop", "version"], capture_output=True, text=True).stdout
    first = out.splitlines()[0] if out else ""
    return [int(x) for x in first.split()[-1].split(".")[:2]] if first else [0, 0]


def build_command(args, envs: Dict[str, object], jar: str) -> List[str]:
    fset, cmd = get_cache_file_set(args)
    env = dict(envs)
    env.update({"DMLC_JOB_CLUSTER": "yarn", "DMLC_WORKER_CORES": args.worker_cores,
                "DMLC_WORKER_MEMORY_MB": args.worker_memory_mb,
                "DMLC_SERVER_CORES": args.server_cores,
                "DMLC_SERVER_MEMORY_MB": args.server_memory_mb,
                "DMLC_NUM_WORKER": args.num_workers, "DMLC_NUM_SERVER": args.num_servers,
                "DMLC_JOB_ARCHIVES": ":".join(args.archives)})
    env.update(user_envs(args))
    argv = ["hadoop", "jar", jar, "org.apache.hadoop.yarn.dmlc.Client"]
    for f in sorted(fset):
        argv += ["-file", f]
    for a in args.archives:
        argv += ["-archive", a]
    argv += ["-jobname", args.jobname or "dmlc", "-tempdir", args.hdfs_tempdir,
             "-queue", args.queue]
    for k, v in sorted(env.items()):
        argv += ["-env", f"{k}={v}"]
    return argv + ["./launcher.sh", cmd]


def submit(args):
    app_dir = args.yarn_app_dir or os.environ.get("DMLC_YARN_APP_DIR", "")
    jar = os.path.join(app_dir, "dmlc-yarn.jar")

    def launch(nworker, nserver, envs):
        c = build_command(args, envs, jar)
        if args.dry_run:
            print(" ".join(c))
            return
        if not os.path.exists(jar):
            raise SystemExit(f"{jar} not found: build the YARN ApplicationMaster jar and pass "
                             "--yarn-app-dir")
        if hadoop_version()[0] < 2:
            raise SystemExit("YARN backend needs Hadoop >= 2")
        subprocess.check_call(c)

    if args.dry_run:
        launch(args.num_workers, args.num_servers, {})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch, host_ip=args.host_ip or "auto",
                   pscmd=" ".join(args.command), timeout=args.timeout,
                   heartbeat_timeout=args.heartbeat_timeout)
    return 0
