"""YARN backend, client side (reference `tracker/dmlc_tracker/yarn.py:16-129`
and `tracker/yarn/src/main/java/org/apache/hadoop/yarn/dmlc/Client.java`).

Two ways to reach a cluster:

* ``--yarn-app-dir DIR`` holding a ``dmlc-yarn.jar``: the reference-style
  ``hadoop jar ... org.apache.hadoop.yarn.dmlc.Client`` invocation with the
  resource env (DMLC_WORKER_CORES/MEMORY_MB, ...) and shipped files/archives.
* otherwise (no JVM needed on the submitting host): the ResourceManager's YARN
  Services REST API (``$YARN_RM_ADDRESS``, Hadoop >= 3.1).  One component per
  role, one container per task, ``yarn.amd.com/gpu``-style GPU resources when
  ``--gpus-per-node`` is set.  `YarnServiceJob.wait` applies the dmlc
  ApplicationMaster's policy to the containers the service reports
  (`yarn_am.py`): a memory-limit kill aborts the job, other failures are
  retried by YARN up to DMLC_MAX_ATTEMPT, and more than that aborts.
"""
from __future__ import annotations

import json
import os
import subprocess
import time
import urllib.error
import urllib.request
from typing import Dict, List, Optional

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


def _mb(s) -> int:
    s = str(s).strip().lower()
    mult = {"g": 1024, "m": 1, "t": 1024 * 1024}.get(s[-1:], None)
    return int(float(s[:-1]) * mult) if mult else int(s)


_MEMORY_KILL = ("beyond physical memory", "beyond virtual memory",
                "exceeding allocated physical", "exceeding allocated virtual")


def service_spec(args, envs: Dict[str, object], name: str) -> dict:
    """YARN Services spec: a `worker` (and `server`) component, one container
    per task, restart on failure up to DMLC_MAX_ATTEMPT - 1 times."""
    _, cmd = get_cache_file_set(args)
    max_attempt = int(os.environ.get("DMLC_MAX_ATTEMPT", "3"))
    env = {k: str(v) for k, v in envs.items()}
    env.update({k: str(v) for k, v in user_envs(args).items()})
    env.update({"DMLC_JOB_CLUSTER": "yarn", "DMLC_NUM_WORKER": str(args.num_workers),
                "DMLC_NUM_SERVER": str(args.num_servers)})
    comps = []
    for role, n, cores, mem in (("worker", args.num_workers, args.worker_cores, args.worker_memory),
                                ("server", args.num_servers, args.server_cores, args.server_memory)):
        if n <= 0:
            continue
        res = {"cpus": int(cores), "memory": str(_mb(mem))}
        if role == "worker" and getattr(args, "gpus_per_node", 0):
            res["additional"] = {"amd.com/gpu": {"value": int(args.gpus_per_node)}}
        comps.append({
            "name": role, "number_of_containers": int(n), "launch_command": cmd,
            "resource": res, "restart_policy": "ON_FAILURE",
            "configuration": {
                "env": dict(env, DMLC_ROLE=role),
                "properties": {"yarn.service.container-failure.retry.max": str(max_attempt - 1)}},
        })
    return {"name": name, "version": "1.0", "queue": args.queue, "components": comps}


class YarnServiceJob:
    """Submit / watch / kill one YARN service over the RM's REST API."""

    def __init__(self, rm: str, name: str, user: Optional[str] = None):
        self.base = rm.rstrip("/") + "/app/v1/services"
        self.name = name
        self.user = user or os.environ.get("HADOOP_USER_NAME") or os.environ.get("USER", "dmlc")

    def _call(self, method: str, path: str = "", body: Optional[dict] = None) -> dict:
        url = f"{self.base}{path}?user.name={self.user}"
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(url, data=data, method=method,
                                     headers={"Content-Type": "application/json"})
        try:
            with urllib.request.urlopen(req, timeout=60) as r:
                txt = r.read().decode() or "{}"
        except urllib.error.HTTPError as e:
            raise RuntimeError(f"YARN {method} {url}: HTTP {e.code} {e.read()[:300]!r}") from None
        return json.loads(txt)

    def submit(self, spec: dict) -> dict:
        return self._call("POST", "", spec)

    def status(self) -> dict:
        return self._call("GET", f"/{self.name}")

    def kill(self) -> None:
        self._call("DELETE", f"/{self.name}")

    def wait(self, poll: float = 2.0, max_attempt: Optional[int] = None,
             timeout: Optional[float] = None) -> "tuple[bool, str]":
        """Poll until the service finishes.  (ok, diagnostics)."""
        max_attempt = max_attempt or int(os.environ.get("DMLC_MAX_ATTEMPT", "3"))
        failures: Dict[str, int] = {}
        seen = set()  # failed container ids already counted
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            st = self.status()
            state = st.get("state", "")
            for comp in st.get("components", []):
                for c in comp.get("containers", []):
                    if c.get("state") != "FAILED" or c.get("id") in seen:
                        continue
                    seen.add(c.get("id"))
                    diag = str(c.get("diagnostics", ""))
                    if any(m in diag for m in _MEMORY_KILL):
                        self.kill()
                        return False, (f"[DMLC] {comp['name']} container {c.get('id')} killed because of "
                                       f"exceeding allocated memory: {diag}")
                    key = f"{comp['name']}/{c.get('component_instance_name', c.get('id'))}"
                    failures[key] = failures.get(key, 0) + 1
                    if failures[key] >= max_attempt:
                        self.kill()
                        return False, f"[DMLC] Task {key} failed more than {failures[key]} times"
            if state in ("SUCCEEDED", "STOPPED"):
                return True, state
            if state == "FAILED":
                return False, st.get("diagnostics", "service FAILED")
            if deadline is not None and time.monotonic() > deadline:
                self.kill()
                return False, "[DMLC] YARN service timed out"
            time.sleep(poll)


def submit(args):
    app_dir = args.yarn_app_dir or os.environ.get("DMLC_YARN_APP_DIR", "")
    jar = os.path.join(app_dir, "dmlc-yarn.jar")
    rm = os.environ.get("YARN_RM_ADDRESS", "")
    if rm and not os.path.exists(jar):
        return submit_service(args, rm)

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


def submit_service(args, rm: str):
    """JVM-free path: the tracker runs here, tasks run in YARN service containers."""
    name = (args.jobname or "dmlc") + f"-{os.getpid()}"

    def launch(nworker, nserver, envs):
        spec = service_spec(args, envs, name)
        if args.dry_run:
            print(json.dumps(spec, indent=1, sort_keys=True))
            return
        job = YarnServiceJob(rm, name)
        job.submit(spec)
        ok, diag = job.wait()
        if not ok:
            raise RuntimeError(diag)

    if args.dry_run:
        launch(args.num_workers, args.num_servers, {})
        return 0
    tracker.submit(args.num_workers, args.num_servers, launch, host_ip=args.host_ip or "auto",
                   pscmd=" ".join(args.command), timeout=args.timeout,
                   heartbeat_timeout=args.heartbeat_timeout)
    return 0
