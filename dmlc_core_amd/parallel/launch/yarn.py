"""YARN backend, client side (reference `tracker/dmlc_tracker/yarn.py:16-129`
and `tracker/yarn/src/main/java/org/apache/hadoop/yarn/dmlc/Client.java`).

The reference submits through its own Java ApplicationMaster
(``hadoop jar dmlc-yarn.jar org.apache.hadoop.yarn.dmlc.Client``).  This
backend needs no JVM and no jar: the ResourceManager's YARN Services REST API
(``$YARN_RM_ADDRESS``, Hadoop >= 3.1) runs the containers and the AM's
per-task policy runs here, in `YarnServiceJob.wait`.  One component per
  role, one container per task; with ``--gpus-per-node`` every worker
  container asks for one ``amd.com/gpu`` (one process per GPU) and binds
  local rank 0.  Each container exports its own ``DMLC_TASK_ID`` /
  ``DMLC_WORKER_ID`` (or ``DMLC_SERVER_ID``) from the service's
  ``${COMPONENT_ID}``, ``DMLC_NODE_HOST``, and ``DMLC_NUM_ATTEMPT`` (the
  tracker's launch count of that task id, `dmlc_core_amd.parallel.attempt`).
  `YarnServiceJob.wait` applies the dmlc ApplicationMaster's policy to the
  containers the service reports (simulated end to end in
  `tests/yarn_am_sim.py`): a memory-limit kill aborts the job, other failures
  are retried by YARN up to DMLC_MAX_ATTEMPT, and more than that aborts.
  The node of every failed container is blacklisted (the service AM is asked
  to with ``yarn.service.node-blacklist.threshold`` = 1, and a task re-placed
  on such a node counts as a failed attempt).
  ``--files`` / ``--archives`` (and auto-cached command files) are uploaded
  through the WebHDFS backend to ``$DMLC_YARN_STAGING/<job>/`` and localised
  in the spec (`stage_files`), as the reference Client does with -file /
  -archive.
"""
from __future__ import annotations

import json
import os
import time
import urllib.error
import urllib.request
from typing import Dict, List, Optional

from .. import tracker
from .opts import get_cache_file_set, user_envs


def _mb(s) -> int:
    s = str(s).strip().lower()
    mult = {"g": 1024, "m": 1, "t": 1024 * 1024}.get(s[-1:], None)
    return int(float(s[:-1]) * mult) if mult else int(s)


_MEMORY_KILL = ("beyond physical memory", "beyond virtual memory",
                "exceeding allocated physical", "exceeding allocated virtual")


def staging_root(args) -> Optional[str]:
    """Where -file / -archive payloads are staged for the service containers:
    ``$DMLC_YARN_STAGING`` (any writable dmlc URI, e.g.
    ``webhdfs://nn:9870/user/me/.dmlc``), else ``--hdfs-tempdir`` on the
    WebHDFS endpoint ``$DMLC_WEBHDFS_ENDPOINT``."""
    root = os.environ.get("DMLC_YARN_STAGING", "")
    if root:
        return root.rstrip("/")
    ep = os.environ.get("DMLC_WEBHDFS_ENDPOINT", "")
    if ep:
        ep = ep.split("://", 1)[-1].rstrip("/")
        return f"webhdfs://{ep}/{args.hdfs_tempdir.strip('/')}"
    return None


def _cluster_path(uri: str) -> str:
    """webhdfs://host:port/a/b -> /a/b (the path YARN resolves on its default FS)."""
    if "://" not in uri:
        return uri
    rest = uri.split("://", 1)[1]
    return "/" + rest.split("/", 1)[1] if "/" in rest else "/"


def stage_files(args, name: str, upload: bool = True) -> List[dict]:
    """Ship the job's files like the reference Client (`Client.java:122-160`:
    copy every -file / -archive into the job's HDFS temp dir and localise it
    in each container): upload them through the native filesystem layer (the
    WebHDFS backend, no JVM) under ``<staging>/<name>/`` and return the YARN
    Services ``configuration.files`` entries -- STATIC for files, ARCHIVE
    (unpacked into a directory of the same name) for archives."""
    fset, _ = get_cache_file_set(args)
    items = [(f, "STATIC") for f in sorted(fset)] + [(a, "ARCHIVE") for a in args.archives]
    if not items:
        return []
    root = staging_root(args)
    if root is None:
        raise SystemExit("YARN services submission ships files through HDFS: set DMLC_YARN_STAGING "
                         "(e.g. webhdfs://namenode:9870/user/<me>/.dmlc) or DMLC_WEBHDFS_ENDPOINT")
    entries = []
    for local, kind in items:
        base = os.path.basename(local.rstrip("/"))
        dst = f"{root}/{name}/{base}"
        if upload:
            from ... import io as dio
            out = dio.Stream(dst, "w")
            with open(local, "rb") as f:
                while True:
                    buf = f.read(16 << 20)
                    if not buf:
                        break
                    out.write(buf)
            out.close()
        entries.append({"type": kind, "src_file": _cluster_path(dst), "dest_file": base})
    return entries


def service_spec(args, envs: Dict[str, object], name: str,
                 files: Optional[List[dict]] = None) -> dict:
    """YARN Services spec: a `worker` (and `server`) component, one container
    per task, restart on failure up to DMLC_MAX_ATTEMPT - 1 times; `files`
    (from `stage_files`) are localised into every container."""
    _, cmd = get_cache_file_set(args)
    max_attempt = int(os.environ.get("DMLC_MAX_ATTEMPT", "3"))
    env = {k: str(v) for k, v in envs.items()}
    env.update({k: str(v) for k, v in user_envs(args).items()})
    env.update({"DMLC_JOB_CLUSTER": "yarn", "DMLC_NUM_WORKER": str(args.num_workers),
                "DMLC_NUM_SERVER": str(args.num_servers),
                "DMLC_JOB_ARCHIVES": ":".join(os.path.basename(a) for a in args.archives)})
    comps = []
    for role, n, cores, mem in (("worker", args.num_workers, args.worker_cores, args.worker_memory),
                                ("server", args.num_servers, args.server_cores, args.server_memory)):
        if n <= 0:
            continue
        res = {"cpus": int(cores), "memory": str(_mb(mem))}
        gpu = role == "worker" and bool(getattr(args, "gpus_per_node", 0))
        if gpu:
            # one rank per container, so one GPU per container (YARN isolates
            # it: the container sees it as device 0); --gpus-per-node only
            # says that GPU workers are wanted, never N GPUs for one rank
            res["additional"] = {"amd.com/gpu": {"value": 1}}
        # per-container identity, as the dmlc AM gives each launch
        # (reference ApplicationMaster.java:443-446): the service expands
        # ${COMPONENT_ID} to the instance index (0..n-1) in the launch command;
        # servers follow the workers in task-id space, like the tracker's ranks
        base = 0 if role == "worker" else int(args.num_workers)
        # a relaunched container (restart_policy ON_FAILURE) keeps its
        # instance: its attempt number comes from the tracker's launch count
        # of that task id (dmlc_core_amd.parallel.attempt; 0 without one)
        ident = (f"export DMLC_TASK_ID=$(( ${{COMPONENT_ID}} + {base} )) "
                 f"DMLC_{role.upper()}_ID=${{COMPONENT_ID}} DMLC_NODE_HOST=$(hostname -f); "
                 "export DMLC_NUM_ATTEMPT=$(python3 -m dmlc_core_amd.parallel.attempt "
                 "2>/dev/null || echo 0); "
                 + ("export DMLC_LOCAL_RANK=0 LOCAL_RANK=0 LOCAL_WORLD_SIZE=1; " if gpu else ""))
        comps.append({
            "name": role, "number_of_containers": int(n), "launch_command": ident + cmd,
            "resource": res, "restart_policy": "ON_FAILURE",
            "configuration": {
                "env": dict(env, DMLC_ROLE=role),
                "properties": {
                    "yarn.service.container-failure.retry.max": str(max_attempt - 1),
                    # the dmlc AM blacklists the node of every failed container
                    # (reference ApplicationMaster.java:511-617, updateBlacklist
                    # on each failure): the service AM does it after 1 failure
                    "yarn.service.node-blacklist.threshold": "1"},
                "files": [dict(f) for f in (files or [])]},
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

    @staticmethod
    def _host(c: dict) -> str:
        return str(c.get("bare_host") or c.get("hostname") or c.get("ip") or "")

    def wait(self, poll: float = 2.0, max_attempt: Optional[int] = None,
             timeout: Optional[float] = None) -> "tuple[bool, str]":
        """Poll until the service finishes.  (ok, diagnostics).

        The dmlc AM's policy over the containers the service reports: a
        memory-limit kill aborts; every failure counts an attempt of its task
        and blacklists its node (``self.blacklist``; the spec asks the service
        AM to exclude it, ``yarn.service.node-blacklist.threshold`` = 1); a
        task re-placed on a blacklisted node counts as one more failed attempt
        (the placement broke the policy); max_attempt attempts abort.

        Misplacement is judged at placement time: a container's host is
        checked against the blacklist as it stood before the poll in which
        the container first appears, so a healthy container whose node is
        blacklisted later (by another task's failure) is never penalised --
        as in the reference AM, which only blacklists on failure
        (ApplicationMaster.java:511-617)."""
        max_attempt = max_attempt or int(os.environ.get("DMLC_MAX_ATTEMPT", "3"))
        failures: Dict[str, int] = {}
        seen = set()  # failed / misplaced container ids already counted
        placed_bad: Dict[str, bool] = {}  # container id -> host blacklisted when first seen
        self.blacklist = set()
        deadline = None if timeout is None else time.monotonic() + timeout
        while True:
            st = self.status()
            state = st.get("state", "")
            before = set(self.blacklist)  # this poll's placements are judged against it
            for comp in st.get("components", []):
                for c in comp.get("containers", []):
                    key = f"{comp['name']}/{c.get('component_instance_name', c.get('id'))}"
                    host = self._host(c)
                    cid = c.get("id")
                    if cid not in placed_bad:
                        placed_bad[cid] = host in before
                    if (c.get("state") in ("RUNNING_BUT_UNREADY", "READY", "RUNNING")
                            and placed_bad[cid] and key in failures
                            and cid not in seen):
                        seen.add(c.get("id"))
                        failures[key] += 1
                        if failures[key] >= max_attempt:
                            self.kill()
                            return False, (f"[DMLC] Task {key} placed on blacklisted node {host} "
                                           f"after {failures[key]} attempts")
                        continue
                    if c.get("state") != "FAILED" or c.get("id") in seen:
                        continue
                    seen.add(c.get("id"))
                    if host:
                        self.blacklist.add(host)
                    diag = str(c.get("diagnostics", ""))
                    if any(m in diag for m in _MEMORY_KILL):
                        self.kill()
                        return False, (f"[DMLC] {comp['name']} container {c.get('id')} killed because of "
                                       f"exceeding allocated memory: {diag}")
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
    """--cluster yarn: the Services REST path (the only one; see the module
    docstring for why there is no ``hadoop jar`` mode)."""
    rm = os.environ.get("YARN_RM_ADDRESS", "")
    if not rm:
        raise SystemExit("--cluster yarn submits through the YARN Services REST API: set "
                         "YARN_RM_ADDRESS (e.g. http://resourcemanager:8088; Hadoop >= 3.1)")
    return submit_service(args, rm)


def submit_service(args, rm: str):
    """JVM-free path: the tracker runs here, tasks run in YARN service containers."""
    name = (args.jobname or "dmlc") + f"-{os.getpid()}"
    staged: List[dict] = []

    def launch(nworker, nserver, envs):
        if not staged:
            staged.extend(stage_files(args, name, upload=not args.dry_run))
        spec = service_spec(args, envs, name, staged)
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
