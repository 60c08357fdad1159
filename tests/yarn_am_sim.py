"""DMLC ApplicationMaster: task bookkeeping and failure policy for YARN jobs.

Behaviour of the reference ApplicationMaster
(`tracker/yarn/src/main/java/org/apache/hadoop/yarn/dmlc/ApplicationMaster.java`),
re-done in Python without a JVM:

* one task per worker/server (ids 0..n-1, servers after workers), each asking
  for a container with the role's vcores / memory (`DMLC_WORKER_CORES`,
  `DMLC_WORKER_MEMORY_MB`, ... `:200-213`);
* a task is launched with every `DMLC_*` variable of the AM plus
  `DMLC_NODE_HOST`, `DMLC_TASK_ID`, `DMLC_ROLE`, `DMLC_NUM_ATTEMPT` (`:425-447`);
* a container on a blacklisted node is handed back unused (`:482-503`);
* a container that exits non-zero is stopped, its node blacklisted and the task
  re-queued with `attempt += 1`; at `DMLC_MAX_ATTEMPT` (default 3) attempts the
  job aborts (`:536-570`);
* exit status KILLED_EXCEEDED_PMEM (-104) or KILLED_EXCEEDED_VMEM (-103) aborts
  the job at once: a memory-limit kill would repeat on any node (`:584-610`);
* abort stops every running container and moves pending tasks to killed; the
  final diagnostics are "num_tasks, finished, failed" plus the abort reason
  (`:270-283`, `:511-531`).

The container side is a small interface (`ContainerBackend`): the YARN
Services REST backend in `yarn.py` drives real clusters, `LocalContainerBackend`
runs tasks as local processes on named virtual nodes (tests, single host).
"""
from __future__ import annotations

import os
import subprocess
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional, Sequence, Tuple

SUCCESS = 0
KILLED_EXCEEDED_VMEM = -103
KILLED_EXCEEDED_PMEM = -104


@dataclass
class Container:
    id: str
    node: str


@dataclass
class TaskRecord:
    task_id: int
    role: str  # "worker" | "server"
    attempt: int = 0
    container: Optional[Container] = None
    abort_requested: bool = False


@dataclass
class Resource:
    vcores: int = 1
    memory_mb: int = 1024


class ContainerBackend:
    """What the AM needs from a cluster (the AMRMClient + NMClient pair)."""

    def request(self, role: str, res: Resource) -> None:
        """Ask for one more container of this shape."""
        raise NotImplementedError

    def release(self, c: Container) -> None:
        """Give back an allocated container that was never launched."""
        raise NotImplementedError

    def launch(self, c: Container, command: Sequence[str], env: Dict[str, str]) -> None:
        raise NotImplementedError

    def stop(self, c: Container) -> None:
        raise NotImplementedError

    def poll(self, timeout: float) -> Tuple[List[Container], List[Tuple[str, int, str]]]:
        """(newly allocated containers, completed (container id, exit status, diagnostics))."""
        raise NotImplementedError


@dataclass
class AMResult:
    success: bool
    finished: int
    failed: int
    diagnostics: str
    attempts: Dict[int, int] = field(default_factory=dict)
    blacklist: List[str] = field(default_factory=list)


class ApplicationMaster:
    def __init__(self, backend: ContainerBackend, command: Sequence[str],
                 num_worker: int, num_server: int = 0,
                 worker_res: Resource = Resource(), server_res: Resource = Resource(),
                 max_attempt: int = 3, env: Optional[Dict[str, str]] = None):
        self.backend = backend
        self.command = list(command)
        self.num_tasks = num_worker + num_server
        self.res = {"worker": worker_res, "server": server_res}
        self.max_attempt = max_attempt
        self.env = {k: v for k, v in (env if env is not None else os.environ).items()
                    if k.startswith("DMLC_")}
        self.pending: Deque[TaskRecord] = deque()
        self.running: Dict[str, TaskRecord] = {}
        self.finished: List[TaskRecord] = []
        self.killed: List[TaskRecord] = []
        self.blacklist: set = set()
        self.aborting = False
        self.abort_reason = ""
        self.lock = threading.Lock()
        tasks = [TaskRecord(i, "worker") for i in range(num_worker)]
        tasks += [TaskRecord(num_worker + i, "server") for i in range(num_server)]
        self._submit(tasks)

    @classmethod
    def from_env(cls, backend: ContainerBackend, command: Sequence[str],
                 env: Optional[Dict[str, str]] = None) -> "ApplicationMaster":
        e = env if env is not None else dict(os.environ)

        def geti(k, d):
            return int(e.get(k, d))
        return cls(backend, command, geti("DMLC_NUM_WORKER", 0), geti("DMLC_NUM_SERVER", 0),
                   Resource(geti("DMLC_WORKER_CORES", 1), geti("DMLC_WORKER_MEMORY_MB", 1024)),
                   Resource(geti("DMLC_SERVER_CORES", 1), geti("DMLC_SERVER_MEMORY_MB", 1024)),
                   geti("DMLC_MAX_ATTEMPT", 3), e)

    # ------------------------------------------------------------- bookkeeping
    def _submit(self, tasks: Sequence[TaskRecord]) -> None:
        for t in tasks:
            self.pending.append(t)
            self.backend.request(t.role, self.res[t.role])

    def done(self) -> bool:
        return not self.pending and not self.running

    def progress(self) -> float:
        return 1.0 - len(self.pending) / max(1, self.num_tasks)

    def on_allocated(self, containers: Sequence[Container]) -> None:
        with self.lock:
            for c in containers:
                if self.aborting:
                    self.backend.release(c)
                    continue
                if c.node in self.blacklist:
                    # hand it back and ask again for the task it was meant for
                    self.backend.release(c)
                    if self.pending:
                        self.backend.request(self.pending[0].role, self.res[self.pending[0].role])
                    continue
                if not self.pending:
                    self.backend.release(c)
                    continue
                t = self.pending.popleft()
                self._launch(c, t)

    def _launch(self, c: Container, t: TaskRecord) -> None:
        env = dict(self.env)
        env.update({"DMLC_NODE_HOST": c.node, "DMLC_TASK_ID": str(t.task_id),
                    "DMLC_ROLE": t.role, "DMLC_NUM_ATTEMPT": str(t.attempt)})
        t.container = c
        self.running[c.id] = t
        self.backend.launch(c, self.command, env)

    def abort(self, msg: str) -> None:
        if not self.aborting:
            self.abort_reason = msg
        self.aborting = True
        for t in self.running.values():
            if not t.abort_requested:
                self.backend.stop(t.container)
                t.abort_requested = True
                self.killed.append(t)
        self.killed.extend(self.pending)
        self.pending.clear()
        self.running.clear()

    def on_completed(self, statuses: Sequence[Tuple[str, int, str]]) -> None:
        with self.lock:
            failed = []
            for cid, status, diag in statuses:
                t = self.running.get(cid)
                if t is None:
                    continue
                if status == SUCCESS:
                    self.finished.append(self.running.pop(cid))
                    continue
                if status == KILLED_EXCEEDED_PMEM:
                    self.abort(f"[DMLC] Task {t.task_id} killed because of exceeding allocated "
                               "physical memory")
                    return
                if status == KILLED_EXCEEDED_VMEM:
                    self.abort(f"[DMLC] Task {t.task_id} killed because of exceeding allocated "
                               "virtual memory")
                    return
                failed.append((cid, status, diag))
            retry = []
            for cid, status, diag in failed:
                t = self.running.pop(cid, None)
                if t is None:
                    continue
                t.attempt += 1
                self.backend.stop(t.container)
                self.blacklist.add(t.container.node)
                t.container = None
                retry.append(t)
                if t.attempt >= self.max_attempt:
                    self.abort(f"[DMLC] Task {t.task_id} failed more than {t.attempt} times "
                               f"(last exit status {status}: {diag})")
            if self.aborting:
                self.killed.extend(retry)
            else:
                self._submit(retry)

    # -------------------------------------------------------------------- loop
    def run(self, poll_sec: float = 0.05, timeout: Optional[float] = None) -> AMResult:
        deadline = None if timeout is None else time.monotonic() + timeout
        while not self.done():
            if deadline is not None and time.monotonic() > deadline:
                with self.lock:
                    self.abort("[DMLC] ApplicationMaster timed out")
                break
            alloc, done = self.backend.poll(poll_sec)
            if alloc:
                self.on_allocated(alloc)
            if done:
                self.on_completed(done)
        ok = not self.aborting and len(self.finished) == self.num_tasks
        diag = (f"Diagnostics., num_tasks{self.num_tasks}, finished={len(self.finished)}, "
                f"failed={len(self.killed)}\n{self.abort_reason}")
        attempts = {t.task_id: t.attempt for t in self.finished + self.killed}
        return AMResult(ok, len(self.finished), len(self.killed), diag, attempts,
                        sorted(self.blacklist))


class LocalContainerBackend(ContainerBackend):
    """Containers as local processes, allocated round-robin over virtual node
    names.  `fail_nodes` maps a node name to the exit status every container
    there reports (tests: a bad node, a memory-limit kill) without running."""

    def __init__(self, nodes: Sequence[str] = ("node0",), fail_nodes: Optional[Dict[str, int]] = None,
                 cwd: Optional[str] = None):
        self.nodes = list(nodes)
        self.fail_nodes = dict(fail_nodes or {})
        self.cwd = cwd
        self.next_node = 0
        self.seq = 0
        self.requests: Deque[str] = deque()
        self.procs: Dict[str, subprocess.Popen] = {}
        self.fake_done: List[Tuple[str, int, str]] = []
        self.launched: List[Tuple[str, str, Dict[str, str]]] = []  # (container, node, env)
        self.released: List[str] = []

    def request(self, role, res):
        self.requests.append(role)

    def release(self, c):
        self.released.append(c.id)

    def launch(self, c, command, env):
        self.launched.append((c.id, c.node, dict(env)))
        if c.node in self.fail_nodes:
            self.fake_done.append((c.id, self.fail_nodes[c.node], f"injected failure on {c.node}"))
            return
        full = dict(os.environ)
        full.update(env)
        self.procs[c.id] = subprocess.Popen(list(command), env=full, cwd=self.cwd,
                                            stdout=subprocess.DEVNULL, stderr=subprocess.PIPE)

    def stop(self, c):
        p = self.procs.pop(c.id, None)
        if p is not None and p.poll() is None:
            p.kill()
            p.wait()

    def poll(self, timeout):
        alloc = []
        while self.requests:
            self.requests.popleft()
            node = self.nodes[self.next_node % len(self.nodes)]
            self.next_node += 1
            alloc.append(Container(f"container_{self.seq:06d}", node))
            self.seq += 1
        done, self.fake_done = self.fake_done, []
        end = time.monotonic() + timeout
        while True:
            for cid, p in list(self.procs.items()):
                rc = p.poll()
                if rc is not None:
                    err = p.stderr.read().decode(errors="replace")[-500:] if p.stderr else ""
                    del self.procs[cid]
                    done.append((cid, rc, err))
            if alloc or done or time.monotonic() >= end:
                return alloc, done
            time.sleep(min(0.01, timeout))
