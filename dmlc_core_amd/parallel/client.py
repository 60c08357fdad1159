"""Worker side of the tracker protocol (Python twin of the C++
``dmlc::dist::TrackerClient`` in src/dist/tracker_client.cc).

Every command is one short TCP connection: handshake (magic, rank,
world_size, jobid, cmd) followed by the command body, exactly as rabit
workers talk to the reference tracker.  The data
plane is RCCL, so the worker reports every topology link as already
established: the tracker then brokers no TCP peer connections.
"""
from __future__ import annotations

import os
import socket
import threading
from dataclasses import dataclass, field
from typing import Callable, List, Optional

from .tracker import MAGIC, Channel


@dataclass
class Topology:
    rank: int
    parent: int
    world_size: int
    tree: List[int] = field(default_factory=list)
    ring_prev: int = -1
    ring_next: int = -1


class TrackerClient:
    def __init__(self, uri: Optional[str] = None, port: Optional[int] = None,
                 jobid: Optional[str] = None, rank: int = -1, world_size: int = -1,
                 timeout: float = 600.0):
        self.uri = uri or os.environ.get("DMLC_TRACKER_URI", "127.0.0.1")
        self.port = int(port or os.environ.get("DMLC_TRACKER_PORT", 9091))
        self.jobid = jobid or os.environ.get("DMLC_TASK_ID", "NULL")
        self.rank = rank
        self.world_size = world_size
        self.timeout = timeout
        self.topology: Optional[Topology] = None
        self._hb_stop: Optional[threading.Event] = None

    def _connect(self, cmd: str) -> Channel:
        sock = socket.create_connection((self.uri, self.port), timeout=self.timeout)
        ch = Channel(sock)
        ch.send_int(MAGIC)
        magic = ch.recv_int()
        if magic != MAGIC:
            ch.close()
            raise ConnectionError(f"tracker answered magic {magic:#x}")
        ch.send_int(self.rank)
        ch.send_int(self.world_size)
        ch.send_str(self.jobid)
        ch.send_str(cmd)
        return ch

    def start(self, recover: bool = False) -> Topology:
        """Join the job; returns this worker's rank and topology."""
        ch = self._connect("recover" if recover else "start")
        try:
            rank = ch.recv_int()
            parent = ch.recv_int()
            world = ch.recv_int()
            nnbr = ch.recv_int()
            tree = [ch.recv_int() for _ in range(nnbr)]
            prev = ch.recv_int()
            nxt = ch.recv_int()
            links = sorted(set(tree) | {r for r in (prev, nxt) if r != -1})
            ch.send_int(len(links))
            for r in links:
                ch.send_int(r)
            nconn = ch.recv_int()
            _naccept = ch.recv_int()
            for _ in range(nconn):  # nothing to connect: links reported good
                ch.recv_str()
                ch.recv_int()
                ch.recv_int()
            ch.send_int(0)  # no errors
            ch.send_int(0)  # listen port (unused: RCCL is the data plane)
        finally:
            ch.close()
        self.rank, self.world_size = rank, world
        self.topology = Topology(rank, parent, world, tree, prev, nxt)
        return self.topology

    def print(self, msg: str) -> None:
        ch = self._connect("print")
        try:
            ch.send_str(msg)
        finally:
            ch.close()

    def shutdown(self) -> None:
        self.stop_heartbeat()
        ch = self._connect("shutdown")
        ch.close()

    def heartbeat(self) -> Optional[str]:
        """One liveness ping; returns None while the job is healthy, else the
        tracker's failure reason."""
        ch = self._connect("heartbeat")
        try:
            status = ch.recv_int()
            return ch.recv_str() if status != 0 else None
        finally:
            ch.close()

    def abort(self, msg: str) -> None:
        """Report a fatal error of this rank: the tracker fails the job and
        every other rank hears it on its next heartbeat."""
        ch = self._connect("abort")
        try:
            ch.send_str(msg)
            ch.wait_closed()  # the tracker closes after recording the failure
        finally:
            ch.close()

    def start_heartbeat(self, period: float = 5.0,
                        on_failure: Optional[Callable[[str], None]] = None) -> None:
        """Background heartbeats so the tracker detects this rank dying; if the
        job fails (another rank died / aborted, or the tracker is gone)
        ``on_failure(reason)`` runs once on the heartbeat thread."""
        self._hb_stop = threading.Event()
        stop = self._hb_stop

        def report(reason: str) -> None:
            if on_failure is not None:
                on_failure(reason)

        def loop():
            while not stop.wait(period):
                try:
                    reason = self.heartbeat()
                except (OSError, ConnectionError) as e:
                    if not stop.is_set():
                        report(f"tracker unreachable: {e}")
                    return
                if reason is not None:
                    report(reason)
                    return

        reason = self.heartbeat()
        if reason is not None:
            report(reason)
            return
        threading.Thread(target=loop, name="dmlc-heartbeat", daemon=True).start()

    def stop_heartbeat(self) -> None:
        if self._hb_stop is not None:
            self._hb_stop.set()
            self._hb_stop = None

    def rccl_put(self, key: str, blob: bytes) -> None:
        ch = self._connect("rccl")
        try:
            ch.send_int(0)
            ch.send_str(key)
            ch.send_bytes(blob)
            ch.recv_int()
        finally:
            ch.close()

    def rccl_get(self, key: str) -> bytes:
        ch = self._connect("rccl")
        try:
            ch.send_int(1)
            ch.send_str(key)
            return ch.recv_bytes()
        finally:
            ch.close()

    def attempt(self) -> int:
        """This launch's attempt number for the task id ``jobid`` (0 the
        first time the tracker hears it, then 1, 2, ...)."""
        ch = self._connect("attempt")
        try:
            return ch.recv_int()
        finally:
            ch.close()

    def barrier(self, key: str = "default", count: Optional[int] = None) -> None:
        ch = self._connect("barrier")
        try:
            ch.send_str(key)
            ch.send_int(count if count is not None else self.world_size)
            ch.recv_int()
        finally:
            ch.close()

    def exchange_unique_id(self, make_id, key: str = "world") -> bytes:
        """RCCL bootstrap: rank 0 creates the id with make_id() and uploads it;
        everyone (rank 0 included) returns the same bytes."""
        if self.rank == 0:
            blob = bytes(make_id())
            self.rccl_put(key, blob)
            return blob
        return self.rccl_get(key)
