"""Rendezvous tracker: the rabit wire protocol plus RCCL bootstrap.

Parity (reference `tracker/dmlc_tracker/tracker.py`):
  * framing: native-endian int32, strings = int32 length + bytes (:24-47);
  * handshake magic 0xff99 echoed back, then rank, world_size, jobid, cmd
    (:50, :58-71); commands start / recover / shutdown / print (:256-291);
  * batch rank assignment once every pending worker arrived, sorted by host,
    jobid -> rank map for restarted workers (:73-78, :293-311);
  * topology: binary-heap tree + a ring sharing tree edges, relabelled so ring
    neighbours are consecutive ranks (:166-252); link negotiation loop
    (:105-135);
  * PS scheduler launch with DMLC_PS_ROOT_URI/PORT (:336-386);
  * get_host_ip / submit / standalone DMLC_TRACKER_ENV_START..END (:389-451).

New in this implementation:
  * ``rccl`` command: rank 0 uploads its ncclUniqueId (any opaque bytes, keyed
    by communicator name), every rank downloads it -- the RCCL bootstrap;
  * ``barrier`` command: named, counted barrier held by the tracker;
  * ``heartbeat`` command and a liveness timeout: a rank that heartbeated once
    and then goes silent for ``heartbeat_timeout`` seconds fails the job
    instead of hanging it (reference §7.4 quirk #8).  The reply to every
    heartbeat is a status int (0 ok / 1 failed + reason), so live ranks learn
    of the failure within one heartbeat period and abort their RCCL
    communicators (``ncclCommAbort``) instead of blocking in a collective
    whose peer is gone; the tracker raises after ``abort_grace`` seconds;
  * ``abort`` command: a rank reports its own fatal error (fail fast);
  * an overall ``timeout`` for the rendezvous; the accept loop hands every
    connection to its own thread, so neither a slow ``start`` negotiation nor
    held rccl/barrier sockets ever delay another rank's heartbeat;
  * Python 3 only (the reference breaks on 3.9+ with ``Thread.isAlive``).
"""
from __future__ import annotations

import argparse
import logging
import os
import socket
import struct
import subprocess
import sys
import threading
import time
from typing import Callable, Dict, List, Optional, Tuple

MAGIC = 0xFF99
_INT = struct.Struct("@i")

logger = logging.getLogger("dmlc.tracker")


class TrackerError(RuntimeError):
    """The job failed at the rendezvous level (timeout, dead worker, protocol)."""


# --------------------------------------------------------------------------- framing
class Channel:
    """Blocking int32 / string framing over a socket."""

    def __init__(self, sock: socket.socket):
        self.sock = sock

    def _recv_exact(self, n: int) -> bytes:
        buf = bytearray()
        while len(buf) < n:
            chunk = self.sock.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("peer closed the connection")
            buf += chunk
        return bytes(buf)

    def recv_int(self) -> int:
        return _INT.unpack(self._recv_exact(_INT.size))[0]

    def send_int(self, v: int) -> None:
        self.sock.sendall(_INT.pack(int(v)))

    def recv_bytes(self) -> bytes:
        n = self.recv_int()
        if n < 0 or n > (1 << 30):
            raise ConnectionError(f"bad string length {n}")
        return self._recv_exact(n)

    def send_bytes(self, b: bytes) -> None:
        self.send_int(len(b))
        self.sock.sendall(b)

    def recv_str(self) -> str:
        return self.recv_bytes().decode()

    def send_str(self, s: str) -> None:
        self.send_bytes(s.encode())

    def wait_closed(self) -> None:
        """Block until the peer closes the connection (or the socket times out)."""
        try:
            while self.sock.recv(1):
                pass
        except OSError:
            pass

    def close(self) -> None:
        try:
            self.sock.close()
        except OSError:
            pass


# --------------------------------------------------------------------------- topology
def tree_neighbors(rank: int, world: int) -> List[int]:
    """Binary-heap neighbours of `rank`: parent first, then children."""
    out = []
    if rank > 0:
        out.append((rank + 1) // 2 - 1)
    for c in (2 * rank + 1, 2 * rank + 2):
        if c < world:
            out.append(c)
    return out


def tree_parent(rank: int) -> int:
    return (rank + 1) // 2 - 1


def _ring_order(world: int) -> List[int]:
    """Depth-first order of the heap tree; the last child's subtree is walked
    in reverse so consecutive entries are tree edges wherever possible.

    Children are visited in the order a small Python set of ints iterates
    (slot = value & 7), which is what the reference's ``set`` difference
    produces; keeping it makes the relabelled ring identical to the
    reference's for every world size.
    """
    def walk(r: int) -> List[int]:
        kids = [c for c in tree_neighbors(r, world) if c != tree_parent(r)]
        kids.sort(key=lambda c: c & 7)
        order = [r]
        for i, c in enumerate(kids):
            sub = walk(c)
            if i == len(kids) - 1:
                sub.reverse()
            order.extend(sub)
        return order

    sys.setrecursionlimit(max(sys.getrecursionlimit(), 4 * world + 100))
    return walk(0)


def link_map(world: int) -> Tuple[Dict[int, List[int]], Dict[int, int], Dict[int, Tuple[int, int]]]:
    """(tree neighbours, parent, (ring prev, ring next)) after relabelling ranks
    by ring position, so rank r's ring neighbours are r-1 and r+1."""
    order = _ring_order(world)
    assert len(order) == world
    relabel = {old: new for new, old in enumerate(order)}
    tree, parent, ring = {}, {}, {}
    for old in range(world):
        new = relabel[old]
        tree[new] = [relabel[x] for x in tree_neighbors(old, world)]
        parent[new] = -1 if old == 0 else relabel[tree_parent(old)]
        ring[new] = ((new - 1) % world, (new + 1) % world)
    return tree, parent, ring


# --------------------------------------------------------------------------- worker entry
class _Worker:
    """One accepted connection after the common handshake."""

    def __init__(self, sock: socket.socket, addr):
        self.ch = Channel(sock)
        self.host = addr[0]
        magic = self.ch.recv_int()
        if magic != MAGIC:
            raise ConnectionError(f"invalid magic {magic:#x} from {self.host}")
        self.ch.send_int(MAGIC)
        self.rank = self.ch.recv_int()
        self.world_size = self.ch.recv_int()
        self.jobid = self.ch.recv_str()
        self.cmd = self.ch.recv_str()
        self.port: Optional[int] = None
        self.wait_accept = 0

    def decide_rank(self, job_map: Dict[str, int]) -> int:
        if self.rank >= 0:
            return self.rank
        if self.jobid != "NULL" and self.jobid in job_map:
            return job_map[self.jobid]
        return -1

    def assign_rank(self, rank: int, wait_conn: Dict[int, "_Worker"], tree, parent, ring) -> List[int]:
        """Send rank + topology, then broker peer links until the worker
        reports no errors (reference tracker.py:84-135)."""
        self.rank = rank
        ch = self.ch
        nbrs = set(tree[rank])
        prev, nxt = ring[rank]
        ch.send_int(rank)
        ch.send_int(parent[rank])
        ch.send_int(len(tree))
        ch.send_int(len(nbrs))
        for r in nbrs:
            ch.send_int(r)
        for r in (prev, nxt):
            if r != -1 and r != rank:
                nbrs.add(r)
                ch.send_int(r)
            else:
                ch.send_int(-1)
        while True:
            ngood = ch.recv_int()
            good = {ch.recv_int() for _ in range(ngood)}
            if not good.issubset(nbrs):
                raise ConnectionError(f"rank {rank} reported unknown peers {good - nbrs}")
            bad = nbrs - good
            connect = [r for r in bad if r in wait_conn]
            ch.send_int(len(connect))
            ch.send_int(len(bad) - len(connect))
            for r in connect:
                ch.send_str(wait_conn[r].host)
                ch.send_int(wait_conn[r].port)
                ch.send_int(r)
            if ch.recv_int() != 0:
                continue  # worker retries the failed links
            self.port = ch.recv_int()
            done = []
            for r in connect:
                wait_conn[r].wait_accept -= 1
                if wait_conn[r].wait_accept == 0:
                    done.append(r)
            for r in done:
                wait_conn.pop(r, None)
            self.wait_accept = len(bad) - len(connect)
            return done


# --------------------------------------------------------------------------- tracker
class _JobState:
    """Mutable rendezvous state shared by the tracker's connection threads."""

    def __init__(self, n: int):
        self.n = n
        self.shutdown: Dict[int, bool] = {}
        self.wait_conn: Dict[int, _Worker] = {}
        self.job_map: Dict[str, int] = {}
        self.pending: List[_Worker] = []
        self.todo: List[int] = []
        self.tree = self.parent = self.ring = None
        self.rccl_ids: Dict[str, bytes] = {}
        self.rccl_waiters: Dict[str, List[_Worker]] = {}
        self.barriers: Dict[str, List[_Worker]] = {}
        self.last_beat: Dict[int, float] = {}
        # failure state: once a rank is declared dead (or aborts) the job is
        # failed; live ranks learn it from their next heartbeat reply (and
        # abort their RCCL communicators) during a grace period, then the
        # tracker raises.
        self.failed: Optional[str] = None
        self.failed_at = 0.0
        self.dead: Dict[int, bool] = {}
        self.fatal: Optional[BaseException] = None
        # launches seen per task id (``attempt``): a relaunched container
        # learns its DMLC_NUM_ATTEMPT here when its launcher cannot say
        self.attempts: Dict[str, int] = {}


class RabitTracker:
    """Rendezvous server for `nworker` processes."""

    def __init__(self, host_ip: str, nworker: int, port: int = 9091, port_end: int = 9999,
                 timeout: Optional[float] = None, heartbeat_timeout: Optional[float] = None,
                 io_timeout: float = 60.0, abort_grace: Optional[float] = None):
        family = socket.getaddrinfo(host_ip, None)[0][0]
        sock = socket.socket(family, socket.SOCK_STREAM)
        sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 0)
        for p in range(port, port_end):
            try:
                sock.bind((host_ip, p))
                self.port = p
                break
            except OSError:
                continue
        else:
            raise TrackerError(f"no free port in [{port}, {port_end})")
        sock.listen(1024)
        sock.settimeout(0.5)
        self.sock = sock
        self.host_ip = host_ip
        self.nworker = nworker
        self.timeout = timeout
        self.heartbeat_timeout = heartbeat_timeout
        # how long live ranks get to see the failure in a heartbeat reply
        self.abort_grace = abort_grace if abort_grace is not None else (
            heartbeat_timeout if heartbeat_timeout is not None else 5.0)
        self.io_timeout = io_timeout
        self.thread: Optional[threading.Thread] = None
        self.start_time: Optional[float] = None
        self.end_time: Optional[float] = None
        self.error: Optional[BaseException] = None
        self.messages: List[str] = []
        self.assigned: Dict[int, str] = {}
        self._stop = threading.Event()
        self._mu = threading.Lock()        # job state
        self._start_mu = threading.Lock()  # rank assignment / link negotiation
        self._state: Optional[_JobState] = None
        logger.info("tracker listening on %s:%d", host_ip, self.port)

    def worker_envs(self) -> Dict[str, object]:
        return {"DMLC_TRACKER_URI": self.host_ip, "DMLC_TRACKER_PORT": self.port}

    slave_envs = worker_envs  # reference name

    # ---------------------------------------------------------------- main loop
    def _serve(self) -> None:
        """Accept loop. Every connection is handled on its own thread, so a
        slow handshake or a long link negotiation (``start``) never delays
        another rank's heartbeat; shared job state is guarded by ``_mu`` and
        rank assignment is serialised by ``_start_mu`` (never held together
        with blocking I/O under ``_mu``)."""
        st = _JobState(self.nworker)
        self._state = st
        t_begin = time.time()
        while not self._stop.is_set():
            with self._mu:
                if len(st.shutdown) >= st.n:
                    break
                if st.fatal is not None:
                    raise st.fatal
                now = time.time()
                if self.timeout is not None and now - t_begin > self.timeout:
                    raise TrackerError(f"job did not finish within {self.timeout}s "
                                       f"({len(st.shutdown)}/{st.n} ranks shut down)")
                if self.heartbeat_timeout is not None:
                    for r, t in list(st.last_beat.items()):
                        if r not in st.shutdown and r not in st.dead and \
                                now - t > self.heartbeat_timeout:
                            self._fail(st, f"rank {r} missed heartbeats for {now - t:.1f}s "
                                           f"(> {self.heartbeat_timeout}s)", r)
                if st.failed is not None and (
                        now - st.failed_at > self.abort_grace
                        or len(set(st.shutdown) | set(st.dead)) >= st.n):
                    raise TrackerError(st.failed)
            try:
                conn, addr = self.sock.accept()
            except socket.timeout:
                continue
            conn.settimeout(self.io_timeout)
            th = threading.Thread(target=self._handle, args=(st, conn, addr),
                                  name="dmlc-tracker-conn", daemon=True)
            th.start()
        self.end_time = time.time()
        if self.start_time is not None:
            logger.info("all workers finished; %.3f s between start and finish",
                        self.end_time - self.start_time)

    def _fail(self, st: "_JobState", reason: str, rank: int) -> None:
        """Mark the job failed (caller holds _mu). Live ranks learn it from
        their next heartbeat reply during the abort grace period."""
        st.dead[rank] = True
        if st.failed is None:
            st.failed, st.failed_at = reason, time.time()
            logger.error("job failed: %s", reason)
            for group in list(st.rccl_waiters.values()) + list(st.barriers.values()):
                for h in group:  # unblock ranks waiting in rccl get / barrier
                    h.ch.close()
            st.rccl_waiters.clear()
            st.barriers.clear()

    def _handle(self, st: "_JobState", conn: socket.socket, addr) -> None:
        try:
            w = _Worker(conn, addr)
        except (ConnectionError, OSError, UnicodeDecodeError) as e:
            logger.warning("dropping connection from %s: %s", addr, e)
            conn.close()
            return
        try:
            self._dispatch(st, w)
        except TrackerError as e:
            with self._mu:
                if st.fatal is None:
                    st.fatal = e
            w.ch.close()
        except (ConnectionError, OSError, UnicodeDecodeError) as e:
            logger.warning("command %r from %s failed: %s", w.cmd, w.host, e)
            w.ch.close()

    def _dispatch(self, st: "_JobState", w: _Worker) -> None:
        if w.cmd == "print":
            msg = w.ch.recv_str().rstrip()
            with self._mu:
                self.messages.append(msg)
            logger.info("%s", msg)
            w.ch.close()
            return
        if w.cmd == "heartbeat":
            with self._mu:
                st.last_beat[w.rank] = time.time()
                failed = st.failed
            w.ch.send_int(0 if failed is None else 1)
            if failed is not None:
                w.ch.send_str(failed)
            w.ch.close()
            return
        if w.cmd == "abort":
            msg = w.ch.recv_str()
            with self._mu:
                self._fail(st, f"rank {w.rank} aborted: {msg}", w.rank)
            # closed only once recorded: a client waiting for the close knows
            # every later heartbeat reply carries the failure
            w.ch.close()
            return
        if w.cmd == "shutdown":
            with self._mu:
                if w.rank < 0 or w.rank in st.shutdown:
                    raise TrackerError(f"bad shutdown from rank {w.rank}")
                st.shutdown[w.rank] = True
                st.last_beat.pop(w.rank, None)
            logger.debug("shutdown from rank %d", w.rank)
            w.ch.close()
            return
        if w.cmd == "rccl":
            op = w.ch.recv_int()
            key = w.ch.recv_str()
            if op == 0:  # put
                blob = w.ch.recv_bytes()
                w.ch.send_int(0)
                w.ch.close()
                with self._mu:
                    st.rccl_ids[key] = blob
                    waiters = st.rccl_waiters.pop(key, [])
                for h in waiters:
                    self._reply_close(h, lambda c: c.send_bytes(blob))
                return
            with self._mu:
                blob = st.rccl_ids.get(key)
                if blob is None:
                    st.rccl_waiters.setdefault(key, []).append(w)
                    return
            w.ch.send_bytes(blob)
            w.ch.close()
            return
        if w.cmd == "attempt":
            # the n-th launch of a task id (0 first): what the reference
            # ApplicationMaster exports as DMLC_NUM_ATTEMPT per container
            # (ApplicationMaster.java:446); the YARN services launcher asks here
            with self._mu:
                n = st.attempts.get(w.jobid, 0)
                st.attempts[w.jobid] = n + 1
            w.ch.send_int(n)
            w.ch.close()
            return
        if w.cmd == "barrier":
            key = w.ch.recv_str()
            count = w.ch.recv_int()
            with self._mu:
                group = st.barriers.setdefault(key, [])
                group.append(w)
                release = st.barriers.pop(key) if len(group) >= count else []
            for h in release:
                self._reply_close(h, lambda c: c.send_int(0))
            return
        if w.cmd not in ("start", "recover"):
            logger.warning("unknown command %r from %s", w.cmd, w.host)
            w.ch.close()
            return
        with self._start_mu:
            self._start(st, w)

    @staticmethod
    def _reply_close(h: _Worker, fn) -> None:
        try:
            fn(h.ch)
        except OSError as e:
            logger.warning("reply to %s failed: %s", h.host, e)
        h.ch.close()

    def _start(self, st: "_JobState", w: _Worker) -> None:
        """Rank assignment + link negotiation (serialised by _start_mu)."""
        if st.tree is None:
            if w.cmd != "start":
                raise TrackerError("first worker must send start")
            if w.world_size > 0:
                with self._mu:
                    st.n = self.nworker = w.world_size
            st.tree, st.parent, st.ring = link_map(st.n)
            st.todo = list(range(st.n))
        elif w.world_size not in (-1, st.n):
            raise TrackerError(f"world size mismatch: {w.world_size} vs {st.n}")
        if w.cmd == "recover" and w.rank < 0:
            raise TrackerError("recover needs an explicit rank")

        rank = w.decide_rank(st.job_map)
        if rank == -1:
            if not st.todo:
                raise TrackerError("more workers than the world size")
            st.pending.append(w)
            if len(st.pending) == len(st.todo):
                st.pending.sort(key=lambda x: x.host)
                for p in st.pending:
                    r = st.todo.pop(0)
                    if p.jobid != "NULL":
                        st.job_map[p.jobid] = r
                    p.assign_rank(r, st.wait_conn, st.tree, st.parent, st.ring)
                    self.assigned[r] = p.host
                    if p.wait_accept > 0:
                        st.wait_conn[r] = p
                st.pending = []
            if not st.todo and self.start_time is None:
                logger.info("all %d workers started", st.n)
                self.start_time = time.time()
        else:
            if rank in st.todo:
                st.todo.remove(rank)
            w.assign_rank(rank, st.wait_conn, st.tree, st.parent, st.ring)
            self.assigned[rank] = w.host
            if w.wait_accept > 0:
                st.wait_conn[rank] = w
            if not st.todo and self.start_time is None:
                self.start_time = time.time()

    def _run(self) -> None:
        try:
            self._serve()
        except BaseException as e:  # surfaced by join()
            self.error = e
            logger.error("tracker failed: %s", e)
        finally:
            self.sock.close()

    def start(self, nworker: Optional[int] = None) -> None:
        if nworker is not None:
            self.nworker = nworker
        self.thread = threading.Thread(target=self._run, name="dmlc-tracker", daemon=True)
        self.thread.start()

    def alive(self) -> bool:
        return self.thread is not None and self.thread.is_alive()

    def join(self, timeout: Optional[float] = None) -> None:
        if self.thread is not None:
            self.thread.join(timeout)
        if self.error is not None:
            raise TrackerError(str(self.error)) from self.error

    def stop(self) -> None:
        self._stop.set()


class PSTracker:
    """Starts the parameter-server scheduler process (role env only)."""

    def __init__(self, host_ip: str, cmd: Optional[str], port: int = 9091, port_end: int = 9999,
                 envs: Optional[Dict[str, object]] = None):
        self.cmd = cmd
        self.thread = None
        if cmd is None:
            return
        self.host_ip = host_ip
        self.port = None
        for p in range(port, port_end):
            with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
                try:
                    s.bind(("", p))
                    self.port = p
                    break
                except OSError:
                    continue
        if self.port is None:
            raise TrackerError("no free port for the PS scheduler")
        env = os.environ.copy()
        env.update({"DMLC_ROLE": "scheduler", "DMLC_PS_ROOT_URI": str(host_ip),
                    "DMLC_PS_ROOT_PORT": str(self.port)})
        env.update({k: str(v) for k, v in (envs or {}).items()})
        self.thread = threading.Thread(
            target=lambda: subprocess.check_call(cmd, env=env, shell=True), daemon=True)
        self.thread.start()

    def worker_envs(self) -> Dict[str, object]:
        if self.cmd is None:
            return {}
        return {"DMLC_PS_ROOT_URI": self.host_ip, "DMLC_PS_ROOT_PORT": self.port}

    slave_envs = worker_envs

    def alive(self) -> bool:
        return self.thread is not None and self.thread.is_alive()

    def join(self) -> None:
        if self.thread is not None:
            self.thread.join()


def get_host_ip(host_ip: Optional[str] = None) -> str:
    """'auto'/'ip': this host's address (a non-loopback one when the hostname
    resolves to 127.x); 'dns': the FQDN; anything else is returned as is."""
    if host_ip is None or host_ip == "auto":
        host_ip = "ip"
    if host_ip == "dns":
        return socket.getfqdn()
    if host_ip != "ip":
        return host_ip
    try:
        ip = socket.gethostbyname(socket.getfqdn())
    except OSError:
        try:
            ip = socket.gethostbyname(socket.gethostname())
        except OSError:
            ip = "127.0.0.1"
    if ip.startswith("127."):
        try:
            with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
                s.connect(("10.255.255.255", 1))  # no packet is sent
                ip = s.getsockname()[0]
        except OSError:
            ip = "127.0.0.1"
    return ip


def submit(nworker: int, nserver: int, fun_submit: Callable[[int, int, Dict[str, object]], None],
           host_ip: str = "auto", pscmd: Optional[str] = None, timeout: Optional[float] = None,
           heartbeat_timeout: Optional[float] = None) -> Optional[RabitTracker]:
    """Start the rendezvous service, call fun_submit(nworker, nserver, envs)
    to launch the processes, and wait for the job (reference tracker.py:410-433)."""
    envs: Dict[str, object] = {"DMLC_NUM_WORKER": nworker, "DMLC_NUM_SERVER": nserver}
    host_ip = get_host_ip(host_ip)
    if nserver == 0:
        tracker = RabitTracker(host_ip, nworker, timeout=timeout,
                               heartbeat_timeout=heartbeat_timeout)
        envs.update(tracker.worker_envs())
        tracker.start(nworker)
        fun_submit(nworker, nserver, envs)
        tracker.join()
        return tracker
    ps = PSTracker(host_ip, pscmd, envs=envs)
    envs.update(ps.worker_envs())
    fun_submit(nworker, nserver, envs)
    ps.join()
    return None


def start_rabit_tracker(args) -> None:
    """Standalone mode: print the worker environment between markers."""
    envs: Dict[str, object] = {"DMLC_NUM_WORKER": args.num_workers,
                               "DMLC_NUM_SERVER": args.num_servers}
    tracker = RabitTracker(get_host_ip(args.host_ip), args.num_workers, timeout=args.timeout)
    envs.update(tracker.worker_envs())
    tracker.start(args.num_workers)
    sys.stdout.write("DMLC_TRACKER_ENV_START\n")
    for k, v in envs.items():
        sys.stdout.write(f"{k}={v}\n")
    sys.stdout.write("DMLC_TRACKER_ENV_END\n")
    sys.stdout.flush()
    tracker.join()


def main(argv=None) -> None:
    ap = argparse.ArgumentParser(description="dmlc rendezvous tracker")
    ap.add_argument("--num-workers", required=True, type=int)
    ap.add_argument("--num-servers", default=0, type=int)
    ap.add_argument("--host-ip", default="auto", type=str)
    ap.add_argument("--timeout", default=None, type=float)
    ap.add_argument("--log-level", default="INFO", choices=["INFO", "DEBUG"])
    args = ap.parse_args(argv)
    logging.basicConfig(format="%(asctime)-15s %(message)s", level=getattr(logging, args.log_level))
    if args.num_servers == 0:
        start_rabit_tracker(args)
    else:
        raise SystemExit("standalone mode supports only rabit (num_servers == 0)")


if __name__ == "__main__":
    main()
