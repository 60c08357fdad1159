"""One process per MI355X: process-group bootstrap and the collectives of the
ingestion runtime (SURVEY §2.12 call-site table, §5.8).

* :func:`init` builds the torch.distributed process group ("nccl" is RCCL on
  ROCm) from whichever launcher started us: torchrun (RANK/WORLD_SIZE/
  MASTER_*) or dmlc-submit (DMLC_TRACKER_URI/PORT -- the tracker assigns the
  rank and brokers the TCP store address through its ``rccl`` command).
  The GPU is chosen by *local* index (DMLC_LOCAL_RANK / LOCAL_RANK), never
  by tracker rank, which is arrival order.
* :func:`global_stats` is the control collective: one all-reduce(SUM) of the
  counters and one all-reduce(MAX) of max_index -> global NumCol (reference
  ``BasicRowIter::NumCol``, `src/data/basic_row_iter.h:46-48`).
* :class:`GradAllReducer` is the data-parallel gradient path of the sparse
  model demonstrator: gradients are packed into flat buckets (default
  64 MiB -- large messages amortise RCCL's per-call latency over xGMI) and
  all-reduced asynchronously as soon as a bucket's last gradient is
  produced, overlapping communication with the rest of backward.
"""
from __future__ import annotations

import os
import socket
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as tdist

from .client import TrackerClient

_tracker: Optional[TrackerClient] = None


def local_rank() -> int:
    for k in ("DMLC_LOCAL_RANK", "LOCAL_RANK"):
        if k in os.environ:
            return int(os.environ[k])
    return 0


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("", 0))
        return s.getsockname()[1]


def _fail_fast(reason: str) -> None:
    """Default reaction to a tracker-signalled job failure: a peer is gone, so
    any RCCL collective would block forever -- end this rank now (SIGTERM lets
    the launcher's retry policy, DMLC_NUM_ATTEMPT, take over)."""
    import logging
    import signal

    logging.getLogger("dmlc.dist").error("job failed (%s): terminating rank", reason)
    os.kill(os.getpid(), signal.SIGTERM)


def init(backend: Optional[str] = None, timeout_s: float = 600.0,
         on_failure=None) -> Dict[str, int]:
    """Initialise the default process group; returns {rank, world_size, local_rank}.

    Under dmlc-submit the rank heartbeats the tracker every
    ``DMLC_HEARTBEAT_PERIOD`` seconds (default 5, 0 = off); when the job fails
    ``on_failure(reason)`` runs (default: terminate this rank)."""
    global _tracker
    if tdist.is_available() and tdist.is_initialized():
        return {"rank": tdist.get_rank(), "world_size": tdist.get_world_size(),
                "local_rank": local_rank()}
    use_gpu = torch.cuda.is_available()
    backend = backend or ("nccl" if use_gpu else "gloo")
    lr = local_rank()
    if use_gpu:
        torch.cuda.set_device(lr)
    import datetime
    to = datetime.timedelta(seconds=timeout_s)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": torch.device("cuda", lr)} if backend == "nccl" else {}
        tdist.init_process_group(backend, timeout=to, **kw)
    elif "DMLC_TRACKER_URI" in os.environ:
        _tracker = TrackerClient()
        topo = _tracker.start()
        period = float(os.environ.get("DMLC_HEARTBEAT_PERIOD", "5"))
        if period > 0:
            _tracker.start_heartbeat(period, on_failure or _fail_fast)
        if topo.rank == 0:
            host = os.environ.get("DMLC_NODE_HOST") or socket.gethostbyname(socket.gethostname())
            if os.environ.get("DMLC_JOB_CLUSTER") == "local":
                host = "127.0.0.1"
            addr = f"{host}:{_free_port()}"
            _tracker.rccl_put("torch_store", addr.encode())
        else:
            addr = _tracker.rccl_get("torch_store").decode()
        kw = {"device_id": torch.device("cuda", lr)} if backend == "nccl" else {}
        tdist.init_process_group(backend, init_method=f"tcp://{addr}", rank=topo.rank,
                                 world_size=topo.world_size, timeout=to, **kw)
    else:
        return {"rank": 0, "world_size": 1, "local_rank": lr}
    return {"rank": tdist.get_rank(), "world_size": tdist.get_world_size(), "local_rank": lr}


def finalize() -> None:
    global _tracker
    if tdist.is_available() and tdist.is_initialized():
        tdist.destroy_process_group()
    if _tracker is not None:
        _tracker.shutdown()
        _tracker = None


def world() -> int:
    return tdist.get_world_size() if tdist.is_available() and tdist.is_initialized() else 1


def rank() -> int:
    return tdist.get_rank() if tdist.is_available() and tdist.is_initialized() else 0


def _device() -> torch.device:
    if tdist.is_initialized() and tdist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def global_stats(counters: Sequence[float], max_index: int) -> (List[float], int):
    """SUM-all-reduce `counters`, MAX-all-reduce `max_index` (one message each)."""
    dev = _device()
    t = torch.tensor(list(counters), dtype=torch.float64, device=dev)
    m = torch.tensor([max_index], dtype=torch.int64, device=dev)
    if world() > 1:
        tdist.all_reduce(t)
        tdist.all_reduce(m, op=tdist.ReduceOp.MAX)
    return t.tolist(), int(m.item())


def all_gather_counts(rows: int, nnz: int) -> List[List[int]]:
    """Every rank's (rows, nnz): global row offsets for sharded CSR blocks."""
    dev = _device()
    mine = torch.tensor([rows, nnz], dtype=torch.int64, device=dev)
    if world() == 1:
        return [mine.tolist()]
    out = [torch.empty_like(mine) for _ in range(world())]
    tdist.all_gather(out, mine)
    return [o.tolist() for o in out]


def broadcast_object(obj, src: int = 0):
    """Broadcast a small picklable object created by this job (e.g. a
    Parameter dict or an index file's contents) from `src`."""
    if world() == 1:
        return obj
    buf = [obj]
    tdist.broadcast_object_list(buf, src=src)
    return buf[0]


class GradAllReducer:
    """Bucketed, backward-overlapped gradient averaging for data parallelism."""

    def __init__(self, params: Sequence[torch.nn.Parameter], bucket_mb: float = 64.0):
        self.params = [p for p in params if p.requires_grad]
        self.world = world()
        cap = int(bucket_mb * (1 << 20))
        # reverse registration order ~ order in which backward produces grads
        self.buckets: List[List[torch.nn.Parameter]] = []
        cur, size = [], 0
        for p in reversed(self.params):
            nbytes = p.numel() * p.element_size()
            if cur and size + nbytes > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += nbytes
        if cur:
            self.buckets.append(cur)
        self._bucket_of = {id(p): i for i, b in enumerate(self.buckets) for p in b}
        self._pending = [0] * len(self.buckets)
        self._works: List = []
        self._flats: Dict[int, torch.Tensor] = {}
        self._hooks = []
        if self.world > 1:
            for p in self.params:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_grad))
        self._reset()

    def _reset(self) -> None:
        self._pending = [len(b) for b in self.buckets]
        self._works = []
        self._flats = {}

    def _on_grad(self, p: torch.nn.Parameter) -> None:
        i = self._bucket_of[id(p)]
        self._pending[i] -= 1
        if self._pending[i] == 0:
            grads = [q.grad for q in self.buckets[i]]
            flat = torch.cat([g.reshape(-1) for g in grads]) if len(grads) > 1 else grads[0].reshape(-1)
            flat.div_(self.world)
            self._flats[i] = flat
            self._works.append((i, tdist.all_reduce(flat, async_op=True)))

    def synchronize(self) -> None:
        """Wait for every bucket and scatter the averaged values back."""
        if self.world == 1:
            return
        for i, work in self._works:
            work.wait()
            flat = self._flats[i]
            if len(self.buckets[i]) > 1:
                off = 0
                for q in self.buckets[i]:
                    n = q.grad.numel()
                    q.grad.copy_(flat[off:off + n].view_as(q.grad))
                    off += n
            else:
                q = self.buckets[i][0]
                if flat.data_ptr() != q.grad.data_ptr():
                    q.grad.copy_(flat.view_as(q.grad))
        self._reset()

    def remove(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
