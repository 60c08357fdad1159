"""Native RCCL communicator on one MI355X (world size 1: RCCL refuses two
ranks on one device, and multi-GPU runs belong to the driver's 8-GPU node).
Checks every collective against the trivially known result, and that the
communicator reuses PyTorch's RCCL instead of loading a second copy."""
import pytest
import torch

from dmlc_core_amd import _dmlc

pytestmark = pytest.mark.gpu


def _ptr(t):
    return t.data_ptr()


def test_rccl_collectives_world1():
    assert _dmlc.Communicator.available()
    # torch (imported first by dmlc_core_amd) already loaded its RCCL: the
    # communicator must resolve to that same library, not load a second copy
    import os
    path = _dmlc.Communicator.library_path()
    assert path and "rccl" in os.path.basename(path), path
    loaded = set()
    with open("/proc/self/maps") as f:
        for line in f:
            if "librccl" in line:
                loaded.add(os.path.realpath(line.split()[-1]))
    assert len(loaded) == 1 and os.path.realpath(path) in loaded, (path, loaded)
    uid = _dmlc.Communicator.new_unique_id()
    assert len(uid) == 128
    comm = _dmlc.Communicator(0, 1, 0, uid)
    s = torch.cuda.current_stream().cuda_stream
    x = torch.arange(1000, dtype=torch.float32, device="cuda")
    y = torch.empty_like(x)
    comm.all_reduce(_ptr(x), _ptr(y), x.numel(), _dmlc.DataType.float32, _dmlc.ReduceOp.sum, s)
    g = torch.empty_like(x)
    comm.all_gather(_ptr(x), _ptr(g), x.numel(), _dmlc.DataType.float32, s)
    b = torch.zeros_like(x)
    comm.broadcast(_ptr(x), _ptr(b), x.numel(), _dmlc.DataType.float32, 0, s)
    m = torch.tensor([5, 9], dtype=torch.int64, device="cuda")
    mo = torch.empty_like(m)
    comm.all_reduce(_ptr(m), _ptr(mo), 2, _dmlc.DataType.int64, _dmlc.ReduceOp.max, s)
    a2a = torch.empty(300, dtype=torch.float32, device="cuda")
    comm.all_to_all_v(_ptr(x), [300], [100], _ptr(a2a), [300], [0], _dmlc.DataType.float32, s)
    comm.barrier(s)
    torch.cuda.synchronize()
    assert torch.equal(y, x) and torch.equal(g, x) and torch.equal(b, x)
    assert mo.tolist() == [5, 9]
    assert torch.equal(a2a, x[100:400])
    del comm


def test_torch_rccl_process_group_world1(tmp_path):
    import torch.distributed as td
    from dmlc_core_amd.parallel import dist
    import os
    os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "MASTER_ADDR": "127.0.0.1",
                       "MASTER_PORT": "29533"})
    try:
        info = dist.init("nccl")
        assert info["world_size"] == 1
        counts, mx = dist.global_stats([3.0, 4.0], 17)
        assert counts == [3.0, 4.0] and mx == 17
        assert td.get_backend() == "nccl"
    finally:
        dist.finalize()
        for k in ("RANK", "WORLD_SIZE", "MASTER_PORT"):
            os.environ.pop(k, None)


def test_native_recordio_worker_via_dmlc_submit(tmp_path):
    """BASELINE config 3 end to end, no Python in the worker: dmlc-submit ->
    tracker -> C++ TrackerClient -> rccl id exchange -> RCCL communicator ->
    sharded K7 RecordIO decode -> RCCL all-reduce of the counts."""
    import json
    import os
    import subprocess
    import sys

    from dmlc_core_amd import data

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "build", "dmlc_recordio_dist")
    assert os.path.exists(exe), "build with `make tools` (done by __graft_entry__.build)"
    rec = str(tmp_path / "d.rec")
    data.write_synthetic(rec, 0, 50000, format="recordio", seed=2, record_bytes=200)
    env = dict(os.environ, PYTHONPATH=root)
    p = subprocess.run([sys.executable, "-m", "dmlc_core_amd.parallel.launch.submit",
                        "--cluster", "local", "--num-workers", "1", "--gpus-per-node", "1",
                        "--host-ip", "127.0.0.1", "--timeout", "100", exe, rec, "3", "1", "1"],
                       capture_output=True, text=True, timeout=110, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    out = json.loads(line)
    assert out["records"] == 50000 and out["n_gpus"] == 1
    assert out["payload_bytes"] == 50000 * 200
    assert out["value"] > 0


def test_communicator_aborts_on_tracker_failure():
    """A peer's failure reaches this rank through its heartbeat reply and
    aborts the RCCL communicator (ncclCommAbort); later collectives raise."""
    import threading
    import time

    from dmlc_core_amd.parallel import tracker as trk
    from dmlc_core_amd.parallel.client import TrackerClient

    t = trk.RabitTracker("127.0.0.1", 2, port=19091, port_end=19999, heartbeat_timeout=30.0,
                         timeout=60, abort_grace=2.0)
    t.start(2)
    native = _dmlc.TrackerClient("127.0.0.1", t.port, "n0", -1, -1, 30.0)
    peer = TrackerClient("127.0.0.1", t.port, jobid="p1")
    th = [threading.Thread(target=native.start), threading.Thread(target=peer.start)]
    for x in th:
        x.start()
    for x in th:
        x.join(30)
    comm = _dmlc.Communicator(0, 1, 0, _dmlc.Communicator.new_unique_id())
    comm.abort_on_tracker_failure(native)
    native.start_heartbeat(0.2)
    x = torch.ones(16, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    comm.all_reduce(_ptr(x), _ptr(x), 16, _dmlc.DataType.float32, _dmlc.ReduceOp.sum, s)
    torch.cuda.synchronize()
    peer.abort("injected failure")
    deadline = time.time() + 20
    while not comm.aborted and time.time() < deadline:
        time.sleep(0.05)
    assert comm.aborted
    with pytest.raises(_dmlc.DMLCError, match="aborted"):
        comm.all_reduce(_ptr(x), _ptr(x), 16, _dmlc.DataType.float32, _dmlc.ReduceOp.sum, s)
    native.stop_heartbeat()
    del comm
    with pytest.raises(trk.TrackerError):
        t.join(30)
