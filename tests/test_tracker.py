"""Tracker / launcher tests with in-process fake workers:
topology parity with the reference, rank assignment, recover, the new rccl /
barrier / heartbeat commands, dmlc-submit --cluster local end to end, a
gloo process group bootstrapped through the tracker, and the command lines
of the cluster backends (dry run)."""
import os
import subprocess
import sys
import textwrap
import threading
import time

import pytest

from dmlc_core_amd.parallel import tracker as trk
from dmlc_core_amd.parallel.client import TrackerClient

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _reference_link_map(n):
    """The reference algorithm, written out with Python sets (test oracle)."""
    def nbr(r):
        r1 = r + 1
        out = []
        if r1 > 1:
            out.append(r1 // 2 - 1)
        if r1 * 2 - 1 < n:
            out.append(r1 * 2 - 1)
        if r1 * 2 < n:
            out.append(r1 * 2)
        return out
    tree = {r: nbr(r) for r in range(n)}
    parent = {r: (r + 1) // 2 - 1 for r in range(n)}

    def share(r):
        cset = set(tree[r]) - {parent[r]}
        if not cset:
            return [r]
        lst, cnt = [r], 0
        for v in cset:
            sub = share(v)
            cnt += 1
            if cnt == len(cset):
                sub.reverse()
            lst += sub
        return lst
    order = share(0)
    ring = {order[i]: (order[(i - 1) % n], order[(i + 1) % n]) for i in range(n)}
    rmap, k = {0: 0}, 0
    for i in range(n - 1):
        k = ring[k][1]
        rmap[k] = i + 1
    return ({rmap[k]: [rmap[x] for x in v] for k, v in tree.items()},
            {rmap[k]: (-1 if k == 0 else rmap[v]) for k, v in parent.items()},
            {rmap[k]: (rmap[a], rmap[b]) for k, (a, b) in ring.items()})


def test_topology_matches_reference_measurement():
    tree, parent, ring = trk.link_map(8)
    # SURVEY §2.11 [measured] 8-rank output of the reference tracker
    expect = {0: [1, 7], 1: [0, 2, 4], 2: [1, 3], 3: [2], 4: [1], 5: [7], 6: [7], 7: [0, 5, 6]}
    assert {k: sorted(v) for k, v in tree.items()} == expect
    assert ring[0] == (7, 1)
    assert all(ring[r] == ((r - 1) % 8, (r + 1) % 8) for r in range(8))


@pytest.mark.parametrize("n", list(range(1, 40)) + [64, 100, 257])
def test_topology_equals_reference_algorithm(n):
    tree, parent, ring = trk.link_map(n)
    rt, rp, rr = _reference_link_map(n)
    assert {k: sorted(v) for k, v in tree.items()} == {k: sorted(v) for k, v in rt.items()}
    assert parent == rp
    assert ring == rr


def _start_tracker(n, **kw):
    t = trk.RabitTracker("127.0.0.1", n, port=19091, port_end=19999, **kw)
    t.start(n)
    return t


def test_fake_workers_rank_rccl_barrier_print_shutdown():
    n = 6
    t = _start_tracker(n, timeout=60)
    results = {}
    errors = []

    def worker(i):
        try:
            c = TrackerClient("127.0.0.1", t.port, jobid=f"job{i}")
            topo = c.start()
            uid = c.exchange_unique_id(lambda: b"\x01" * 128, key="world")
            c.barrier("b1")
            c.print(f"hello from {topo.rank}")
            c.barrier("b2")
            results[i] = (topo, uid)
            c.shutdown()
        except Exception as e:  # pragma: no cover - surfaced below
            errors.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join(60)
    t.join(30)
    assert not errors, errors
    ranks = sorted(r[0].rank for r in results.values())
    assert ranks == list(range(n))
    assert all(r[1] == b"\x01" * 128 for r in results.values())
    assert all(r[0].world_size == n for r in results.values())
    tree, parent, ring = trk.link_map(n)
    for topo, _ in results.values():
        assert sorted(topo.tree) == sorted(tree[topo.rank])
        assert topo.parent == parent[topo.rank]
    assert len([m for m in t.messages if m.startswith("hello from")]) == n


def test_recover_keeps_rank_by_jobid():
    t = _start_tracker(2, timeout=60)
    out = {}

    def run(i):
        c = TrackerClient("127.0.0.1", t.port, jobid=f"task{i}")
        out[i] = c.start().rank
        if i == 1:
            # restart: a fresh client with the same jobid and its old rank
            c2 = TrackerClient("127.0.0.1", t.port, jobid=f"task{i}", rank=out[i])
            out["re"] = c2.start(recover=True).rank
        c.shutdown()

    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(60)
    t.join(30)
    assert out["re"] == out[1]


def test_attempt_counts_launches_per_task_id():
    """``attempt``: the n-th launch of a task id learns n (0 first), per id,
    and the job's rendezvous is untouched by it"""
    from dmlc_core_amd import _dmlc
    t = _start_tracker(1, timeout=60)
    seen = [TrackerClient("127.0.0.1", t.port, jobid="attempt:worker:3").attempt() for _ in range(2)]
    # the C++ client's twin of the command
    seen.append(_dmlc.TrackerClient("127.0.0.1", t.port, "attempt:worker:3", -1, -1, 30.0).attempt())
    other = TrackerClient("127.0.0.1", t.port, jobid="attempt:worker:4").attempt()
    c = TrackerClient("127.0.0.1", t.port, jobid="w0")
    assert c.start().rank == 0
    c.shutdown()
    t.join(30)
    assert seen == [0, 1, 2] and other == 0


def test_heartbeat_timeout_fails_the_job():
    t = _start_tracker(2, heartbeat_timeout=1.0, timeout=60)
    c0 = TrackerClient("127.0.0.1", t.port)
    c1 = TrackerClient("127.0.0.1", t.port)
    th = [threading.Thread(target=c.start) for c in (c0, c1)]
    for x in th:
        x.start()
    for x in th:
        x.join(30)
    c0.heartbeat()
    c1.heartbeat()
    c1.shutdown()
    # c0 "dies": no more heartbeats and no shutdown
    with pytest.raises(trk.TrackerError, match="missed heartbeats"):
        t.join(30)


def test_job_timeout():
    t = _start_tracker(3, timeout=1.0)
    with pytest.raises(trk.TrackerError, match="did not finish"):
        t.join(30)


WORKER = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {root!r})
    from dmlc_core_amd.parallel.client import TrackerClient
    c = TrackerClient()
    topo = c.start()
    uid = c.exchange_unique_id(lambda: os.urandom(128))
    c.barrier("x")
    c.print("rank=%d task=%s local=%s uid=%s" % (topo.rank, os.environ["DMLC_TASK_ID"],
            os.environ.get("DMLC_LOCAL_RANK"), uid[:4].hex()))
    c.shutdown()
""")


def _submit(args, timeout=240, **extra_env):
    env = dict(os.environ, PYTHONPATH=ROOT, **extra_env)
    return subprocess.run([sys.executable, "-m", "dmlc_core_amd.parallel.launch.submit", *args],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)


def test_submit_local_end_to_end(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(root=ROOT))
    p = _submit(["--cluster", "local", "--num-workers", "4", "--gpus-per-node", "2",
                 "--host-ip", "127.0.0.1", "--timeout", "200", sys.executable, str(script)])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stderr.splitlines() if "rank=" in l]
    assert len(lines) == 4
    uids = {l.split("uid=")[1] for l in lines}
    assert len(uids) == 1  # everyone got rank 0's id
    assert sorted(l.split("local=")[1].split()[0] for l in lines) == ["0", "0", "1", "1"]


TORCH_WORKER = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {root!r})
    import torch
    from dmlc_core_amd.parallel import dist
    info = dist.init("gloo")
    counts, mx = dist.global_stats([1.0, float(info["rank"])], max_index=10 * info["rank"])
    g = dist.all_gather_counts(info["rank"] + 1, 2 * info["rank"])
    model = torch.nn.Linear(4, 1)
    torch.manual_seed(info["rank"])
    red = dist.GradAllReducer(model.parameters(), bucket_mb=0.00001)
    loss = model(torch.randn(8, 4)).sum()
    loss.backward()
    red.synchronize()
    ref = torch.tensor([model.weight.grad.sum().item()])
    import torch.distributed as td
    allg = [torch.zeros(1) for _ in range(info["world_size"])]
    td.all_gather(allg, ref)
    assert all(torch.allclose(a, ref) for a in allg), "grads differ across ranks"
    assert counts[0] == info["world_size"], counts
    assert mx == 10 * (info["world_size"] - 1)
    assert [x[0] for x in g] == list(range(1, info["world_size"] + 1))
    print("OK", info["rank"], flush=True)
    dist.finalize()
""")


def test_gloo_process_group_via_tracker(tmp_path):
    script = tmp_path / "t.py"
    script.write_text(TORCH_WORKER.format(root=ROOT))
    p = _submit(["--cluster", "local", "--num-workers", "3", "--host-ip", "127.0.0.1",
                 "--timeout", "200", sys.executable, str(script)])
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert p.stdout.count("OK") == 3


def test_gloo_process_group_via_torch_env(tmp_path):
    script = tmp_path / "t.py"
    script.write_text(TORCH_WORKER.format(root=ROOT).replace(
        'info = dist.init("gloo")',
        'os.environ.pop("DMLC_TRACKER_URI"); info = dist.init("gloo")\n'
        'c = __import__("dmlc_core_amd.parallel.client", fromlist=["x"]).TrackerClient()\n'
        'c.rank = info["rank"]'))
    # the tracker still needs a shutdown per rank: send it from the worker
    script.write_text(script.read_text().replace(
        "dist.finalize()", "dist.finalize(); c.shutdown()"))
    p = _submit(["--cluster", "local", "--num-workers", "2", "--torch-env", "1",
                 "--host-ip", "127.0.0.1", "--timeout", "200", sys.executable, str(script)])
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    assert p.stdout.count("OK") == 2


@pytest.mark.parametrize("cluster,needle", [
    ("mpi", "mpirun -n 4"),
    ("slurm", "srun --share --exclusive=user"),
    ("sge", "qsub -cwd -t 1-4"),
    ("mesos", "mesos-execute"),
    ("kubernetes", "amd.com/gpu"),
    ("yarn", '"number_of_containers": 4'),  # the Services spec (no hadoop jar mode)
    ("local", "DMLC_LOCAL_RANK=1"),
])
def test_backend_dry_run(cluster, needle, tmp_path):
    args = ["--cluster", cluster, "--num-workers", "4", "--gpus-per-node", "8", "--dry-run",
            "--env", "FOO=bar", "echo", "hi"]
    if cluster == "mesos":
        args = ["--mesos-master", "m:5050"] + args
    rm = {"YARN_RM_ADDRESS": "http://rm.invalid:8088"} if cluster == "yarn" else {}
    p = _submit(args, timeout=120, **rm)
    assert p.returncode == 0, p.stderr[-2000:]
    assert needle in p.stdout
    assert "FOO" in p.stdout


@pytest.mark.parametrize("nworker,gpus,per_rank", [(12, 8, False), (8, 8, False), (3, 8, True),
                                                     (5, 0, False)])
def test_kubernetes_one_process_per_gpu(nworker, gpus, per_rank):
    """Worker pods never request more GPUs than they run ranks: pod-per-node
    (G GPUs, G ranks started inside the pod with local ranks 0..G-1) or
    pod-per-rank (1 GPU, local rank 0).  The pod command is run through bash
    for every completion index: the task ids cover 0..N-1 once each."""
    import subprocess
    from dmlc_core_amd.parallel.launch import kubernetes
    from dmlc_core_amd.parallel.launch.opts import get_opts
    argv = ["--cluster", "kubernetes", "--num-workers", str(nworker), "--gpus-per-node", str(gpus),
            "--num-servers", "1"]
    if per_rank:
        argv += ["--kube-pod-per-rank", "1"]
    args = get_opts(argv + ["echo", "hi"])
    ms = kubernetes.manifests(args, {}, 'echo "$DMLC_TASK_ID ${DMLC_LOCAL_RANK:-none}"')
    worker = ms[0]
    pods = worker["spec"]["completions"]
    c = worker["spec"]["template"]["spec"]["containers"][0]
    req = c["resources"]["limits"].get("amd.com/gpu", 0)
    seen = []
    for idx in range(pods):
        out = subprocess.run(["bash", "-c", c["command"][2]], capture_output=True, text=True,
                             env=dict(os.environ, JOB_COMPLETION_INDEX=str(idx)), check=True).stdout
        ranks = [l.split() for l in out.splitlines()]
        assert len(ranks) <= max(req, 1)  # no pod runs fewer ranks than GPUs it asked for... nor more
        seen += ranks
    assert sorted(int(t) for t, _ in seen) == list(range(nworker))
    if gpus == 0:
        assert req == 0 and pods == nworker and all(l == "none" for _, l in seen)
    elif per_rank:
        assert req == 1 and pods == nworker and all(l == "0" for _, l in seen)
    else:
        assert pods == -(-nworker // gpus) and req == min(gpus, nworker)
        assert sorted(int(l) for t, l in seen if int(t) < gpus) == list(range(min(gpus, nworker)))
    server = ms[2]["spec"]["template"]["spec"]["containers"][0]
    assert "amd.com/gpu" not in server["resources"]["limits"]


def test_ssh_dry_run(tmp_path):
    hf = tmp_path / "hosts"
    hf.write_text("10.0.0.1\n10.0.0.2:2222\n")
    p = _submit(["--cluster", "ssh", "--num-workers", "4", "--host-file", str(hf), "--dry-run",
                 "--gpus-per-node", "8", "echo", "hi"], timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("ssh")]
    assert len(lines) == 4
    assert sum("10.0.0.2" in l and "-p 2222" in l for l in lines) == 2


def test_native_cpp_client_against_python_tracker():
    from dmlc_core_amd import _dmlc
    n = 4
    t = _start_tracker(n, timeout=60)
    out, errors = {}, []

    def worker(i):
        try:
            c = _dmlc.TrackerClient("127.0.0.1", t.port, f"cpp{i}", -1, -1, 30.0)
            rank, parent, world, tree, prev, nxt = c.start()
            if rank == 0:
                c.rccl_put("world", b"\x07" * 128)
                uid = b"\x07" * 128
            else:
                uid = c.rccl_get("world")
            c.barrier("cpp")
            c.print(f"cpp rank {rank}")
            out[i] = (rank, parent, world, sorted(tree), prev, nxt, uid)
            c.shutdown()
        except Exception as e:  # pragma: no cover
            errors.append(e)

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join(60)
    t.join(30)
    assert not errors, errors
    tree, parent, ring = trk.link_map(n)
    assert sorted(v[0] for v in out.values()) == list(range(n))
    for rank, par, world, tr, prev, nxt, uid in out.values():
        assert world == n and par == parent[rank] and tr == sorted(tree[rank])
        assert (prev, nxt) == ring[rank]
        assert uid == b"\x07" * 128


def _start_two(**kw):
    t = _start_tracker(2, **kw)
    c0 = TrackerClient("127.0.0.1", t.port)
    c1 = TrackerClient("127.0.0.1", t.port)
    th = [threading.Thread(target=c.start) for c in (c0, c1)]
    for x in th:
        x.start()
    for x in th:
        x.join(30)
    return t, c0, c1


def test_dead_rank_is_signalled_to_live_ranks():
    """Failure propagation: rank 1 stops heartbeating; rank 0's
    heartbeat thread learns the job failed (so it can abort its RCCL
    communicator) before the tracker gives up."""
    t, c0, c1 = _start_two(heartbeat_timeout=1.0, timeout=60)
    got = []
    done = threading.Event()
    c1.heartbeat()  # c1 is alive once, then "dies"

    def on_failure(reason):
        got.append(reason)
        done.set()

    c0.start_heartbeat(0.2, on_failure)
    assert done.wait(20), "live rank never heard of the failure"
    assert "rank 1 missed heartbeats" in got[0] or "rank" in got[0]
    c0.stop_heartbeat()
    with pytest.raises(trk.TrackerError, match="missed heartbeats"):
        t.join(30)


def test_abort_command_fails_job_fast():
    t, c0, c1 = _start_two(heartbeat_timeout=30.0, timeout=60, abort_grace=1.0)
    assert c0.heartbeat() is None
    c1.abort("CUDA-free error")
    reason = c0.heartbeat()
    # ranks go to concurrent starters in arrival order: use the one c1 got
    assert reason is not None and f"rank {c1.rank} aborted: CUDA-free error" in reason
    with pytest.raises(trk.TrackerError, match="aborted"):
        t.join(30)


def test_native_client_heartbeat_abort_and_failure_handler():
    from dmlc_core_amd import _dmlc
    t = _start_tracker(2, heartbeat_timeout=30.0, timeout=60, abort_grace=1.0)
    cs = [_dmlc.TrackerClient("127.0.0.1", t.port, f"n{i}", -1, -1, 30.0) for i in range(2)]
    th = [threading.Thread(target=c.start) for c in cs]
    for x in th:
        x.start()
    for x in th:
        x.join(30)
    assert cs[0].heartbeat() is None
    cs[1].abort("disk full")
    assert "disk full" in cs[0].heartbeat()
    with pytest.raises(trk.TrackerError, match="disk full"):
        t.join(30)


def test_slow_start_negotiation_does_not_stall_heartbeats():
    """A worker stuck in `start` link negotiation must not starve other ranks'
    heartbeats (each connection has its own handler thread)."""
    import socket
    import time
    t = _start_tracker(3, heartbeat_timeout=1.0, timeout=60)
    c0 = TrackerClient("127.0.0.1", t.port, rank=0, world_size=3)
    c1 = TrackerClient("127.0.0.1", t.port, rank=1, world_size=3)
    c0.start()
    c1.start()
    stop = threading.Event()

    def beat():
        while not stop.is_set():
            c0.heartbeat()
            c1.heartbeat()
            time.sleep(0.2)

    hb = threading.Thread(target=beat)
    hb.start()
    # rank 2 opens `start`, reads its topology, then stalls for 3x the timeout
    ch = trk.Channel(socket.create_connection(("127.0.0.1", t.port), timeout=30))
    ch.send_int(trk.MAGIC)
    assert ch.recv_int() == trk.MAGIC
    ch.send_int(2)
    ch.send_int(3)
    ch.send_str("slow")
    ch.send_str("start")
    assert ch.recv_int() == 2
    ch.recv_int()  # parent
    ch.recv_int()  # world
    for _ in range(ch.recv_int()):
        ch.recv_int()
    links = {ch.recv_int(), ch.recv_int()} - {-1}
    time.sleep(3.0)
    ch.send_int(len(links))
    for r in links:
        ch.send_int(r)
    nconn = ch.recv_int()
    ch.recv_int()
    for _ in range(nconn):
        ch.recv_str()
        ch.recv_int()
        ch.recv_int()
    ch.send_int(0)
    ch.send_int(0)
    ch.close()
    stop.set()
    hb.join(10)
    c2 = TrackerClient("127.0.0.1", t.port, rank=2, world_size=3)
    for c in (c0, c1, c2):
        c.shutdown()
    t.join(30)  # no "missed heartbeats" failure
    assert t.error is None
