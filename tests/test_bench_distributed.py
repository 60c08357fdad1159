"""The headline bench's distributed flow on CPU (gloo): launched by dmlc-submit
(tracker-assigned ranks, tracker-brokered process group) and by torchrun (the
driver's launcher).  Every rank parses its own byte-range shard; the shards
are disjoint and complete (their rows sum to the dataset's), and rank 0 prints
one JSON line with the per-rank view."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROWS = 20000


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert lines, out[-3000:]
    return json.loads(lines[-1])


def _check(res, world):
    assert res["config"]["rows"] == ROWS
    assert res["steps"] == 2 and res["warmup"] == 1
    pr = res["per_rank"]
    assert [p["rank"] for p in pr] == list(range(world))
    assert sum(p["rows"] for p in pr) == ROWS  # complete, and disjoint
    assert all(p["rows"] > 0 for p in pr)
    assert res["value"] > 0


@pytest.mark.parametrize("world", [2, 4])
def test_bench_via_dmlc_submit_cpu(tmp_path, world):
    env = dict(os.environ, PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1")
    cmd = [sys.executable, "-m", "dmlc_core_amd.parallel.launch.submit", "--cluster", "local",
           "--num-workers", str(world), "--host-ip", "127.0.0.1", "--timeout", "240",
           sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus",
           str(world), "--rows", str(ROWS), "--steps", "2", "--warmup", "1", "--data-dir",
           str(tmp_path)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    _check(_last_json(p.stdout), world)


def test_bench_via_torchrun_cpu(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29611", os.path.join(ROOT, "bench.py"),
           "--device", "cpu", "--gpus", "2", "--rows", str(ROWS), "--steps", "2", "--warmup",
           "1", "--data-dir", str(tmp_path)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    _check(_last_json(p.stdout), 2)


def test_bench_self_launches_ranks_cpu(tmp_path):
    """`python bench.py --gpus 4` with no launcher in the environment starts 4
    tracker-launched ranks itself (the driver's N>1 contract), reports
    n_gpus == 4 and never loads the HIP runtime in the launching process."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "DMLC_TRACKER_URI", "DMLC_TRACKER_PORT")}
    env.update(PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1", DMLC_BENCH_CHECK_MAPS="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "4",
           "--rows", str(ROWS), "--steps", "2", "--warmup", "1", "--data-dir", str(tmp_path)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    res = _last_json(p.stdout)
    assert res["n_gpus"] == 4
    assert len(res["per_rank"]) == 4
    _check(res, 4)
    assert "bench launcher: libamdhip64 mapped = False" in p.stderr, p.stderr[-2000:]
    # exactly one JSON line (rank 0's)
    assert sum(1 for l in p.stdout.splitlines() if l.startswith("{")) == 1


def test_bench_rejects_world_mismatch(tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29613", os.path.join(ROOT, "bench.py"),
           "--device", "cpu", "--gpus", "3", "--rows", str(ROWS), "--steps", "1", "--warmup",
           "0", "--data-dir", str(tmp_path)]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode != 0
    assert "--gpus 3 but the launcher started a world of 2" in p.stderr
