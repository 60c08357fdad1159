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
