"""Two GPU processes against one MI355X: the only pre-scale check of
concurrent hipHostRegister windows, concurrent zero-copy DMA and per-process
HIP state available on a one-GPU box.  Two tracker-launched ranks share
cuda:0 (gloo control plane); their shards must be disjoint and complete and
each must equal the CPU parser's shard."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from dmlc_core_amd import data

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_ranks_share_one_gpu(tmp_path):
    path = str(tmp_path / "d.libsvm")
    data.write_synthetic(path, 0, 60000, format="libsvm", seed=21)  # ~38 MB
    out = str(tmp_path / "ranks.json")
    env = dict(os.environ, PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1")
    cmd = [sys.executable, "-m", "dmlc_core_amd.parallel.launch.submit", "--cluster", "local",
           "--num-workers", "2", "--gpus-per-node", "1", "--host-ip", "127.0.0.1",
           "--timeout", "150", "--auto-file-cache", "0", sys.executable, "-u",
           os.path.join(ROOT, "tests", "two_rank_gpu_worker.py"), path, out]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=180, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    res = json.load(open(out))
    ranks = sorted(res["ranks"])
    assert [r[0] for r in ranks] == [0, 1]
    assert all(r[1] > 0 for r in ranks)
    cpu = list(data.iter_blocks(path, 0, 1, "libsvm"))
    rows = sum(len(b["label"]) for b in cpu)
    nnz = sum(len(b["index"]) for b in cpu)
    csum = int(sum(b["index"].astype(np.uint64).sum() for b in cpu))
    assert sum(r[1] for r in ranks) == rows  # complete and disjoint
    assert sum(r[2] for r in ranks) == nnz
    assert sum(r[3] for r in ranks) == csum


@pytest.mark.parametrize("mode", ["stream", "cache"])
def test_bench_share_gpu_two_ranks(tmp_path, mode):
    """bench.py's own multi-rank GPU branch (launcher -> tracker ranks ->
    per-world dataset -> NUMA binding -> barriers -> NumCol all-reduce ->
    per-rank gather -> all-reduce probe), two ranks on GPU 0 over gloo: the
    JSON line a SCALE run prints, with rows summing to the dataset."""
    env = dict(os.environ, PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu",
           "--steps", "2", "--warmup", "1", "--rows", "120000", "--mode", mode,
           "--data-dir", str(tmp_path / "bench")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["config"]["rows"] == 120000 and out["config"]["global_batch"] == 120000
    assert "all ranks on GPU 0" in out["config"]["parallelism"]
    assert sorted(r["rank"] for r in out["per_rank"]) == [0, 1]
    assert sum(r["rows"] for r in out["per_rank"]) == 120000
    probe = out["allreduce_busbw_GBps"]
    assert probe["backend"] == "gloo" and probe["4MB"] > 0 and probe["256MB"] > 0


@pytest.mark.timeout(330)
def test_bench_share_gpu_eight_ranks(tmp_path):
    """The world-8 rehearsal on one GPU: bench.py --gpus 8 --share-gpu starts
    8 tracker ranks on GPU 0 (gloo control plane), the shape of the driver's
    8-GPU SCALE run.  Per-rank rows sum to the dataset, the all-reduce probe
    reports, and the zero-copy pin budget is shared: every rank's budget is
    the host budget / 8 (or less, by MemAvailable) and no rank pinned more
    than its budget -- 8 ranks never lock 8 x the host budget."""
    env = dict(os.environ, PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "8", "--share-gpu",
           "--steps", "2", "--warmup", "1", "--rows", "400000",
           "--data-dir", str(tmp_path / "bench")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert out["n_gpus"] == 8 and out["config"]["rows"] == 400000
    ranks = out["per_rank"]
    assert sorted(r["rank"] for r in ranks) == list(range(8))
    assert sum(r["rows"] for r in ranks) == 400000
    assert all(r["rows"] > 0 for r in ranks)
    probe = out["allreduce_busbw_GBps"]
    assert probe["backend"] == "gloo" and probe["4MB"] > 0
    host_budget = 64 << 30  # DeviceParserConfig::zc_pin_budget
    for r in ranks:
        assert 0 < r["zc_pin_budget"] <= host_budget // 8
        assert 0 < r["zc_pinned_peak"] <= r["zc_pin_budget"]
        assert r["last_pass_sec"] > 0 and 0 < r["last_fill_sec"] <= r["last_pass_sec"]
    assert sum(r["zc_pinned_peak"] for r in ranks) <= host_budget


@pytest.mark.timeout(300)
@pytest.mark.parametrize("mode", ["stream", "hbm"])
def test_bench_two_gpus_over_rccl(tmp_path, mode):
    """bench.py --gpus 2 on two real GPUs (no --share-gpu): the control plane
    and the NumCol / gradient all-reduce run over RCCL (backend "nccl"), one
    process per GPU.  Skipped where fewer than two GPUs are visible (the
    one-GPU box); the driver's 8-GPU SCALE run takes the same branch."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("needs >= 2 GPUs (RCCL at world 2)")
    env = dict(os.environ, PYTHONPATH=ROOT, DMLC_HEARTBEAT_PERIOD="1")
    cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2",
           "--steps", "2", "--warmup", "1", "--rows", "200000", "--mode", mode,
           "--data-dir", str(tmp_path / "bench")]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=280, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-5000:]
    out = json.loads([x for x in p.stdout.splitlines() if x.startswith("{")][-1])
    assert out["n_gpus"] == 2 and out["config"]["rows"] == 200000
    assert "all ranks on GPU 0" not in out["config"]["parallelism"]
    ranks = out["per_rank"]
    assert sorted(r["rank"] for r in ranks) == [0, 1]
    assert sum(r["rows"] for r in ranks) == 200000
    probe = out["allreduce_busbw_GBps"]
    assert probe["backend"] == "nccl" and probe["4MB"] > 0 and probe["256MB"] > 0
