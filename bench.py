#!/usr/bin/env python3
"""Headline benchmark: LibSVM text -> CSR RowBlocks in MI355X HBM.

Metric (BASELINE.json): parsed rows/sec (LibSVM->CSR) with host->device GB/s,
at 1/2/4/8 MI355X.  Config: synthetic 10M-row sparse LibSVM dataset (20-60
nnz/row, ~640 B/line, ~6.4 GB) generated deterministically into 16 part files;
random content, same shape as the reference measurement.

One step = one full epoch over this rank's InputSplit shard (byte-range
sharding, part=rank of nparts=world): parallel pread from the page cache into
the pinned ring -> hipMemcpyAsync -> HIP line-index/count/scan/fill kernels ->
whole-shard CSR resident in HBM -> RCCL all-reduce of (rows, nnz, max index)
for the global NumCol.  Nothing is cached between steps: every step re-reads
and re-parses the text.  Total work is fixed as N grows (strong scaling).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
       dmlc-submit --cluster local --num-workers N --gpus-per-node N python bench.py --gpus N
         (the dmlc tracker assigns ranks and bootstraps the RCCL/gloo group)

With ``--gpus N > 1`` and no launcher in the environment, this process is only
a launcher: before touching torch or the HIP runtime it starts the N ranks
through ``dmlc-submit --cluster local`` (reference
`tracker/dmlc_tracker/local.py:47-72`), forwards their output (rank 0's JSON
line) and exits with their status.  Every rank checks that the world it joined
has exactly ``--gpus`` ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_ROWS_PER_SEC = 2.20e6  # reference CPU parser, 8 threads
NUM_PARTS = 16

# per format: the reference number it is compared with (measured
# CPU reference), the metric name and the default dataset size
# same-host CPU baseline (profiles/r05_cpu): the reference's own parsers built
# from source and run on the MI355X box's CPU (2 x EPYC 9575F; 16 CPUs = one
# GPU's share), best-of runs; recorded, not re-measured per bench run
SAME_HOST_CPU = {
    "libsvm": {"ref_8t": 7.105e6, "ref_16t": 13.631e6},
    "libfm": {"ref_8t": 5.394e6, "ref_16t": 9.932e6},
    "csv": {"ref_8t": 13.057e6, "ref_16t": 24.528e6},
    "recordio": {"ref_1t": 57.477e6},
}

FORMATS = {
    "libsvm": dict(baseline=2.201e6, rows=10_000_000,
                   metric="parsed rows/sec (LibSVM->CSR in device memory), aggregate over GPUs",
                   model="LibSVM tokenize -> device CSR RowBlock (synthetic 10M-row sparse file)",
                   dtype="fp32 values / u32 indices (text parse, no matmul)"),
    "libfm": dict(baseline=1.954e6, rows=10_000_000,
                  metric="parsed rows/sec (LibFM->CSR in device memory), aggregate over GPUs",
                  model="LibFM tokenize -> device CSR RowBlock with fields (synthetic 10M rows)",
                  dtype="fp32 values / u32 indices and fields (text parse, no matmul)"),
    "csv": dict(baseline=6.61e6, rows=10_000_000,
                metric="parsed rows/sec (CSV->CSR in device memory, label_column=0), aggregate over GPUs",
                model="CSV (29 columns) -> device CSR RowBlock (synthetic 10M rows)",
                dtype="fp32 values / u32 indices (text parse, no matmul)"),
    "recordio": dict(baseline=11.31e6, rows=4_000_000,
                     metric="decoded records/sec (RecordIO -> device byte-CSR), aggregate over GPUs",
                     model="RecordIO decode (4M x 512 B records, 1/64 multi-part) -> HBM byte-CSR",
                     dtype="raw bytes (u64 offsets)"),
}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--format", default="libsvm", choices=sorted(FORMATS),
                    help="libsvm (the BASELINE headline), libfm, csv or recordio")
    ap.add_argument("--rows", type=int, default=0, help="0: the format's default size")
    ap.add_argument("--data-dir", default=os.environ.get("DMLC_BENCH_DIR", "/tmp/dmlc_bench"))
    ap.add_argument("--chunk-mb", type=int, default=64)
    ap.add_argument("--read-threads", type=int, default=0, help="0: auto")
    ap.add_argument("--pinned-slots", type=int, default=4)
    ap.add_argument("--device-slots", type=int, default=3)
    ap.add_argument("--device", choices=["auto", "gpu", "cpu"], default="auto")
    ap.add_argument("--zero-copy", default="auto", choices=["auto", "0", "1"],
                    help="mmap + hipHostRegister the shard (DMA from page cache)")
    ap.add_argument("--mode", default="stream", choices=["stream", "hbm", "cache"],
                    help="stream: every step re-reads the text from the page cache over PCIe; "
                         "hbm: HBM epoch cache -- the warmup epoch keeps the text resident in "
                         "HBM and timed epochs parse it from there (kernel-bound); "
                         "cache: the `#cache` binary page file (DiskRowIter format, built once "
                         "from a GPU parse) is DMA'd zero-copy into the device CSR every step")
    ap.add_argument("--replay-first-mb", type=float, default=None,
                    help="HBM replay: first merged chunk (0: no ramp; default: the parser's)")
    ap.add_argument("--replay-chunk-mb", type=float, default=None,
                    help="HBM replay: merged chunk cap (default: the parser's)")
    ap.add_argument("--no-prelaunch", action="store_true",
                    help="HBM replay: count + scan in line (no second stream), to price kernels alone")
    ap.add_argument("--one-pass", action="store_true",
                    help="HBM replay: one launch per chunk (look-back fill, no count kernel)")
    ap.add_argument("--shape", default="uniform", choices=["uniform", "skewed", "mixed"],
                    help="synthetic row shape (dmlc/synthetic.h): uniform 20-60 tokens of "
                         "0.dddddd; skewed power-law tokens per line (some lines > 8 KiB), "
                         "Zipf-like ids; mixed = skewed + exponent / long / integer / "
                         "valueless values, weights and qid")
    ap.add_argument("--shuffle-parts", type=int, default=1,
                    help="K > 1: shuffled epochs (InputSplitShuffle's GPU twin: K sub-shards per "
                         "rank visited in a new order every epoch, one pipeline)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="every rank uses GPU 0 (gloo control plane): rehearses the multi-rank "
                         "GPU branch on a one-GPU box (RCCL refuses two ranks on one device)")
    args = ap.parse_args()
    if args.rows <= 0:
        args.rows = FORMATS[args.format]["rows"]
    return args


def dataset_dir(args, world: int) -> str:
    # one copy per world size: the page cache of a part lives on the NUMA node
    # of the rank that wrote it, which must be the rank that reads it
    shape = "" if args.shape == "uniform" else f"_{args.shape}"
    return os.path.join(args.data_dir,
                        f"{args.format}_{args.rows}r_{NUM_PARTS}p_seed0{shape}_w{world}")


def ensure_dataset(args, rank: int, world: int, barrier) -> str:
    """Rank r writes the parts its byte-range shard covers (parts
    [16r/N, 16(r+1)/N) for N | 16), so their page-cache pages are first-touched
    on its GPU's NUMA node; a .done marker per part.  The content depends only
    on --rows (deterministic row ranges), never on N."""
    import shutil

    from dmlc_core_amd.data import write_synthetic

    d = dataset_dir(args, world)
    if rank == 0 and os.path.isdir(args.data_dir):
        prefix = f"{args.format}_"
        for name in os.listdir(args.data_dir):
            if name.startswith(prefix) and os.path.join(args.data_dir, name) != d:
                shutil.rmtree(os.path.join(args.data_dir, name), ignore_errors=True)
    barrier()
    os.makedirs(d, exist_ok=True)
    per = (args.rows + NUM_PARTS - 1) // NUM_PARTS
    nthread = max(1, min(16, len(os.sched_getaffinity(0))))
    for p in range(NUM_PARTS):
        if p * world // NUM_PARTS != rank:
            continue
        path = os.path.join(d, f"part-{p:05d}.{args.format}")
        done = path + ".done"
        if os.path.exists(done):
            continue
        b, e = p * per, min(args.rows, (p + 1) * per)
        tmp = path + f".tmp{rank}"
        write_synthetic(tmp, b, e, format=args.format, seed=0, nthread=nthread,
                        shape=args.shape if args.format != "recordio" else "uniform")
        os.replace(tmp, path)
        open(done, "w").close()
    barrier()
    return d


def _launcher_present() -> bool:
    env = os.environ
    return ("RANK" in env and "WORLD_SIZE" in env) or "DMLC_TRACKER_URI" in env


def _parent_maps_hip() -> bool:
    try:
        with open("/proc/self/maps") as f:
            return "libamdhip64" in f.read()
    except OSError:
        return False


def launch_ranks(args) -> int:
    """Start --gpus ranks via dmlc-submit (tracker-assigned ranks, one process
    per GPU bound by local index) and wait for them.  Runs with neither torch
    nor the native extension imported: a process that has initialised the GPU
    must not fork/exec the ranks."""
    import shlex
    import subprocess

    n = args.gpus
    child = [sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:]
    per_node = 1 if args.share_gpu else n  # share-gpu: every rank's local index is 0
    cmd = [sys.executable, "-m", "dmlc_core_amd.parallel.launch.submit", "--cluster", "local",
           "--num-workers", str(n), "--gpus-per-node", str(per_node), "--host-ip", "127.0.0.1",
           "--auto-file-cache", "0"] + [shlex.quote(c) for c in child]
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    rc = subprocess.call(cmd, env=env, cwd=ROOT)
    if os.environ.get("DMLC_BENCH_CHECK_MAPS") == "1":
        print(f"bench launcher: libamdhip64 mapped = {_parent_maps_hip()}", file=sys.stderr)
    return rc


def allreduce_probe(dist, cdev, world: int, sizes=(4 << 20, 256 << 20), iters: int = 5):
    """All-reduce bus bandwidth of the bench's process group, measured after
    the timed region: f32 buffers of 4 MB and 256 MB, 2 untimed + `iters` timed
    calls each; busbw = 2 (n - 1) / n * bytes / t (the ring's per-link load,
    what xGMI's point-to-point links bound).  Under gloo (--share-gpu) the
    buffers live on the host and the number describes the control plane."""
    import torch

    out = {"backend": dist.get_backend(), "device": cdev.type}
    for nbytes in sizes:
        x = torch.ones(nbytes // 4, dtype=torch.float32, device=cdev)
        for _ in range(2):
            dist.all_reduce(x)
        if cdev.type == "cuda":
            torch.cuda.synchronize(cdev)
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(iters):
            dist.all_reduce(x)
        if cdev.type == "cuda":
            torch.cuda.synchronize(cdev)
        t = (time.perf_counter() - t0) / iters
        # the slowest rank's time is the collective's time
        tt = torch.tensor([t], dtype=torch.float64, device=cdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        t = float(tt.item())
        out[f"{nbytes >> 20}MB"] = round(2 * (world - 1) / world * nbytes / t / 1e9, 2)
        del x
    return out


def main():
    args = parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and not _launcher_present():
        sys.exit(launch_ranks(args))

    import torch

    from dmlc_core_amd.parallel import dist as ddist

    use_gpu = args.device == "gpu" or (args.device == "auto" and torch.cuda.is_available())
    # torchrun (RANK/WORLD_SIZE/MASTER_*) or dmlc-submit (DMLC_TRACKER_URI/PORT:
    # the tracker assigns the rank and brokers the process-group address)
    info = ddist.init("nccl" if use_gpu and not args.share_gpu else "gloo")
    rank, world, local_rank = info["rank"], info["world_size"], info["local_rank"]
    if args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started a world of "
                         f"{world} rank(s)")
    dist = None
    if world > 1:
        import torch.distributed as dist  # noqa: F811
    if use_gpu:
        torch.cuda.set_device(local_rank)

    dev = torch.device("cuda", local_rank) if use_gpu else torch.device("cpu")
    # collectives run on the process group's device: the GPU under RCCL, the
    # host under gloo (--share-gpu, or no GPU)
    cdev = dev if use_gpu and not args.share_gpu else torch.device("cpu")
    numa = {"numa_node": -1}
    if use_gpu:
        from dmlc_core_amd.parallel.affinity import bind_to_gpu

        numa = bind_to_gpu(local_rank)

    def barrier():
        if dist is not None:
            if cdev.type == "cuda":
                dist.barrier(device_ids=[local_rank])
            else:
                dist.barrier()

    def sync():
        if use_gpu:
            torch.cuda.synchronize()

    from dmlc_core_amd import data

    ddir = ensure_dataset(args, rank, world, barrier)
    read_threads = args.read_threads or max(4, min(16, len(os.sched_getaffinity(0))))

    local = {}  # this rank's own counters, gathered to rank 0 after timing
    if args.mode == "hbm" and args.warmup < 1:
        raise SystemExit("--mode hbm needs --warmup >= 1 (the warmup epoch fills the cache)")
    if use_gpu and args.format == "recordio":
        from dmlc_core_amd import io as dio

        rextra = {} if args.replay_chunk_mb is None else {"replay_chunk_mb": args.replay_chunk_mb}
        if args.one_pass:
            rextra["one_pass"] = 1
        parser = dio.GPURecordIO(ddir, rank, world, chunk_mb=args.chunk_mb,
                                 device_slots=args.device_slots, pinned_slots=args.pinned_slots,
                                 zero_copy=args.zero_copy, device=local_rank,
                                 hbm_cache=int(args.mode == "hbm"), **rextra)

        def step():
            parser.before_first()
            b = parser.read_all()
            local["rows"], local["bytes"] = b["size"], parser.partition_bytes
            return b["size"], b["bytes"], 0, parser.partition_bytes
    elif use_gpu and args.mode == "cache":
        extra = {"label_column": 0} if args.format == "csv" else {}
        # beside the dataset directory, never inside it (the parser reads every
        # file of the directory)
        cache_path = os.path.join(args.data_dir,
                                  f"rowcache_{os.path.basename(ddir)}_r{rank}of{world}.bin")
        if not os.path.exists(cache_path):
            build = data.GPUParser(ddir, rank, world, format=args.format, chunk_mb=args.chunk_mb,
                                   read_threads=read_threads, device=local_rank,
                                   zero_copy=args.zero_copy, **extra)
            tmp = data.DeviceCSR()
            build.parse_all(tmp)
            data.write_page_cache(tmp, cache_path + ".tmp")
            os.replace(cache_path + ".tmp", cache_path)
            del build, tmp
        parser = data.PageCache(cache_path, device=local_rank)
        csr = data.DeviceCSR()

        def step():
            parser.load(csr)
            local["rows"], local["bytes"] = csr.rows, parser.bytes
            return csr.rows, csr.nnz, csr.max_index, parser.bytes
    elif use_gpu:
        extra = {"label_column": 0} if args.format == "csv" else {}
        if args.replay_first_mb is not None:
            extra["replay_first_mb"] = args.replay_first_mb
        if args.replay_chunk_mb is not None:
            extra["replay_chunk_mb"] = args.replay_chunk_mb
        if args.one_pass:
            extra["one_pass"] = 1
        if args.no_prelaunch:
            extra["prelaunch"] = 0
        parser = data.GPUParser(ddir, rank, world, format=args.format, chunk_mb=args.chunk_mb,
                                read_threads=read_threads, pinned_slots=args.pinned_slots,
                                device_slots=args.device_slots, device=local_rank,
                                zero_copy=args.zero_copy,
                                hbm_cache=int(args.mode == "hbm"),
                                shuffle_parts=args.shuffle_parts, **extra)
        csr = data.DeviceCSR()

        def step():
            parser.before_first()
            csr.clear()
            parser.parse_all(csr)
            local["rows"], local["bytes"] = csr.rows, parser.partition_bytes
            return csr.rows, csr.nnz, csr.max_index, parser.partition_bytes
    elif args.format == "recordio":
        from dmlc_core_amd import io as dio

        def step():
            split = dio.InputSplit(ddir, rank, world, "recordio")
            n = nbytes = 0
            while True:
                rec = split.next_record()
                if rec is None:
                    break
                n += 1
                nbytes += len(rec)
            local["rows"], local["bytes"] = n, nbytes
            return n, nbytes, 0, nbytes
    else:
        uri = ddir + f"?format={args.format}" + ("&label_column=0" if args.format == "csv" else "")

        def step():
            p = data.Parser(uri, rank, world, args.format)
            rows, nnz, _ = p.drain()
            local["rows"], local["bytes"] = rows, p.bytes_read()
            return rows, nnz, 0, p.bytes_read()

    def global_counts(rows, nnz, max_index, nbytes):
        if dist is None:  # one rank: the totals are its own (no device round trip)
            return [float(rows), float(nnz), float(nbytes)], int(max_index)
        t = torch.tensor([rows, nnz, nbytes], dtype=torch.float64, device=cdev)
        m = torch.tensor([max_index], dtype=torch.float64, device=cdev)
        dist.all_reduce(t)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        return t.tolist(), int(m.item())

    for _ in range(args.warmup):
        r = step()
        global_counts(*r)
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    totals = None
    for _ in range(args.steps):
        r = step()
        totals = global_counts(*r)
    sync()
    barrier()
    sync()
    elapsed = time.perf_counter() - t0
    # per-rank view (rows, bytes, own time, host waits) gathered to every rank
    st = parser.stats() if use_gpu and args.mode != "cache" else {}
    mine = torch.tensor([rank, local["rows"], local["bytes"], elapsed,
                         st.get("wait_reader_sec", 0.0), st.get("wait_gpu_sec", 0.0),
                         st.get("zc_pin_budget", 0), st.get("zc_pinned_peak", 0),
                         st.get("last_fill_sec", 0.0), st.get("last_drain_sec", 0.0),
                         st.get("last_pass_sec", 0.0)],
                        dtype=torch.float64, device=cdev)
    gathered = [torch.zeros_like(mine) for _ in range(world)]
    if dist is not None:
        dist.all_gather(gathered, mine)
    else:
        gathered = [mine]
    per_rank = []
    for g in sorted((x.tolist() for x in gathered), key=lambda v: v[0]):
        r, rows_r, bytes_r, el_r, wr, wg, pin_b, pin_p, fill_s, drain_s, pass_s = g
        per_rank.append({"rank": int(r), "rows": int(rows_r), "bytes": int(bytes_r),
                         "rows_per_sec": round(rows_r * args.steps / el_r, 1),
                         "input_GBps": round(bytes_r * args.steps / el_r / 1e9, 3),
                         "wait_reader_sec": round(wr, 4), "wait_gpu_sec": round(wg, 4),
                         # zero-copy: this rank's share of the host pin budget and
                         # its peak registered bytes; the last step's pipeline
                         # fill / drain / pass seconds (host clock)
                         "zc_pin_budget": int(pin_b), "zc_pinned_peak": int(pin_p),
                         "last_fill_sec": round(fill_s, 5), "last_drain_sec": round(drain_s, 5),
                         "last_pass_sec": round(pass_s, 5)})
    elapsed = max(float(x[3]) for x in gathered)  # the slowest rank sets the step time
    # structured per-stage metrics ($DMLC_METRICS_FILE, JSONL, one file per rank
    # with "{rank}" in the path) and their cross-rank reduction
    from dmlc_core_amd.utils.metrics import MetricsLogger, parser_record, reduce_across_ranks

    rec = {"rows": local["rows"], "bytes": local["bytes"], "elapsed_sec": float(mine[3])}
    rec.update(parser_record(st))
    reduced = reduce_across_ranks(rec, device=cdev)
    probe = (allreduce_probe(dist, cdev, world, iters=5 if cdev.type == "cuda" else 2)
             if world > 1 else None)
    with MetricsLogger() as ml:
        ml.log("ingest", steps=args.steps, **rec)
        if rank == 0:
            ml.log("ingest_reduced", steps=args.steps,
                   **{f"{k}_{agg}": v[agg] for k, v in reduced.items()
                      for agg in ("sum", "min", "max")})
    (rows, nnz, nbytes), max_index = totals
    ms = elapsed / max(1, args.steps) * 1e3
    value = rows * args.steps / elapsed
    fmt = FORMATS[args.format]
    if rank == 0:
        ingest = ("HBM epoch cache (input resident in HBM after the warmup epoch)"
                  if use_gpu and args.mode == "hbm" else
                  "#cache page file: zero-copy DMA of binary RowBlock pages (no parse)"
                  if use_gpu and args.mode == "cache" else
                  "zero-copy mmap+hipHostRegister DMA" if use_gpu and parser.stats().get("zero_copy")
                  else "parallel pread -> pinned ring -> hipMemcpyAsync" if use_gpu else "CPU")
        out = {
            "metric": fmt["metric"],
            "value": round(value, 1),
            "unit": "records/s" if args.format == "recordio" else "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": round(value / fmt["baseline"], 3),
            "dtype": fmt["dtype"],
            "data": f"synthetic (deterministic {args.format}, 16 part files"
                    + (f", {args.shape} rows" if args.shape != "uniform" else "") + ")",
            "config": {
                "model": fmt["model"],
                "global_batch": int(rows),
                "seq_len": None,
                "parallelism": (f"dp{world} (InputSplit byte-range shards, "
                                + ("RCCL" if cdev.type == "cuda" else "gloo") + " NumCol all-reduce"
                                + (", all ranks on GPU 0" if args.share_gpu else "") + ")"
                                if world > 1 else "dp1 (one InputSplit shard, no collective)"),
                "format": args.format,
                "rows": int(rows),
                "nnz" if args.format != "recordio" else "payload_bytes": int(nnz),
                "num_col": max_index + 1,
                "input_bytes": int(nbytes),
                "chunk_mb": args.chunk_mb,
                "read_threads": read_threads,
                "device": "gpu" if use_gpu else "cpu",
                "numa_node_rank0": numa.get("numa_node", -1),
                "ingest": ingest,
            },
            "per_gpu_rows_per_sec": round(value / max(1, world), 1),
            "input_GBps": round(nbytes * args.steps / elapsed / 1e9, 3),
            "mode": args.mode,
            "shape": args.shape,
            "shuffle_parts": args.shuffle_parts,
            "baseline_value": fmt["baseline"],
            "same_host_cpu_baseline": dict(SAME_HOST_CPU[args.format],
                                           host="AMD EPYC 9575F (MI355X box)",
                                           source="profiles/r05_cpu"),
        }
        out["per_rank"] = per_rank
        out["allreduce_busbw_GBps"] = probe
        if use_gpu and args.mode == "cache":
            out["metric"] = fmt["metric"].replace("->CSR", " #cache pages->CSR")
            out["cache"] = {"bytes": parser.bytes, "pages": len(parser.pages()),
                            "zero_copy": parser.zero_copy}
        elif use_gpu:
            out["parser_stats_last_rank0"] = parser.stats()
        print(json.dumps(out), flush=True)
    ddist.finalize()


if __name__ == "__main__":
    main()
