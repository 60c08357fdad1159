#!/usr/bin/env python3
"""RecordIO decode throughput: GPU (K7, resident in HBM) vs the CPU reader.

Reference CPU numbers on 1M x 512 B records: RecordIOReader
7.0M rec/s, InputSplit NextRecord 8.7M rec/s, NextChunk+ChunkReader 11.3M
rec/s.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--records", type=int, default=4_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--chunk-mb", type=int, default=64)
    ap.add_argument("--dir", default="/tmp/dmlc_bench_rec")
    ap.add_argument("--cpu", action="store_true", help="also time the CPU InputSplit path")
    args = ap.parse_args()
    import torch
    from dmlc_core_amd import data, io

    os.makedirs(args.dir, exist_ok=True)
    path = os.path.join(args.dir, f"rec_{args.records}.rec")
    if not os.path.exists(path + ".done"):
        data.write_synthetic(path, 0, args.records, format="recordio", seed=0, nthread=16)
        open(path + ".done", "w").close()
    nbytes = os.path.getsize(path)
    out = {"records": args.records, "file_bytes": nbytes}
    r = io.GPURecordIO(path, chunk_mb=args.chunk_mb)
    r.read_all()  # warm-up (page cache, allocations)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r.before_first()
        b = r.read_all()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    assert b["size"] == args.records, b["size"]
    out.update({"gpu_rec_per_sec": round(args.records / dt, 1), "gpu_GBps": round(nbytes / dt / 1e9, 3),
                "gpu_ms": round(dt * 1e3, 3), "stats": r.stats()})
    if args.cpu:
        t0 = time.perf_counter()
        n = sum(1 for _ in io.iter_records(path, 0, 1, "recordio"))
        dt = time.perf_counter() - t0
        out.update({"cpu_python_iter_rec_per_sec": round(n / dt, 1)})
    out["vs_reference_chunkreader_11.3M"] = round(out["gpu_rec_per_sec"] / 11.3e6, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
