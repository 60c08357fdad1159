#!/usr/bin/env python3
"""GPU parse throughput for every text format (LibSVM / LibFM / CSV) next to
the reference's measured CPU numbers (LibSVM 2.20M rows/s,
LibFM 1.95M, CSV 6.61M at 8 threads).  One JSON line per format."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF = {"libsvm": 2.20e6, "libfm": 1.95e6, "csv": 6.61e6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--formats", default="libsvm,libfm,csv")
    ap.add_argument("--dir", default="/tmp/dmlc_bench_fmt")
    ap.add_argument("--zero-copy", default="auto")
    args = ap.parse_args()
    import torch
    from dmlc_core_amd import data

    os.makedirs(args.dir, exist_ok=True)
    for fmt in args.formats.split(","):
        path = os.path.join(args.dir, f"{fmt}_{args.rows}.{fmt}")
        if not os.path.exists(path + ".done"):
            data.write_synthetic(path, 0, args.rows, format=fmt, seed=0, nthread=16)
            open(path + ".done", "w").close()
        uri = path + ("?label_column=0" if fmt == "csv" else "")
        kw = {"label_column": 0} if fmt == "csv" else {}
        p = data.GPUParser(uri, 0, 1, format=fmt, zero_copy=args.zero_copy, **kw)
        csr = data.DeviceCSR()
        p.parse_all(csr)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            p.before_first()
            csr.clear()
            p.parse_all(csr)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        nbytes = os.path.getsize(path)
        print(json.dumps({"format": fmt, "rows": csr.rows, "nnz": csr.nnz,
                          "rows_per_sec": round(csr.rows / dt, 1), "GBps": round(nbytes / dt / 1e9, 3),
                          "ms": round(dt * 1e3, 2), "vs_reference_cpu": round(csr.rows / dt / REF[fmt], 1),
                          "stats": p.stats()}), flush=True)


if __name__ == "__main__":
    main()
