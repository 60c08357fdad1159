#!/usr/bin/env python3
"""K11 at the SURVEY §7.3 demo scale: the 10 M-row LibSVM set parsed into HBM,
then the sparse logistic-regression step -- SpMV (forward), SpMV^T (gradient,
one f32 atomic per nonzero) and the full SparseLogReg forward + backward --
timed with HIP events.  Prints one JSON object (bytes moved and the implied
bandwidth / atomic rate per kernel).

usage: python scripts/bench_linear.py [--rows N] [--iters K]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--data", default="/tmp/dmlc_linear_bench")
    ap.add_argument("--num-features", type=int, default=0,
                    help="feature space of the synthetic data (0: the generator's default, ~1 M)")
    ap.add_argument("--skip-models", action="store_true", help="kernels and transpose only")
    args = ap.parse_args()
    if args.num_features:
        args.data = f"{args.data}_{args.num_features}"
    import torch

    from dmlc_core_amd import data, ops
    from dmlc_core_amd.models import SparseLogReg

    os.makedirs(args.data, exist_ok=True)
    nfiles = 16
    per = (args.rows + nfiles - 1) // nfiles
    for i in range(nfiles):
        f = os.path.join(args.data, f"part-{i:03d}.libsvm")
        if not os.path.exists(f):
            kw = {"num_features": args.num_features} if args.num_features else {}
            data.write_synthetic(f + ".tmp", i * per, min(args.rows, (i + 1) * per), seed=0,
                                 nthread=16, **kw)
            os.replace(f + ".tmp", f)
    csr = data.GPUParser(args.data).parse_all()
    t = data.csr_to_torch(csr)
    nrows, nnz, nfeat = csr.rows, csr.nnz, max(csr.max_index + 1, args.num_features)
    w = torch.randn(nfeat, device="cuda") * 0.01
    d = torch.randn(nrows, device="cuda")

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(args.iters):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.iters

    idx_b = t["index"].element_size()
    csr_bytes = nnz * (idx_b + 4) + (nrows + 1) * 8
    res = {"rows": nrows, "nnz": nnz, "num_features": nfeat}
    ms = timed(lambda: ops.spmv(t, w))
    res["spmv"] = {"ms": round(ms, 3), "csr_GBps": round(csr_bytes / ms / 1e6, 1)}
    ms = timed(lambda: ops.spmv_t(t, d, nfeat))
    res["spmv_t"] = {"ms": round(ms, 3), "csr_GBps": round(csr_bytes / ms / 1e6, 1),
                     "G_atomics_per_s": round(nnz / ms / 1e6, 1)}
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    tt = ops.transpose(t, nfeat)
    b.record()
    torch.cuda.synchronize()
    res["transpose_build_ms"] = round(a.elapsed_time(b), 1)
    # again, with the allocator's blocks cached (the build of a further shard)
    del tt
    torch.cuda.synchronize()
    a.record()
    tt = ops.transpose(t, nfeat)
    b.record()
    torch.cuda.synchronize()
    res["transpose_build_warm_ms"] = round(a.elapsed_time(b), 1)
    # into a previous result (out=): the kernels alone, no allocation at all
    torch.cuda.synchronize()
    a.record()
    tt = ops.transpose(t, nfeat, out=tt)
    b.record()
    torch.cuda.synchronize()
    res["transpose_build_out_ms"] = round(a.elapsed_time(b), 1)
    ms = timed(lambda: ops.spmv(tt, d, 0.0))
    tt_bytes = nnz * 8 + (nfeat + 1) * 8
    res["spmv_t_gather"] = {"ms": round(ms, 3), "csc_GBps": round(tt_bytes / ms / 1e6, 1)}
    del tt
    for mode in () if args.skip_models else ("atomic", "transpose"):
        model = SparseLogReg(nfeat, grad=mode).cuda()

        def step():
            model.zero_grad(set_to_none=True)
            model.loss(t).backward()

        ms = timed(step)  # the first (untimed) call builds the cached transpose
        res[f"logreg_fwd_bwd_{mode}"] = {"ms": round(ms, 3),
                                         "rows_per_sec": round(nrows / ms * 1e3, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
