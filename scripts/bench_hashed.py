#!/usr/bin/env python3
"""BASELINE config 5: LibFM -> hashed fp8 dense batch on one MI355X.

Times (a) the two-step path, tile parser -> device CSR -> K9 hashed_dense, and
(b) the fused kernel (GPUParser.parse_all_hashed: tokenize -> hash -> fp8,
no CSR), both over text already resident in HBM (hbm_cache, warm epoch
first), plus HashedFM forward+backward on the batch.  Prints one JSON line.

usage: python scripts/bench_hashed.py [--rows N] [--dim D] [--steps K]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--sweep", default="128,256,1024",
                    help="extra dims timed for fused vs CSR+K9 (comma list, '' to skip)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--data", default="/tmp/dmlc_hashed_bench.libfm")
    ap.add_argument("--replay-first-mb", type=float, default=None,
                    help="first merged replay chunk (0: no ramp; default: the parser's)")
    ap.add_argument("--replay-chunk-mb", type=float, default=None,
                    help="merged replay chunk cap (default: the parser's)")
    ap.add_argument("--hash-one-pass", type=int, default=None,
                    help="reused batch: 1 one look-back launch per chunk, 0 C1 + C2 + the "
                         "counted kernel (default: the parser's)")
    args = ap.parse_args()
    import torch

    from dmlc_core_amd import data, ops
    from dmlc_core_amd.models import HashedFM

    if not os.path.exists(args.data):
        data.write_synthetic(args.data + ".tmp", 0, args.rows, format="libfm", seed=0, nthread=16)
        os.replace(args.data + ".tmp", args.data)
        os.sync()  # no dirty-page writeback under the timed loops
    nbytes = os.path.getsize(args.data)
    cfg = {}
    if args.replay_first_mb is not None:
        cfg["replay_first_mb"] = args.replay_first_mb
    if args.replay_chunk_mb is not None:
        cfg["replay_chunk_mb"] = args.replay_chunk_mb
    two = data.GPUParser(args.data, format="libfm", hbm_cache=1, **cfg)
    fcfg = dict(cfg) if args.hash_one_pass is None else dict(cfg, hash_one_pass=args.hash_one_pass)
    fused = data.GPUParser(args.data, format="libfm", hbm_cache=1, **fcfg)

    def step_two():
        two.before_first()
        csr = two.parse_all()
        return ops.hashed_dense(data.csr_to_torch(csr), args.dim, seed=1, fp8=True, scale=0.5)

    prev = {}

    def step_fused():
        # the batch of the previous pass is refilled in place (out=)
        fused.before_first()
        prev["b"] = fused.parse_all_hashed(args.dim, seed=1, fp8=True, scale=0.5, strategy="fused",
                                           out=prev.get("b"))
        return prev["b"]["x"]

    res = {}
    for name, fn in (("csr_then_k9", step_two), ("fused", step_fused)):
        fn()  # warm: fills the HBM cache
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            x = fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.steps
        res[name] = {"ms": round(dt * 1e3, 3), "rows_per_sec": round(x.shape[0] / dt, 1),
                     "text_GBps": round(nbytes / dt / 1e9, 2)}
    a = step_two().view(torch.uint8)
    b = step_fused().view(torch.uint8).clone()
    res["identical_fp8"] = bool(torch.equal(a, b))
    res["mismatch_frac"] = float((a != b).float().mean())
    model = HashedFM(dim=args.dim, rank=16).cuda()
    fused.before_first()
    batch = fused.parse_all_hashed(args.dim, seed=1, fp8=True, scale=0.5, strategy="fused")
    y = model(batch["x"], scale=0.5)
    loss = torch.nn.functional.binary_cross_entropy_with_logits(y, batch["label"].clamp(0, 1))
    loss.backward()
    lab = batch["label"].clamp(0, 1)

    def two_pass():
        model.zero_grad()
        y = model(batch["x"], scale=0.5)
        torch.nn.functional.binary_cross_entropy_with_logits(y, lab).backward()

    def fused_step():
        model.zero_grad()
        model.loss(batch["x"], lab, scale=0.5).backward()

    for name, fn in (("two_pass", two_pass), ("fused", fused_step)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps * 1e3
        # GPU time of the same step (events around it: no host gaps between steps)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        for _ in range(args.steps):
            fn()
        ev1.record()
        torch.cuda.synchronize()
        res[f"hashed_fm_{name}_step_ms"] = round(wall, 3)
        res[f"hashed_fm_{name}_step_event_ms"] = round(ev0.elapsed_time(ev1) / args.steps, 3)
        res[f"hashed_fm_{name}_gemm"] = model.gemm
    # the framework's training step (model.loss: the fused kernel on this shape)
    res["hashed_fm_step_ms"] = res["hashed_fm_fused_step_ms"]
    res["hashed_fm_step_event_ms"] = res["hashed_fm_fused_step_event_ms"]
    res["hashed_fm_gemm"] = res["hashed_fm_fused_gemm"]
    res["replay"] = fcfg
    res.update({"rows": int(batch["x"].shape[0]), "dim": args.dim, "text_bytes": nbytes,
                "speedup_fused_vs_csr_k9": round(res["csr_then_k9"]["ms"] / res["fused"]["ms"], 3)})
    sweep = {}
    for d in [int(x) for x in args.sweep.split(",") if x]:
        t = {}
        for name, fn in (("csr_then_k9", lambda: ops.hashed_dense(
                data.csr_to_torch(two.parse_all()), d, seed=1, fp8=True, scale=0.5)),
                         ("fused", lambda: prev.__setitem__("b", fused.parse_all_hashed(
                             d, seed=1, fp8=True, scale=0.5, strategy="fused", out=prev.get("b"))))):
            (two if name == "csr_then_k9" else fused).before_first()
            fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                (two if name == "csr_then_k9" else fused).before_first()
                fn()
            torch.cuda.synchronize()
            t[name] = round((time.perf_counter() - t0) / args.steps * 1e3, 3)
        t["speedup"] = round(t["csr_then_k9"] / t["fused"], 3)
        sweep[str(d)] = t
    res["dim_sweep_ms"] = sweep
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
