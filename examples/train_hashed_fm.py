#!/usr/bin/env python3
"""BASELINE config 5 end to end, one process per MI355X: a LibFM shard ->
fused tokenize / hash / fp8 kernel (GPUParser.parse_all_hashed, no CSR) ->
HashedFM trained on the fp8 batch with the bf16-MFMA forward / backward
kernels -> RCCL gradient all-reduce -> Adam.

    # one node, 8 GPUs
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_hashed_fm.py data/
    # or through the dmlc tracker
    scripts/dmlc-submit --cluster local --num-workers 8 --gpus-per-node 8 \\
        python examples/train_hashed_fm.py data/

Without a data path a synthetic LibFM shard is generated per rank.  Prints one
JSON line (rank 0) with the loss per epoch and the step time.
"""
import argparse
import json
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("uri", nargs="?", default=None)
    ap.add_argument("--rows", type=int, default=200_000, help="synthetic rows per rank")
    ap.add_argument("--dim", type=int, default=1024, help="hashed features (multiple of 128)")
    ap.add_argument("--scale", type=float, default=0.5, help="fp8 quantisation scale")
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-rows", type=int, default=65536)
    ap.add_argument("--lr", type=float, default=0.01)
    args = ap.parse_args()

    import torch

    from dmlc_core_amd import data
    from dmlc_core_amd.models import HashedFM
    from dmlc_core_amd.parallel import dist

    info = dist.init()
    rank, world = info["rank"], info["world_size"]
    uri = args.uri
    if uri is None:
        uri = os.path.join(tempfile.mkdtemp(prefix="dmlc_hfm_"), "shard.libfm")
        data.write_synthetic(uri, rank * args.rows, (rank + 1) * args.rows, format="libfm",
                             seed=11, nthread=8)
        part, nparts = 0, 1
    else:
        part, nparts = rank, world
    t0 = time.perf_counter()
    batch = data.GPUParser(uri, part, nparts, format="libfm").parse_all_hashed(
        args.dim, seed=1, fp8=True, scale=args.scale)
    torch.cuda.synchronize()
    t_parse = time.perf_counter() - t0
    x8, label = batch["x"], batch["label"].clamp(0, 1)
    n = x8.shape[0]
    model = HashedFM(dim=args.dim, rank=16).cuda()
    reducer = dist.GradAllReducer(model.parameters())
    opt = torch.optim.Adam(model.parameters(), lr=args.lr)
    history, steps, t_train = [], 0, 0.0
    for epoch in range(args.epochs):
        tot = 0.0
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for b in range(0, n, args.batch_rows):
            e = min(n, b + args.batch_rows)
            y = model(x8[b:e], scale=args.scale)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(y, label[b:e])
            opt.zero_grad(set_to_none=False)
            loss.backward()
            reducer.synchronize()
            opt.step()
            tot += float(loss.detach()) * (e - b)
            steps += 1 if epoch else 0
        torch.cuda.synchronize()
        if epoch:  # the first epoch also loads code objects and sets up Adam
            t_train += time.perf_counter() - t1
        (loss_sum, rows_seen), _ = dist.global_stats([tot, n], 0)
        history.append(loss_sum / rows_seen)
    if rank == 0:
        print(json.dumps({"world": world, "rows_rank0": n, "dim": args.dim, "gemm": model.gemm,
                          "parse_hash_sec_rank0": round(t_parse, 4),
                          "ms_per_step": round(t_train / max(steps, 1) * 1e3, 3),
                          "loss_per_epoch": [round(v, 5) for v in history]}), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
