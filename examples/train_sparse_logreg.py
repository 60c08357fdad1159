#!/usr/bin/env python3
"""End-to-end demonstrator: sharded LibSVM ->
GPU parser -> CSR resident in HBM -> HIP SpMV logistic regression -> RCCL
gradient all-reduce -> SGD, one process per MI355X.

    # one node, 8 GPUs, torchrun rendezvous
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/train_sparse_logreg.py data/
    # or through the dmlc tracker
    scripts/dmlc-submit --cluster local --num-workers 8 --gpus-per-node 8 \
        python examples/train_sparse_logreg.py data/

Without a data path a synthetic shard is generated per rank.
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
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--batch-rows", type=int, default=65536)
    ap.add_argument("--lr", type=float, default=0.5)
    ap.add_argument("--bucket-mb", type=float, default=64.0)
    args = ap.parse_args()

    import torch
    from dmlc_core_amd import data
    from dmlc_core_amd.models import SparseLogReg
    from dmlc_core_amd.parallel import dist

    info = dist.init()
    rank, world = info["rank"], info["world_size"]
    tmp = None
    uri = args.uri
    if uri is None:
        tmp = tempfile.mkdtemp(prefix="dmlc_logreg_")
        uri = os.path.join(tmp, "shard.libsvm")
        data.write_synthetic(uri, rank * args.rows, (rank + 1) * args.rows, seed=7, nthread=8)
        part, nparts = 0, 1
    else:
        part, nparts = rank, world

    t0 = time.perf_counter()
    csr = data.GPUParser(uri, part, nparts).parse_all()
    torch.cuda.synchronize()
    t_parse = time.perf_counter() - t0
    (rows, nnz), max_index = dist.global_stats([csr.rows, csr.nnz], csr.max_index)
    num_features = max_index + 1
    t = data.csr_to_torch(csr)
    label = t["label"].float()
    model = SparseLogReg(num_features).cuda()
    reducer = dist.GradAllReducer(model.parameters(), bucket_mb=args.bucket_mb)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr)
    n = csr.rows
    history = []
    for epoch in range(args.epochs):
        tot, cnt = 0.0, 0
        for b in range(0, n, args.batch_rows):
            e = min(n, b + args.batch_rows)
            batch = {"offset": t["offset"][b:e + 1], "index": t["index"], "value": t["value"]}
            logits = model(batch)
            loss = torch.nn.functional.binary_cross_entropy_with_logits(logits, label[b:e])
            opt.zero_grad(set_to_none=False)
            loss.backward()
            reducer.synchronize()
            opt.step()
            tot += float(loss.detach()) * (e - b)
            cnt += e - b
        (loss_sum, rows_seen), _ = dist.global_stats([tot, cnt], 0)
        history.append(loss_sum / rows_seen)
    if rank == 0:
        print(json.dumps({"world": world, "rows": int(rows), "nnz": int(nnz),
                          "num_features": num_features, "parse_sec_rank0": round(t_parse, 4),
                          "loss_per_epoch": [round(x, 5) for x in history]}), flush=True)
    dist.finalize()


if __name__ == "__main__":
    main()
