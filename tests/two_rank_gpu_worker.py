"""Worker of tests/test_gpu_two_ranks.py: one rank of a dmlc-submit job whose
ranks all share cuda:0 (gloo control plane -- RCCL refuses two ranks on one
device).  Each rank parses its byte-range shard on the GPU with zero-copy DMA
in sliding registration windows and NUMA binding on, checks it against the
CPU parser of the same shard, and all-gathers (rows, nnz, checksum)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as td  # noqa: E402

from dmlc_core_amd import data  # noqa: E402
from dmlc_core_amd.parallel import dist  # noqa: E402
from dmlc_core_amd.parallel.affinity import bind_to_gpu  # noqa: E402


def main():
    path, out = sys.argv[1], sys.argv[2]
    info = dist.init("gloo")
    rank, world = info["rank"], info["world_size"]
    torch.cuda.set_device(0)
    numa = bind_to_gpu(0)
    p = data.GPUParser(path, rank, world, format="libsvm", chunk_mb=2, zero_copy=1,
                       zc_pin_budget_mb=1, zc_window_mb=4, read_threads=4)
    rows = nnz = 0
    csum = 0
    for epoch in range(2):
        if epoch:
            p.before_first()
        csr = p.parse_all()
        h = csr.to_host()
        cpu = list(data.iter_blocks(path, rank, world, "libsvm"))
        lab = np.concatenate([b["label"] for b in cpu]) if cpu else np.zeros(0, np.float32)
        idx = np.concatenate([b["index"] for b in cpu]) if cpu else np.zeros(0, np.uint32)
        assert np.array_equal(h["label"], lab), rank
        assert np.array_equal(h["index"], idx), rank
        rows, nnz = csr.rows, csr.nnz
        csum = int(h["index"].astype(np.uint64).sum())
    st = p.stats()
    assert st["zero_copy"], st
    mine = torch.tensor([rank, rows, nnz, csum], dtype=torch.int64)
    allv = [torch.zeros_like(mine) for _ in range(world)]
    td.all_gather(allv, mine)
    if rank == 0:
        with open(out, "w") as f:
            json.dump({"ranks": [v.tolist() for v in allv], "numa": numa.get("numa_node", -1)}, f)
    dist.finalize()


if __name__ == "__main__":
    main()
