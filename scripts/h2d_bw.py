"""Measure pinned host->device copy bandwidth (the PCIe ceiling of ingestion)."""
import json
import time

import torch

torch.cuda.init()
res = {}
for mb in (16, 64, 256):
    n = mb << 20
    h = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d = torch.empty(n, dtype=torch.uint8, device="cuda")
    for _ in range(3):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    iters = max(4, 2048 // mb)
    t = time.perf_counter()
    for _ in range(iters):
        d.copy_(h, non_blocking=True)
    torch.cuda.synchronize()
    res[f"h2d_{mb}MiB_GBps"] = round(n * iters / (time.perf_counter() - t) / 1e9, 2)
    # two streams in parallel (second DMA engine?)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    half = n // 2
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        with torch.cuda.stream(s1):
            d[:half].copy_(h[:half], non_blocking=True)
        with torch.cuda.stream(s2):
            d[half:].copy_(h[half:], non_blocking=True)
    torch.cuda.synchronize()
    res[f"h2d_{mb}MiB_2streams_GBps"] = round(n * iters / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(res))
