"""H2D copy rate from pinned host memory on one MI355X: one hipMemcpyAsync of a
C2 batch's bytes (23.6 MB) against the same bytes split over 2 / 4 / 8 streams
issued together (do several DMA engines beat one?).  Measurement only (torch
is used for pinned buffers and streams)."""
import json
import time

import torch

n = 23658504
src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
src.fill_(7)
dst = torch.empty(n, dtype=torch.uint8, device="cuda:0")
for parts in (1, 2, 4, 8, 1):
    streams = [torch.cuda.Stream() for _ in range(parts)]
    bounds = [n * k // parts for k in range(parts + 1)]
    ts = []
    for rep in range(25):
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k, s in enumerate(streams):
            with torch.cuda.stream(s):
                dst[bounds[k]:bounds[k + 1]].copy_(src[bounds[k]:bounds[k + 1]], non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    ts.sort()
    med = ts[len(ts) // 2]
    print(json.dumps({"parts": parts, "ms": 1e3 * med, "GB_per_s": n / med / 1e9}))
