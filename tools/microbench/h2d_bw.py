#!/usr/bin/env python3
"""Host-side ceilings of the digester's data path on the GPU box: H2D DMA from pinned memory (64-MB
chunks, as the digester's stages) and host memcpy throughput with 1..16 threads (its gather)."""
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

MB = 1 << 20
out = {}
dev = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
for kind in ("pinned", "pageable"):
    src = torch.empty(64 * MB, dtype=torch.uint8, pin_memory=(kind == "pinned"))
    src.fill_(7)
    for _ in range(3):
        dev[:64 * MB].copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(16):
        dev[(i % 16) * 64 * MB:(i % 16 + 1) * 64 * MB].copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    out["h2d_%s_GBps" % kind] = 16 * 64 * MB / (time.perf_counter() - t0) / 1e9
a = np.ones(512 * MB, np.uint8)
b = np.empty_like(a)
for nt in (1, 2, 4, 8, 16):
    step = len(a) // nt
    with ThreadPoolExecutor(nt) as ex:
        list(ex.map(lambda i: np.copyto(b[i * step:(i + 1) * step], a[i * step:(i + 1) * step]), range(nt)))
        t0 = time.perf_counter()
        for _ in range(3):
            list(ex.map(lambda i: np.copyto(b[i * step:(i + 1) * step], a[i * step:(i + 1) * step]), range(nt)))
        out["memcpy_%dthreads_GBps" % nt] = 3 * len(a) / (time.perf_counter() - t0) / 1e9
print(json.dumps(out))
