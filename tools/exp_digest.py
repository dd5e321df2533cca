#!/usr/bin/env python3
"""Development aid: k_sha512_digest32 time vs number of messages (waves per SIMD), cfg-4 batches."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import bench  # noqa: E402
from narwhal_amd import _lib, device  # noqa: E402

_lib.load()
pool = 4096
data = bench.make_cfg4_pool(pool)
for nb in [int(x) for x in sys.argv[1:]] or [16384, 32768, 65536, 98304, 100000, 131072]:
    starts = (torch.arange(nb, dtype=torch.int64, device="cuda") % pool) * bench.CFG4_STRIDE
    ends = starts + bench.CFG4_BATCH_BYTES
    outs = torch.empty((nb, 32), dtype=torch.uint8, device="cuda")
    f = lambda: device.sha512_trunc32_ranges(data, starts, ends, out=outs)  # noqa: E731
    f()
    ms = bench.timed_kernel(f, 2)
    print("n=%7d waves/SIMD=%.2f  %.2f ms  %.1f GB/s  %.3f us/block-per-lane" % (
        nb, nb / 64 / 1024, ms, nb * bench.CFG4_BATCH_BYTES / ms / 1e6, ms * 1e3 / 3970), flush=True)
