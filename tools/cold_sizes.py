"""Latency of first-sight device calls by size (k_verify_cold vs the one-lane path, NWC_COLD=0):
median of 20 device.verify calls on fresh keys per size, leaf and strict.
    python tools/cold_sizes.py [sizes...]   -> one JSON line"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from narwhal_amd import device  # noqa: E402

sizes = [int(x) for x in sys.argv[1:]] or [3, 64, 256, 1024]
out = {"cold": os.environ.get("NWC_COLD", "1"), "us": {}}
for n in sizes:
    for strict in (False, True):
        ts = []
        for rep in range(22):
            msgs = device.derive32(b"sizes-msg", rep * 7919 + n, n)
            pks, sigs = device.keygen_sign(device.derive32(b"sizes-seed", rep * 7919 + n, n), msgs)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            w = device.verify(msgs, pks, sigs, strict=strict)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            assert device.unpack_bits(w, n).all()
        ts = sorted(ts[2:])
        out["us"]["%d_%s" % (n, "strict" if strict else "leaf")] = round(ts[len(ts) // 2] * 1e6, 1)
print(json.dumps(out))
