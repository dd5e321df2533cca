"""Subprocess helper for tests/test_gpu_paths.py: verifies the triples in an .npz through the C
ABI (strict and leaf) and writes the verdicts.  Path selection comes from the environment
(NWC_VERIFY_PATH, NWC_FORCE_FALLBACK_EVERY), which libnwc reads once per process."""
import sys

import numpy as np
import torch

sys.path.insert(0, sys.argv[3])
from narwhal_amd import device  # noqa: E402

d = np.load(sys.argv[1])
m, p, s = (torch.from_numpy(d[k]).cuda() for k in ("m", "p", "s"))
n = p.shape[0]
out = {}
for strict in (True, False):
    w = device.verify(m, p, s, strict=strict)
    torch.cuda.synchronize()
    out["strict" if strict else "leaf"] = device.unpack_bits(w, n)
np.savez(sys.argv[2], **out)
