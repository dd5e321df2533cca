"""Subprocess helper for tests/test_gpu_host_paths.py: verdicts of nwc_verify_strict_many over the
triples in an .npz, from pageable host buffers, called twice on the same stages and arena.  The
host pipeline's switches (NWC_HOST_PAIR*, NWC_FORCE_FALLBACK_EVERY) come from the environment,
which libnwc reads once per process."""
import ctypes
import sys

import numpy as np

sys.path.insert(0, sys.argv[3])
from narwhal_amd import _lib  # noqa: E402

d = np.load(sys.argv[1])
m, p, s = (np.ascontiguousarray(d[k]) for k in ("m", "p", "s"))
n = p.shape[0]
lib = _lib.load()
outs = []
for _ in range(2):
    out = ctypes.create_string_buffer((n + 7) // 8)
    _lib.check(lib.nwc_verify_strict_many(_lib.buf(m), _lib.buf(p), _lib.buf(s), n, out))
    outs.append(np.unpackbits(np.frombuffer(out.raw, np.uint8), bitorder="little")[:n].astype(bool))
np.savez(sys.argv[2], first=outs[0], second=outs[1])
