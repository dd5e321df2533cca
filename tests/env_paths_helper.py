"""Subprocess body of tests/test_gpu_env_paths.py: the small-call paths that process-wide switches
select (NWC_ZERO_COPY, NWC_AUTO_KEYS -- read once per process).  Runs every golden batch three
times through nwc_verify_batch, the golden strict cases through nwc_verify_strict, with and then
without the committee cache, and reports verdicts, bad sets and the cache sizes."""
import ctypes
import json
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime: torch's)

sys.path.insert(0, sys.argv[2])
from narwhal_amd import _lib  # noqa: E402

lib = _lib.load()
gv = json.load(open(sys.argv[2] + "/tests/golden/ed25519_verify.json"))
gb = json.load(open(sys.argv[2] + "/tests/golden/ed25519_batch.json"))
out = {"batch": [], "strict": [], "stats": []}


def stats():
    c, a = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _lib.check(lib.nwc_cache_stats(ctypes.byref(c), ctypes.byref(a)))
    return [c.value, a.value]


strict_cases = [c for c in gv["cases"] if len(c["msg"]) == 64]
keys = np.unique(np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in strict_cases]
                          + [np.frombuffer(bytes.fromhex(v[0]), np.uint8) for b in gb for v in b["votes"]]), axis=0)
for committee in (True, False):
    _lib.check(lib.nwc_set_committee(_lib.buf(keys) if committee else None, len(keys) if committee else 0))
    for sight in range(3):
        for b in gb:
            n = len(b["votes"])
            d = bytes.fromhex(b["msg"])
            p = b"".join(bytes.fromhex(v[0]) for v in b["votes"])
            s = b"".join(bytes.fromhex(v[1]) for v in b["votes"])
            bad = ctypes.create_string_buffer((n + 7) // 8 + 1)
            rc = lib.nwc_verify_batch(_lib.buf(d), _lib.buf(p) if n else None, _lib.buf(s) if n else None, n, bad)
            bits = np.unpackbits(np.frombuffer(bad.raw, np.uint8), bitorder="little")[:n]
            out["batch"].append([b["name"], rc, [int(i) for i in np.nonzero(bits)[0]]])
        for c in strict_cases:
            m, p, s = (bytes.fromhex(c[k]) for k in ("msg", "pk", "sig"))
            out["strict"].append([c["name"], lib.nwc_verify_strict(_lib.buf(m), _lib.buf(p), _lib.buf(s))])
        out["stats"].append(stats())
json.dump(out, open(sys.argv[1], "w"))
