#!/usr/bin/env python3
"""Latency distribution of config 1 (the reference's 3-vote certificate, committee cached) through
the host ABI: p50 / p90 / p99 / p99.9 / max over N calls.  NWC_ZERO_COPY=0 selects the staged-copy
small path for comparison.   python tools/lat_cfg1.py [N]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402  (one HIP runtime: torch's)
from narwhal_amd import _lib  # noqa: E402

n_calls = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
lib = _lib.load()
gv = json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_verify.json")))
gb = {c["name"]: c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "ed25519_batch.json")))}
committee = np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in gv["reference_keys"]["pks"]])
c = gb["ref-verify_valid_batch"]
d = bytes.fromhex(c["msg"])
p = b"".join(bytes.fromhex(v[0]) for v in c["votes"])
s = b"".join(bytes.fromhex(v[1]) for v in c["votes"])
_lib.check(lib.nwc_set_committee(_lib.buf(committee), len(committee)))
lat = np.empty(n_calls)
for i in range(n_calls + 100):
    t0 = time.perf_counter()
    rc = lib.nwc_verify_batch(_lib.buf(d), _lib.buf(p), _lib.buf(s), 3, None)
    dt = time.perf_counter() - t0
    assert rc == 0 or os.environ.get("NWC_LAT_ANY"), rc
    if i >= 100:
        lat[i - 100] = dt * 1e6
q = np.percentile(lat, [50, 90, 99, 99.9])
print(json.dumps({"zero_copy": os.environ.get("NWC_ZERO_COPY", "1"), "spin_wait": os.environ.get("NWC_SPIN_WAIT", "1"), "calls": n_calls,
                  "p50_us": q[0], "p90_us": q[1], "p99_us": q[2], "p999_us": q[3], "max_us": float(lat.max()),
                  "over_100us": int((lat > 100).sum())}))
