"""Subprocess body of tests/test_gpu_autokeys.py::test_lifecycle (NWC_AUTO_KEYS is read once per
process): fill a 4-key auto cache, overflow it (FIFO replacement), change the committee (the
auto cache empties), and report verdicts, cache sizes and the latency kernel's hit count after
every call."""
import ctypes
import json
import sys

import torch  # noqa: F401  (one HIP runtime: torch's)

sys.path.insert(0, sys.argv[1])
from narwhal_amd import _lib, device  # noqa: E402

lib = _lib.load()
n_keys = 8
seeds = device.derive32(b"lifecycle-seed", 0, n_keys).cpu().numpy().tobytes()
digest = device.derive32(b"lifecycle-digest", 0, 1).cpu().numpy().tobytes()
pks, sigs = device.keygen_sign_host(seeds, digest * n_keys, n_keys)
log = []


def info():
    c, a = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _lib.check(lib.nwc_cache_stats(ctypes.byref(c), ctypes.byref(a)))
    cap, builds, hits = ctypes.c_uint32(0), ctypes.c_uint64(0), ctypes.c_uint64(0)
    _lib.check(lib.nwc_auto_cache_info(ctypes.byref(cap), ctypes.byref(builds), ctypes.byref(hits)))
    return {"committee": c.value, "auto": a.value, "cap": cap.value, "builds": builds.value, "hits": hits.value}


def cert(keys, corrupt=None):
    """A certificate of the given key indices over `digest`; vote `corrupt` (position) invalid."""
    p = b"".join(pks[32 * k:32 * k + 32] for k in keys)
    s = bytearray(b"".join(sigs[64 * k:64 * k + 64] for k in keys))
    if corrupt is not None:
        s[64 * corrupt + 40] ^= 1
    bad = ctypes.create_string_buffer(2)
    rc = lib.nwc_verify_batch(_lib.buf(digest), _lib.buf(p), _lib.buf(bytes(s)), len(keys), bad)
    return rc, bad.raw[0]


def step(tag, keys, corrupt=None):
    rc, bad = cert(keys, corrupt)
    log.append({"tag": tag, "keys": keys, "corrupt": corrupt, "rc": rc, "bad": bad, **info()})


_lib.check(lib.nwc_set_committee(None, 0))
for sight in range(3):
    step("A%d" % sight, [0, 1])                 # 2nd sight builds, 3rd hits
for sight in range(3):
    step("B%d" % sight, [2, 3], 1 if sight == 2 else None)   # cache full at 4 keys
for sight in range(3):
    step("C%d" % sight, [4, 5])                 # FIFO: replaces keys 0 and 1
step("A-after-eviction", [0, 1])            # first sight again: the uncached path
step("C-cached", [4, 5], 0)
_lib.check(lib.nwc_set_committee(pks[32 * 6:32 * 8], 2))   # new committee: keys 6, 7
step("after-committee", [4, 5])             # auto cache emptied: uncached again
step("committee-keys", [6, 7])              # committee cache
for sight in range(3):
    step("C-again%d" % sight, [4, 5])
_lib.check(lib.nwc_set_committee(None, 0))
json.dump(log, open(sys.argv[2], "w"))
