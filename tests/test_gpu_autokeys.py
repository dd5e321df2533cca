"""The auto key cache (nwc_api.hip auto_insert): keys of small host calls outside the committee
cache enter it on their second sight, after which the calls take the latency kernel over it.
Verdicts and bad-vote sets must not depend on it: every golden batch and strict case is run
three times (first sight: general path; second: general path + build; third: auto cache) and
compared with the fixture each time, and random certificates with bad votes likewise.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    return lib


def _stats(lib):
    from narwhal_amd import _lib
    c, a = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _lib.check(lib.nwc_cache_stats(ctypes.byref(c), ctypes.byref(a)))
    return c.value, a.value


def _batch(lib, d: bytes, p: bytes, s: bytes, n: int):
    from narwhal_amd import _lib
    bad = ctypes.create_string_buffer((n + 7) // 8 + 1)
    rc = lib.nwc_verify_batch(_lib.buf(d), _lib.buf(p), _lib.buf(s), n, bad)
    assert rc in (0, 1), rc
    bits = np.unpackbits(np.frombuffer(bad.raw, np.uint8), bitorder="little")[:n]
    return rc == 0, [int(i) for i in np.nonzero(bits)[0]]


def test_golden_batches_three_sights(lib, golden_batch):
    before = _stats(lib)[1]
    for b in golden_batch:
        n = len(b["votes"])
        if n == 0:
            continue
        d = bytes.fromhex(b["msg"])
        p = b"".join(bytes.fromhex(v[0]) for v in b["votes"])
        s = b"".join(bytes.fromhex(v[1]) for v in b["votes"])
        for sight in range(3):
            ok, bad = _batch(lib, d, p, s, n)
            assert ok == b["verdict"], (b["name"], sight)
            assert bad == b["bad"], (b["name"], sight)
    assert _stats(lib)[1] > before, "the auto key cache never engaged"


def test_golden_strict_three_sights(lib, golden_verify):
    from narwhal_amd import _lib
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    for c in cases:
        m, p, s = (bytes.fromhex(c[k]) for k in ("msg", "pk", "sig"))
        for sight in range(3):
            rc = lib.nwc_verify_strict(_lib.buf(m), _lib.buf(p), _lib.buf(s))
            assert rc in (0, 1)
            assert (rc == 0) == c["strict"], (c["name"], sight)


def test_random_certificates_with_bad_votes(lib):
    import torch
    from narwhal_amd import device
    certs, q = 24, 5
    seeds = device.derive32(b"autokeys-seed", 0, certs * q)
    digests = device.derive32(b"autokeys-digest", 0, certs)
    pks, sigs = device.keygen_sign(seeds, digests.repeat_interleave(q, dim=0))
    torch.cuda.synchronize()
    P, S, D = (t.cpu().numpy().copy() for t in (pks, sigs, digests))
    rng = np.random.default_rng(7)
    bad_sets = []
    for c in range(certs):
        k = int(rng.integers(0, q + 1))   # k == q: no bad vote
        if k < q:
            S[c * q + k, 3] ^= 0x40
        bad_sets.append([k] if k < q else [])
    for sight in range(3):
        for c in range(certs):
            ok, bad = _batch(lib, D[c].tobytes(), P[c * q:(c + 1) * q].tobytes(), S[c * q:(c + 1) * q].tobytes(), q)
            assert bad == bad_sets[c], (c, sight)
            assert ok == (not bad_sets[c]), (c, sight)


def test_lifecycle(tmp_path):
    """NWC_AUTO_KEYS=4: the cache fills, new keys replace the oldest (FIFO) and take the latency
    kernel, evicted keys fall back to the uncached path, nwc_set_committee empties it -- and every
    verdict and bad set stays exact (crypto/src/lib.rs:206-219; config/src/lib.rs:154-156)."""
    import json
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    out = tmp_path / "log.json"
    env = dict(os.environ, NWC_AUTO_KEYS="4")
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "autokeys_lifecycle_helper.py"), ROOT, str(out)],
                   env=env, check=True, timeout=300)
    log = {e["tag"]: e for e in json.load(open(out))}
    for e in log.values():
        want_bad = 0 if e["corrupt"] is None else 1 << e["corrupt"]
        assert e["rc"] == (0 if e["corrupt"] is None else 1) and e["bad"] == want_bad, e
        assert e["cap"] == 4
    assert log["A1"]["auto"] == 2 and log["A2"]["hits"] == log["A1"]["hits"] + 1
    assert log["B1"]["auto"] == 4 and log["B2"]["hits"] == log["B1"]["hits"] + 1
    assert log["C1"]["auto"] == 4 and log["C2"]["hits"] == log["C1"]["hits"] + 1      # replaced, then cached
    assert log["A-after-eviction"]["hits"] == log["C2"]["hits"]                        # evicted: uncached path
    assert log["C-cached"]["hits"] == log["C2"]["hits"] + 1
    assert log["after-committee"]["auto"] == 0 and log["after-committee"]["committee"] == 2
    assert log["after-committee"]["hits"] == log["C-cached"]["hits"]
    assert log["C-again2"]["hits"] == log["C-again1"]["hits"] + 1 and log["C-again1"]["auto"] == 2
