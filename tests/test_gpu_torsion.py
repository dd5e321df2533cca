"""Batch-leaf parity for keys with an 8-torsion component (dalek verify_batch's randomized domain).

dalek 1.0.1 scales A_i by (z_i k_i mod l) (crypto/src/lib.rs:218 -> ed25519-dalek batch.rs), so
a vote whose key A = A' + T (T != O) contributes a random multiple of l*T to the batch sum even
when its own residual e_i = O: the reference verdict is randomized and the build answers Err
(oracle/ed25519_ref.py vote_class).  The fixtures' `leaf` field carries that.
Every path must agree: uncached keys (k_tors_* post-pass with per-launch key dedup), cached keys
(KEY_TORSION flag in the comb, latency and cached-ladder kernels) and the comb path's uncached
list.  Batches repeat each key many times, as committees do.
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from narwhal_amd import _lib
    return _lib.load()


def _set_committee(lib, keys):
    from narwhal_amd import _lib
    if keys is None or len(keys) == 0:
        _lib.check(lib.nwc_set_committee(None, 0))
    else:
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        _lib.check(lib.nwc_set_committee(_lib.buf(keys), len(keys)))


def _leaf(m, p, s):
    import torch
    from narwhal_amd import device
    tm, tp, ts = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (m, p, s))
    w = device.verify(tm, tp, ts, strict=False)
    torch.cuda.synchronize()
    return device.unpack_bits(w, p.shape[0])


def _cases(golden_verify):
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    arr = lambda k: np.stack([np.frombuffer(bytes.fromhex(c[k]), np.uint8) for c in cases])  # noqa: E731
    return cases, arr("msg"), arr("pk"), arr("sig")


def test_torsion_keys_every_path(lib, golden_verify):
    cases, m, p, s = _cases(golden_verify)
    tors = [i for i, c in enumerate(cases) if c["name"].startswith("mixed-order-A") and c["name"].endswith("kT0")]
    assert len(tors) == 7 and all(cases[i]["strict"] and not cases[i]["leaf"] for i in tors)
    rng = np.random.default_rng(2)
    n = 5000
    # half the equations are the torsion-key votes (each key ~350 times), the rest any golden case
    idx = np.where(rng.random(n) < 0.5, rng.choice(tors, n), rng.integers(0, len(cases), n))
    exp = np.array([cases[i]["leaf"] for i in idx])
    M, P, S = m[idx], p[idx], s[idx]
    tors_keys = np.unique(p[tors], axis=0)
    all_keys = np.unique(p, axis=0)
    others = np.array([k for k in all_keys if not any((k == t).all() for t in tors_keys)])
    try:
        for label, committee in (("uncached", None), ("all cached (comb)", all_keys),
                                 ("torsion keys uncached (comb list)", others)):
            _set_committee(lib, committee)
            got = _leaf(M, P, S)
            bad = [(int(k), cases[idx[k]]["name"]) for k in np.nonzero(got != exp)[0][:6]]
            assert not bad, (label, bad)
    finally:
        _set_committee(lib, None)


def test_torsion_batches_through_host_abi(lib, golden_batch, golden_verify):
    """nwc_verify_batch (latency kernel when every key is cached) and nwc_verify_batch_many on the
    golden torsion batches: verdict Err and the exact bad-vote set."""
    from narwhal_amd import _lib
    tb = [b for b in golden_batch if "kT0-in-batch" in b["name"] or "zero-residual" in b["name"]]
    assert len(tb) >= 11
    keys = np.unique(np.stack([np.frombuffer(bytes.fromhex(pk), np.uint8) for b in tb for pk, _ in b["votes"]]), axis=0)
    try:
        for committee in (None, keys):
            _set_committee(lib, committee)
            for b in tb:
                n = len(b["votes"])
                P = np.stack([np.frombuffer(bytes.fromhex(pk), np.uint8) for pk, _ in b["votes"]])
                S = np.stack([np.frombuffer(bytes.fromhex(sg), np.uint8) for _, sg in b["votes"]])
                msg = np.frombuffer(bytes.fromhex(b["msg"]), np.uint8)
                bad = ctypes.create_string_buffer((n + 7) // 8)
                rc = _lib.check(lib.nwc_verify_batch(_lib.buf(msg), _lib.buf(P), _lib.buf(S), n, bad))
                got_bad = list(np.nonzero(np.unpackbits(np.frombuffer(bad.raw, np.uint8), bitorder="little")[:n])[0])
                assert (rc == 0) == b["verdict"] and got_bad == b["bad"], (b["name"], committee is not None)
            # all torsion batches as certificates of one verify_batch_many call
            digests = np.stack([np.frombuffer(bytes.fromhex(b["msg"]), np.uint8) for b in tb])
            offs = np.concatenate([[0], np.cumsum([len(b["votes"]) for b in tb])]).astype(np.uint32)
            P = np.stack([np.frombuffer(bytes.fromhex(pk), np.uint8) for b in tb for pk, _ in b["votes"]])
            S = np.stack([np.frombuffer(bytes.fromhex(sg), np.uint8) for b in tb for _, sg in b["votes"]])
            cert = ctypes.create_string_buffer((len(tb) + 7) // 8)
            badv = ctypes.create_string_buffer((int(offs[-1]) + 7) // 8)
            _lib.check(lib.nwc_verify_batch_many(_lib.buf(digests), _lib.buf(offs), _lib.buf(P), _lib.buf(S), len(tb),
                                                 cert, badv))
            bits = np.unpackbits(np.frombuffer(badv.raw, np.uint8), bitorder="little")[:int(offs[-1])]
            exp_bad = np.zeros(int(offs[-1]), np.uint8)
            for c, b in enumerate(tb):
                exp_bad[[offs[c] + j for j in b["bad"]]] = 1
            assert (bits == exp_bad).all()
            got_cert = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:len(tb)].astype(bool)
            assert (got_cert == np.array([b["verdict"] for b in tb])).all()
    finally:
        _set_committee(lib, None)
