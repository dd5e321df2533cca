"""Doubling-free committee path (k_verify_comb): with the committee cache set, equations whose key
is cached are decided by the comb sum R' = sB + k(-A) and the compressed comparison with R.  The
verdicts must equal the oracle's (dalek semantics) on every golden edge case, on randomly mutated
committee votes (incl. non-members in the same waves, which take the list-mode k_verify), and at
full size through the exact-failure property (several batched-inversion chunks per lane)."""
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


def _dev_verify(m, p, s, strict):
    import torch
    from narwhal_amd import device
    tm, tp, ts = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (m, p, s))
    w = device.verify(tm, tp, ts, strict=strict)
    torch.cuda.synchronize()
    return device.unpack_bits(w, p.shape[0])


def _golden_arrays(golden_verify):
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    m = np.stack([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in cases])
    p = np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in cases])
    s = np.stack([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in cases])
    return cases, m, p, s


def test_comb_golden_edge_cases(lib, golden_verify):
    """Every golden case with its key in the committee: small-order / non-canonical / undecodable
    keys, small-order and non-canonical R, s >= l, sign-bit flips, the identity trick."""
    cases, m, p, s = _golden_arrays(golden_verify)
    committee = np.unique(p, axis=0)
    try:
        _set_committee(lib, committee)
        for rep in (1, 7):   # 7 copies: several lanes and batched-inversion slots per case
            mm, pp, ss = (np.tile(x, (rep, 1)) for x in (m, p, s))
            st = _dev_verify(mm, pp, ss, True)
            lf = _dev_verify(mm, pp, ss, False)
            exp_st = np.tile(np.array([c["strict"] for c in cases]), rep)
            exp_lf = np.tile(np.array([c["leaf"] for c in cases]), rep)
            bad = [cases[i % len(cases)]["name"] for i in np.nonzero(st != exp_st)[0][:5]]
            assert (st == exp_st).all(), bad
            bad = [cases[i % len(cases)]["name"] for i in np.nonzero(lf != exp_lf)[0][:5]]
            assert (lf == exp_lf).all(), bad
    finally:
        _set_committee(lib, None)


def _mutated_committee_votes(oracle, rng, n, members, seeds):
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    who = rng.integers(0, len(seeds), n)
    pks, sigs = oracle.keygen_sign_many(seeds[who], msgs)
    kind = rng.integers(0, 10, n)
    L = (1 << 252) + 27742317777372353535851937790883648493
    for i in np.nonzero(kind == 1)[0]:                     # random bit flip in the signature
        sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
    for i in np.nonzero(kind == 2)[0]:                     # wrong message
        msgs[i, rng.integers(0, 32)] ^= 1
    for i in np.nonzero(kind == 3)[0]:                     # s + l (non-canonical scalar)
        sv = int.from_bytes(sigs[i, 32:].tobytes(), "little") + L
        if sv < (1 << 256):
            sigs[i, 32:] = np.frombuffer(sv.to_bytes(32, "little"), np.uint8)
    small_y = [0, 1, (1 << 255) - 20]                      # y = 0, 1, -1: small-order R encodings
    for i in np.nonzero(kind == 4)[0]:                     # small-order or non-canonical R
        y = small_y[rng.integers(0, 3)] + (((1 << 255) - 19) if rng.random() < 0.3 else 0)
        y &= (1 << 255) - 1
        if rng.random() < 0.5:
            y |= 1 << 255
        sigs[i, :32] = np.frombuffer(y.to_bytes(32, "little"), np.uint8)
    for i in np.nonzero(kind == 5)[0]:                     # flip the sign bit of R
        sigs[i, 31] ^= 0x80
    return msgs, pks, sigs, who


def test_comb_mutated_votes_vs_oracle(lib, oracle):
    rng = np.random.default_rng(77)
    N = 100
    seeds = rng.integers(0, 256, (N + 30, 32), dtype=np.uint8)   # 30 non-members
    committee, _ = oracle.keygen_sign_many(seeds[:N], np.zeros((N, 32), np.uint8))
    try:
        _set_committee(lib, committee)
        for n in (1, 3, 64, 300, 20000):
            m, p, s, _ = _mutated_committee_votes(oracle, rng, n, committee, seeds)
            st = _dev_verify(m, p, s, True)
            lf = _dev_verify(m, p, s, False)
            exp_st = oracle.strict_many(m, p, s)
            exp_lf = oracle.leaf_many(m, p, s)
            assert (st == exp_st).all(), (n, np.nonzero(st != exp_st)[0][:10])
            assert (lf == exp_lf).all(), (n, np.nonzero(lf != exp_lf)[0][:10])
    finally:
        _set_committee(lib, None)


def test_comb_certificates_match_uncached(lib, oracle):
    """verify_batch_many over committee certificates: comb path == no cache == oracle."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(5)
    N, Q, m = 100, 67, 300
    seeds = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    committee, _ = oracle.keygen_sign_many(seeds, np.zeros((N, 32), np.uint8))
    digests = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    voter = np.stack([rng.permutation(N)[:Q] for _ in range(m)]).reshape(-1)
    signed = np.repeat(digests, Q, axis=0)
    bad = rng.random(m * Q) < 0.01
    signed[bad, 3] ^= 0x40
    pks, sigs = oracle.keygen_sign_many(seeds[voter], signed)
    offs = (np.arange(m + 1) * Q).astype(np.uint32)
    ocert, obad = oracle.batch_many(digests, offs, pks, sigs)

    def run():
        cert = ctypes.create_string_buffer((m + 7) // 8)
        badv = ctypes.create_string_buffer((m * Q + 7) // 8)
        _lib.check(lib.nwc_verify_batch_many(_lib.buf(digests), _lib.buf(offs), _lib.buf(pks), _lib.buf(sigs), m,
                                             cert, badv))
        bits = lambda raw, k: np.unpackbits(np.frombuffer(raw, np.uint8), bitorder="little")[:k].astype(bool)  # noqa
        return bits(cert.raw, m), bits(badv.raw, m * Q)

    try:
        _set_committee(lib, committee)
        c1, b1 = run()
    finally:
        _set_committee(lib, None)
    c0, b0 = run()
    assert (c1 == ocert).all() and (b1 == obad).all()
    assert (c0 == ocert).all() and (b0 == obad).all()
    assert (b1 == bad).all()


@pytest.mark.slow
def test_comb_full_size_exact_failures(lib, oracle):
    """2.2M committee votes (several COMB_BATCH chunks per lane): all valid verify, then exactly
    the corrupted indices fail."""
    import torch
    from narwhal_amd import device
    N, n = 100, 2_200_000
    kseeds = device.derive32(b"nw-committee", 0, N)
    committee, _ = device.keygen_sign(kseeds, device.derive32(b"nw-zero", 0, N))
    who = torch.from_numpy(np.random.default_rng(3).integers(0, N, n)).cuda()
    msgs = device.derive32(b"comb-msg", 0, n)
    pks, sigs = device.keygen_sign(kseeds[who].contiguous(), msgs)
    torch.cuda.synchronize()
    try:
        _set_committee(lib, committee.cpu().numpy())
        words = device.verify(msgs, pks, sigs, strict=True)
        torch.cuda.synchronize()
        assert device.unpack_bits(words, n).all()
        idx = np.sort(np.random.default_rng(4).choice(n, 301, replace=False))
        ti = torch.from_numpy(idx).cuda()
        sigs[ti, 50] ^= 0x08
        words = device.verify(msgs, pks, sigs, strict=True)
        torch.cuda.synchronize()
        got = device.unpack_bits(words, n)
        assert list(np.nonzero(~got)[0]) == list(idx)
    finally:
        _set_committee(lib, None)
    sub = [t[ti].cpu().numpy() for t in (msgs, pks, sigs)]
    assert not oracle.strict_many(*sub).any()


def test_comb_small_host_calls(lib, golden_verify, oracle):
    """Small host calls with every key cached take the single-launch latency kernel (pinned
    staging, zeroed verdict words in the same copy); mixed batches take the general path."""
    from narwhal_amd import _lib
    cases, m, p, s = _golden_arrays(golden_verify)
    committee = np.unique(p, axis=0)
    try:
        _set_committee(lib, committee)
        for i, c in enumerate(cases):
            rc = _lib.check(lib.nwc_verify_strict(_lib.buf(m[i]), _lib.buf(p[i]), _lib.buf(s[i])))
            assert (rc == 0) == c["strict"], c["name"]
        # batches of 1..70 votes over one digest (verify_batch leaf semantics)
        rng = np.random.default_rng(9)
        for n in (1, 3, 64, 65, 70):
            idx = rng.integers(0, len(cases), n)
            msg = m[idx[0]]
            bad = ctypes.create_string_buffer((n + 7) // 8)
            P, S = np.ascontiguousarray(p[idx]), np.ascontiguousarray(s[idx])   # keep the buffers alive
            rc = _lib.check(lib.nwc_verify_batch(_lib.buf(msg), _lib.buf(P), _lib.buf(S), n, bad))
            got_bad = np.unpackbits(np.frombuffer(bad.raw, np.uint8), bitorder="little")[:n].astype(bool)
            exp_leaf = np.array([oracle.leaf(msg, p[j], s[j]) for j in idx])   # all votes sign `msg`
            diff = np.nonzero(got_bad != ~exp_leaf)[0]
            assert len(diff) == 0, (n, [(int(k), cases[idx[k]]["name"], bool(got_bad[k])) for k in diff[:8]],
                                    cases[idx[0]]["name"])
            assert (rc == 0) == bool(exp_leaf.all())
        # a batch with one key outside the committee -> general path, same verdicts
        _set_committee(lib, committee[1:])
        outside = np.nonzero((p == committee[0]).all(axis=1))[0]
        if len(outside):
            i = int(outside[0])
            rc = _lib.check(lib.nwc_verify_strict(_lib.buf(m[i]), _lib.buf(p[i]), _lib.buf(s[i])))
            assert (rc == 0) == cases[i]["strict"]
    finally:
        _set_committee(lib, None)


def test_latency_kernel_mutated_votes_vs_oracle(lib, oracle):
    """The latency kernel (limb-sliced decompression of R, zero-copy call) on single votes through
    the host ABI: random signature bit flips, wrong messages, s + l, small-order and non-canonical
    R, flipped R sign bits and random R bytes (mostly non-decoding), against the oracle."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(78)
    N = 16
    seeds = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    committee, _ = oracle.keygen_sign_many(seeds, np.zeros((N, 32), np.uint8))
    m, p, s, _ = _mutated_committee_votes(oracle, rng, 1500, committee, seeds)
    rnd = rng.random(len(s)) < 0.1
    s[rnd, :32] = rng.integers(0, 256, (int(rnd.sum()), 32), dtype=np.uint8)   # arbitrary R bytes
    exp_st = oracle.strict_many(m, p, s)
    exp_lf = oracle.leaf_many(m, p, s)
    try:
        _set_committee(lib, committee)
        for i in range(len(s)):
            rc = _lib.check(lib.nwc_verify_strict(_lib.buf(m[i]), _lib.buf(p[i]), _lib.buf(s[i])))
            assert (rc == 0) == exp_st[i], i
            bad = ctypes.create_string_buffer(1)
            rc = _lib.check(lib.nwc_verify_batch(_lib.buf(m[i]), _lib.buf(p[i]), _lib.buf(s[i]), 1, bad))
            assert (rc == 0) == exp_lf[i], i
        assert exp_st.sum() > 100 and (~exp_st).sum() > 100
    finally:
        _set_committee(lib, None)
