"""dalek's batch semantics at the comb path's rate (crypto/src/lib.rs:206-219 -> ed25519-dalek 1.0.1
verify_batch; narwhal_amd/csrc/resolve.h).

nwc_dev_verify_batch_msm / nwc_verify_batch_msm_many, when key combs apply (a committee cache, or a
launch of >= 65,536 votes whose keys repeat: launch keys), decide every vote by the exact leaves and
then evaluate dalek's equation once per certificate over the votes the leaves rejected, in
E[8] = Z/8.  With the per-launch seed fixed (nwc_diag_set("dalek_seed")), z_i = SHA-512(seed ||
u64le(i))[..16] is known, so every certificate -- the randomized domain included -- is checked
EXACTLY against the C oracle's evaluation of dalek's equation for the same z_i
(orc_batch_z8, itself pinned to the term-by-term equation in tests/test_oracle_golden.py)."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

Q = 67


def _seed_bytes(seed: int) -> bytes:
    return seed.to_bytes(4, "little") + bytes(28)


def _zs(seed: int, nv: int) -> np.ndarray:
    sb = _seed_bytes(seed)
    return np.frombuffer(b"".join(hashlib.sha512(sb + v.to_bytes(8, "little")).digest()[:16] for v in range(nv)),
                         np.uint8).reshape(nv, 16)


def _instance(oracle, golden_batch, filler_certs=1000, bad_rate=0.0, seed=5):
    """Honest 67-vote certificates of a 100-key committee (enough votes for launch keys), then every
    non-empty golden batch as a certificate of its own, then the empty one."""
    rng = np.random.default_rng(seed)
    kseeds = rng.integers(0, 256, (100, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (filler_certs, 32), dtype=np.uint8)
    who = np.concatenate([rng.permutation(100)[:Q] for _ in range(filler_certs)])
    pks, sigs = oracle.keygen_sign_many(kseeds[who], np.repeat(dig, Q, axis=0))
    bad = rng.random(filler_certs * Q) < bad_rate
    sigs[bad, 33] ^= 1
    sizes = [Q] * filler_certs
    digs, P, S = [dig], [pks], [sigs]
    names = ["filler"] * filler_certs
    for b in golden_batch:
        if len(bytes.fromhex(b["msg"])) != 32:
            continue
        n = len(b["votes"])
        digs.append(np.frombuffer(bytes.fromhex(b["msg"]), np.uint8)[None, :])
        if n:
            P.append(np.frombuffer(b"".join(bytes.fromhex(p) for p, _ in b["votes"]), np.uint8).reshape(n, 32))
            S.append(np.frombuffer(b"".join(bytes.fromhex(s) for _, s in b["votes"]), np.uint8).reshape(n, 64))
        sizes.append(n)
        names.append(b["name"])
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    committee = np.unique(np.concatenate([oracle.keygen_sign_many(kseeds, np.zeros((100, 32), np.uint8))[0]] +
                                         [p for p in P[1:]]), axis=0)
    return (np.concatenate(digs), offs, np.concatenate(P), np.concatenate(S), names, committee)


def _dev_run(dig, offs, pks, sigs):
    import torch
    from narwhal_amd import device
    m, nv = len(offs) - 1, int(offs[-1])
    mi = np.repeat(np.arange(m, dtype=np.int32), np.diff(offs))
    t = lambda a, dt=torch.uint8: torch.from_numpy(np.ascontiguousarray(a)).to(dt).cuda()  # noqa: E731
    do = t(offs.astype(np.int32), torch.int32)
    leaf = device.verify_batch_msm(t(dig), do, t(mi, torch.int32), t(pks), t(sigs))
    cert, bad = device.cert_reduce(leaf, do, nv)
    torch.cuda.synchronize()
    return device.unpack_bits(cert, m), device.unpack_bits(bad, nv)


def _expected(oracle, dig, offs, pks, sigs, seed):
    nv = int(offs[-1])
    cert = oracle.batch_z_many(dig, offs.astype(np.uint32), pks, sigs, _zs(seed, nv), z8=True)
    # votes of a certificate the equation rejects: the exact leaves' failures (the bisection's set)
    leaf = oracle.leaf_many(np.repeat(dig, np.diff(offs), axis=0), pks, sigs).astype(bool)
    bad = ~leaf & ~np.repeat(cert, np.diff(offs))
    return cert, bad


@pytest.mark.parametrize("keys", ["launch", "committee"])
def test_every_certificate_equals_dalek_equation_for_the_same_z(oracle, golden_batch, keys):
    """Launch keys (the golden batches' odd keys stay uncached: the ladder inside the resolution) and
    a committee cache holding every key (torsion-bearing and undecodable ones included: the comb
    inside the resolution).  Five seeds: every certificate's verdict and bad-vote set equal the
    oracle's for the same z_i, and both dalek outcomes occur on the randomized class."""
    from narwhal_amd import _lib
    lib = _lib.load()
    dig, offs, pks, sigs, names, committee = _instance(oracle, golden_batch)
    rand = [i for i, n in enumerate(names) if n != "filler" and
            {b["name"]: b["class"] for b in golden_batch}.get(n) == "randomized"]
    outcomes = set()
    try:
        if keys == "committee":
            _lib.check(lib.nwc_set_committee(_lib.buf(np.ascontiguousarray(committee)), len(committee)))
        for seed in (11, 12, 13, 14, 15):
            _lib.diag_set("dalek_seed", seed)
            cert, bad = _dev_run(dig, offs, pks, sigs)
            ocert, obad = _expected(oracle, dig, offs, pks, sigs, seed)
            assert (cert == ocert).all(), [names[i] for i in np.nonzero(cert != ocert)[0]]
            assert (bad == obad).all(), np.nonzero(bad != obad)[0][:10]
            assert cert[:1000].all()
            outcomes |= {bool(cert[i]) for i in rand}
    finally:
        _lib.diag_set("dalek_seed", 0)
        _lib.check(lib.nwc_set_committee(None, 0))
    assert outcomes == {True, False}


def test_one_percent_bad_committee_traffic(oracle, golden_batch):
    """Config 3 in miniature with launch keys: 1,500 certificates x 67 votes, 1 % bad (deterministic
    domain): verdicts and bad sets equal the oracle's leaves, whatever the seed."""
    from narwhal_amd import _lib
    dig, offs, pks, sigs, names, _ = _instance(oracle, [], filler_certs=1500, bad_rate=0.01, seed=9)
    ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs)
    cert, bad = _dev_run(dig, offs, pks, sigs)
    assert (cert == ocert).all() and (bad == obad).all()
    assert (~ocert).sum() > 300


def test_host_entry_fixed_seed(oracle, golden_batch):
    """nwc_verify_batch_msm_many (host buffers, one device range: vote indices are the call's) with a
    fixed seed: certificate bits equal the oracle's equation for the same z_i."""
    from narwhal_amd import _lib
    lib = _lib.load()
    dig, offs, pks, sigs, names, _ = _instance(oracle, golden_batch)
    m, nv = len(dig), int(offs[-1])
    offs32 = offs.astype(np.uint32)
    cert = ctypes.create_string_buffer((m + 7) // 8)
    badb = ctypes.create_string_buffer((nv + 7) // 8)
    try:
        _lib.diag_set("dalek_seed", 21)
        _lib.check(lib.nwc_verify_batch_msm_many(_lib.buf(dig), _lib.buf(offs32), _lib.buf(pks), _lib.buf(sigs), m,
                                                 cert, badb))
    finally:
        _lib.diag_set("dalek_seed", 0)
    c = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:m].astype(bool)
    b = np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:nv].astype(bool)
    ocert, obad = _expected(oracle, dig, offs, pks, sigs, 21)
    assert (c == ocert).all() and (b == obad).all()
