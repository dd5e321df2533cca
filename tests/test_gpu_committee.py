"""Committee key cache (nwc_set_committee): verdicts with the cache equal verdicts without it
and the oracle's, for members, non-members (mixed waves), an undecodable key and small-order keys."""
import ctypes
import hashlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(raw, n):
    return np.unpackbits(np.frombuffer(raw, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def _batch_many(lib, digests, offs, p, s):
    from narwhal_amd import _lib
    m = len(offs) - 1
    cert = ctypes.create_string_buffer((m + 7) // 8)
    bad = ctypes.create_string_buffer((int(offs[-1]) + 7) // 8)
    _lib.check(lib.nwc_verify_batch_many(_lib.buf(digests), _lib.buf(offs), _lib.buf(p), _lib.buf(s), m, cert, bad))
    return _bits(cert.raw, m), _bits(bad.raw, int(offs[-1]))


def test_committee_cache_parity(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(31)
    N, Q, m = 100, 67, 200
    seeds = rng.integers(0, 256, (N + 20, 32), dtype=np.uint8)
    committee_pk, _ = oracle.keygen_sign_many(seeds[:N], np.zeros((N, 32), np.uint8))
    # poison two committee slots: an undecodable key (y = 2) and a small-order key (identity)
    bogus = np.zeros((2, 32), np.uint8)
    bogus[0, 0] = 2
    bogus[1, 0] = 1
    committee = np.concatenate([committee_pk, bogus])
    digests = np.stack([np.frombuffer(hashlib.sha512(b"c" + bytes([c % 256, c // 256])).digest()[:32], np.uint8)
                        for c in range(m)])
    voter = np.stack([rng.permutation(N + 20)[:Q] for _ in range(m)])   # some non-members (ids >= N)
    vs = seeds[voter.reshape(-1)]
    vm = np.repeat(digests, Q, axis=0).copy()
    badmask = rng.random(m * Q) < 0.02
    vm_signed = vm.copy()
    vm_signed[badmask, 0] ^= 1
    pks, sigs = oracle.keygen_sign_many(vs, vm_signed)
    # a few votes by the bogus keys (identity-trick signature for the small-order one)
    pks[5] = bogus[0]
    pks[77] = bogus[1]
    sigs[77, :32] = bogus[1]
    sigs[77, 32:] = 0
    offs = (np.arange(m + 1) * Q).astype(np.uint32)
    ocert, obad = oracle.batch_many(digests, offs, pks, sigs)
    assert obad[5] and not obad[77]          # small-order identity trick is a valid leaf
    try:
        _lib.check(lib.nwc_set_committee(None, 0))
        c0, b0 = _batch_many(lib, digests, offs, pks, sigs)
        _lib.check(lib.nwc_set_committee(_lib.buf(committee), len(committee)))
        c1, b1 = _batch_many(lib, digests, offs, pks, sigs)
        # certificates whose voters are all members: make one wave fully cached
        mem = voter.copy()
        mem[:] = np.stack([rng.permutation(N)[:Q] for _ in range(m)])
        vs2 = seeds[mem.reshape(-1)]
        pk2, sg2 = oracle.keygen_sign_many(vs2, vm_signed)
        oc2, ob2 = oracle.batch_many(digests, offs, pk2, sg2)
        c2, b2 = _batch_many(lib, digests, offs, pk2, sg2)
        # strict verify of member-signed triples through the cached kernel
        out = ctypes.create_string_buffer((m * Q + 7) // 8)
        _lib.check(lib.nwc_verify_strict_many(_lib.buf(vm_signed), _lib.buf(pk2), _lib.buf(sg2), m * Q, out))
        st = _bits(out.raw, m * Q)
    finally:
        _lib.check(lib.nwc_set_committee(None, 0))
    assert (c0 == ocert).all() and (b0 == obad).all()
    assert (c1 == ocert).all() and (b1 == obad).all()
    assert (c2 == oc2).all() and (b2 == ob2).all()
    assert (st == oracle.strict_many(vm_signed, pk2, sg2)).all()
