"""Large host calls (the Rust shim's situation: pageable host buffers in, bitmaps out) against the
oracle: nwc_verify_strict_many and nwc_verify_batch_many over several pipelined chunks, whose
inputs travel through the device's pinned stages (copy_pool.h HostStager) -- chunk boundaries,
stage boundaries (32 MB) and the verdict merge all crossed -- and, for the certificates, launch
keys picking the committee up inside the chunks (crypto/src/lib.rs:200-219)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _bits(buf, n):
    return np.unpackbits(np.frombuffer(buf.raw, np.uint8), bitorder="little")[:n].astype(bool)


def test_strict_many_host_chunks(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(81)
    n = 400_000   # chunks of 131,072 then x3: two chunks, the second across stage boundaries
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    bad = rng.random(n) < 0.02
    bad[[0, 63, 64, 131071, 131072, 131073, n - 1]] = True
    sigs[bad, 45] ^= 4
    out = ctypes.create_string_buffer((n + 7) // 8)
    _lib.check(lib.nwc_verify_strict_many(_lib.buf(msgs), _lib.buf(pks), _lib.buf(sigs), n, out))
    got = _bits(out, n)
    exp = oracle.strict_many(msgs, pks, sigs)
    assert (exp == ~bad).all()
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_batch_many_host_chunks(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    rng = np.random.default_rng(82)
    m, Q, N = 6000, 67, 100
    cseeds = rng.integers(0, 256, (N, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    voters = np.argsort(rng.random((m, N)), axis=1)[:, :Q].reshape(-1)
    signed = np.repeat(dig, Q, axis=0)
    bad = rng.random(m * Q) < 0.01
    signed[bad, 3] ^= 1
    pks, sigs = oracle.keygen_sign_many(cseeds[voters], signed)
    offs = (np.arange(m + 1) * Q).astype(np.uint32)
    cert = ctypes.create_string_buffer((m + 7) // 8)
    badb = ctypes.create_string_buffer((m * Q + 7) // 8)
    for _ in range(2):   # first call: the launch keys join; second: steady state
        _lib.check(lib.nwc_verify_batch_many(_lib.buf(dig), _lib.buf(offs), _lib.buf(pks), _lib.buf(sigs), m, cert, badb))
        assert (_bits(badb, m * Q) == bad).all()
        assert (_bits(cert, m) == ~bad.reshape(m, Q).any(axis=1)).all()
    ocert, obad = oracle.batch_many(dig, offs, pks, sigs)
    assert (obad == bad).all() and (ocert == ~bad.reshape(m, Q).any(axis=1)).all()
    h = ctypes.c_uint32()
    _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
    assert h.value == N
    _lib.check(lib.nwc_set_committee(None, 0))
