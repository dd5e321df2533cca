"""GPU edge cases of the C ABI: empty and ragged inputs, and concurrent callers.

The reference calls the crate from concurrent tokio tasks (`primary/src/core.rs:88-114`,
`worker/src/worker.rs:182,227`), with empty vote lists (`crypto/src/lib.rs:206-219`: an empty
iterator verifies) and batches of any length, so the ABI must give exact verdicts at every size
and from several host threads at once.  Expected verdicts: the oracle (tests/oracle_lib.py) and
hashlib.
"""
import ctypes
import hashlib
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    from narwhal_amd import _lib
    return _lib.load()


@pytest.fixture(scope="module")
def orc():
    from tests.oracle_lib import load_oracle
    return load_oracle()


def _bits(raw: bytes, n: int) -> np.ndarray:
    return np.unpackbits(np.frombuffer(raw, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def _signed_set(orc, n: int, seed: int, bad_every: int = 0):
    """n (msg, pk, sig) triples signed by the oracle; every bad_every-th signature corrupted."""
    rng = np.random.default_rng(seed)
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks = np.zeros((n, 32), np.uint8)
    sigs = np.zeros((n, 64), np.uint8)
    for i in range(n):
        pks[i] = np.frombuffer(orc.public_key(seeds[i].tobytes()), np.uint8)
        sigs[i] = np.frombuffer(orc.sign(seeds[i].tobytes(), msgs[i].tobytes()), np.uint8)
        if bad_every and i % bad_every == bad_every - 1:
            sigs[i, 5 + i % 50] ^= 1 << (i % 8)
    return msgs, pks, sigs


def _strict_many(lib, msgs, pks, sigs):
    from narwhal_amd import _lib
    n = pks.shape[0]
    out = ctypes.create_string_buffer(max(1, (n + 7) // 8))
    _lib.check(lib.nwc_verify_strict_many(_lib.buf(msgs), _lib.buf(pks), _lib.buf(sigs), n, out))
    return _bits(out.raw, n)


def test_empty_inputs(lib):
    """n = 0 everywhere: an empty vote list verifies (lib.rs:206-219), empty calls succeed, and a
    zero-length message digests to SHA-512("")[..32]."""
    from narwhal_amd import _lib
    z32 = bytes(32)
    assert lib.nwc_verify_batch(z32, None, None, 0, None) == 0
    assert lib.nwc_verify_strict_many(None, None, None, 0, None) == 0
    offs = np.zeros(1, np.uint32)
    assert lib.nwc_verify_batch_many(None, _lib.buf(offs), None, None, 0, None, None) == 0
    # a certificate with no votes between two with votes is valid (empty batch)
    dig = np.zeros((3, 32), np.uint8)
    offs = np.array([0, 0, 0, 0], np.uint32)
    cert = ctypes.create_string_buffer(1)
    _lib.check(lib.nwc_verify_batch_many(_lib.buf(dig), _lib.buf(offs), None, None, 3, cert, None))
    assert _bits(cert.raw, 3).all()
    o64 = np.zeros(2, np.uint64)
    out = ctypes.create_string_buffer(32)
    _lib.check(lib.nwc_sha512_trunc32_many(b"", _lib.buf(o64), 1, out))
    assert out.raw == hashlib.sha512(b"").digest()[:32]
    assert lib.nwc_sha512_trunc32_many(None, _lib.buf(o64), 0, None) == 0


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 129, 255, 257, 1000])
def test_ragged_sizes_strict(lib, orc, n):
    """verdict bitmaps at sizes around the wave (64) and word boundaries, 1/7 corrupted."""
    msgs, pks, sigs = _signed_set(orc, n, seed=n, bad_every=7)
    got = _strict_many(lib, msgs, pks, sigs)
    exp = orc.strict_many(msgs, pks, sigs, threads=4).astype(bool)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    assert got.sum() == n - n // 7


@pytest.mark.parametrize("n", [1, 3, 64, 65, 300])
def test_ragged_batch_bad_sets(lib, orc, n):
    """verify_batch over one digest: verdict and the exact bad-vote set at ragged sizes."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(100 + n)
    digest = rng.integers(0, 256, 32, dtype=np.uint8)
    _, pks, sigs = _signed_set(orc, n, seed=200 + n)
    # re-sign every vote over the one digest, corrupt every 5th
    seeds = np.random.default_rng(200 + n).integers(0, 256, (n, 32), dtype=np.uint8)
    for i in range(n):
        sigs[i] = np.frombuffer(orc.sign(seeds[i].tobytes(), digest.tobytes()), np.uint8)
        if i % 5 == 4:
            sigs[i, 33] ^= 0x10
    bad = ctypes.create_string_buffer((n + 7) // 8)
    rc = lib.nwc_verify_batch(_lib.buf(digest), _lib.buf(pks), _lib.buf(sigs), n, bad)
    exp_bad = np.array([i % 5 == 4 for i in range(n)])
    assert rc == (1 if exp_bad.any() else 0)
    assert (_bits(bad.raw, n) == exp_bad).all()


def test_concurrent_host_calls(lib, orc):
    """8 host threads calling verify_batch / verify_strict_many / the digest at the same time (ctypes
    drops the GIL inside the call): every result exact."""
    from narwhal_amd import _lib
    sets = [_signed_set(orc, 40 + 13 * t, seed=300 + t, bad_every=(0 if t % 2 else 9)) for t in range(8)]
    exp = [orc.strict_many(m, p, s, threads=2).astype(bool) for m, p, s in sets]
    blobs = [np.random.default_rng(400 + t).integers(0, 256, 5000 + 777 * t, dtype=np.uint8) for t in range(8)]
    errors = []

    def worker(t):
        try:
            m, p, s = sets[t]
            for it in range(25):
                got = _strict_many(lib, m, p, s)
                if not (got == exp[t]).all():
                    errors.append((t, it, "strict"))
                rc = lib.nwc_verify_batch(_lib.buf(m[0]), _lib.buf(p[:1]), _lib.buf(s[:1]), 1, None)
                if rc != (0 if exp[t][0] else 1):
                    errors.append((t, it, "batch", rc))
                offs = np.array([0, len(blobs[t])], np.uint64)
                out = ctypes.create_string_buffer(32)
                if lib.nwc_sha512_trunc32_many(_lib.buf(blobs[t]), _lib.buf(offs), 1, out) != 0 or \
                        out.raw != hashlib.sha512(blobs[t].tobytes()).digest()[:32]:
                    errors.append((t, it, "digest"))
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((t, repr(e)))

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=150)
    assert not any(th.is_alive() for th in threads), "a host thread did not finish"
    assert not errors, errors[:5]
