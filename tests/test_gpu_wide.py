"""GPU parity of the half-size ladder's wide windows (narwhal_amd/csrc/kernels.hip, half_scalarmult).

The window count W is wave-uniform: the smallest W in [33, 37] covering max(|c|, d) of every lane
(lattice.h).  ~9 % of random waves run W = 34 and rarely more, so the random parity tests reach the
wide digit layouts only by chance.  Here triples whose challenge reduces to 132+ bit scalars are
searched among device-generated signatures (the host restatement of the reduction picks them), each
is placed in a wave of its own with 63 ordinary triples, a quarter of all triples are corrupted, and
the verdicts are compared with the oracle (dalek verify_strict restated).  Natural 136+-bit lanes
(W >= 35) are rarer than 1 in 10^6, so W = 34..37 are also forced on ordinary batches through the
nwc_diag_set("force_windows") test hook (extra top windows carry zero digits; the verdicts must not change).
"""
import ctypes
import hashlib
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

L = 2**252 + 27742317777372353535851937790883648493
LAT_SO = os.path.join(ROOT, "tests", "cpp", "build", "liblattice_host.so")


def _lattice_lib():
    if not os.path.exists(LAT_SO):
        os.makedirs(os.path.dirname(LAT_SO), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "narwhal_amd", "csrc"),
                        "-o", LAT_SO, os.path.join(ROOT, "tests", "cpp", "lattice_host.cpp")], check=True)
    return ctypes.CDLL(LAT_SO)


def _bits_of(lat, k: int) -> int:
    kw = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
    c, d = (ctypes.c_uint32 * 5)(), (ctypes.c_uint32 * 5)()
    cn, ok = ctypes.c_int(), ctypes.c_int()
    lat.lat_reduce(kw, c, d, ctypes.byref(cn), ctypes.byref(ok))
    if not ok.value:
        return 999
    cv = sum(c[i] << (32 * i) for i in range(5))
    dv = sum(d[i] << (32 * i) for i in range(5))
    return max(cv.bit_length(), dv.bit_length())


def test_wide_windows_strict(oracle):
    import torch
    from narwhal_amd import device
    assert torch.cuda.is_available()
    lat = _lattice_lib()
    n = 1 << 17
    msgs = device.derive32(b"wide-msg", 0, n)
    pks, sigs = device.keygen_sign(device.derive32(b"wide-seed", 0, n), msgs)
    m, p, s = (t.cpu().numpy() for t in (msgs, pks, sigs))
    bits = np.empty(n, dtype=np.int32)
    for i in range(n):
        k = int.from_bytes(hashlib.sha512(s[i, :32].tobytes() + p[i].tobytes() + m[i].tobytes()).digest(), "little") % L
        bits[i] = _bits_of(lat, k)
    wide = np.nonzero(bits >= 132)[0]
    normal = np.nonzero(bits <= 128)[0]
    assert len(wide) >= 64 and bits[wide].max() >= 133, (len(wide), int(bits.max()))
    rng = np.random.default_rng(7)
    rows = []
    for j, w in enumerate(wide):
        fill = rng.choice(normal, 63, replace=False)
        wave = np.insert(fill, rng.integers(0, 64), w)
        rows.append(wave)
    idx = np.concatenate(rows)
    mm, pp, ss = m[idx].copy(), p[idx].copy(), s[idx].copy()
    bad = rng.random(len(idx)) < 0.25
    kind = rng.integers(0, 3, len(idx))
    for i in np.nonzero(bad)[0]:
        if kind[i] == 0:
            ss[i, 32 + rng.integers(0, 31)] ^= 1 << rng.integers(0, 8)   # s (stays < 2^253)
        elif kind[i] == 1:
            mm[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)        # message: another k
        else:
            ss[i, rng.integers(0, 32)] ^= 1 << rng.integers(0, 8)        # R
    words = device.verify(torch.from_numpy(mm).cuda(), torch.from_numpy(pp).cuda(), torch.from_numpy(ss).cuda(),
                          strict=True)
    torch.cuda.synchronize()
    got = device.unpack_bits(words, len(idx))
    exp = oracle.strict_many(mm, pp, ss)
    assert (got == exp).all(), np.nonzero(got != exp)[0][:10]
    # the untouched wide triples are valid signatures and must verify
    pos = np.arange(len(idx))[np.isin(idx, wide) & ~bad]
    assert got[pos].all()


@pytest.mark.parametrize("W", [34, 35, 36, 37])
def test_forced_windows(oracle, W):
    import torch
    from narwhal_amd import device
    n = 4096
    msgs = device.derive32(b"forcew-msg", W, n)
    pks, sigs = device.keygen_sign(device.derive32(b"forcew-seed", W, n), msgs)
    m, p, s = (t.cpu().numpy().copy() for t in (msgs, pks, sigs))
    rng = np.random.default_rng(W)
    for i in np.nonzero(rng.random(n) < 0.25)[0]:
        col = rng.integers(0, 64)
        s[i, col] ^= 1 << rng.integers(0, 8 if col < 63 else 4)
    from narwhal_amd import _lib
    _lib.diag_set("force_windows", W)
    try:
        got = {}
        for strict in (True, False):
            words = device.verify(torch.from_numpy(m).cuda(), torch.from_numpy(p).cuda(), torch.from_numpy(s).cuda(),
                                  strict=strict)
            torch.cuda.synchronize()
            got[strict] = device.unpack_bits(words, n)
    finally:
        _lib.diag_set("force_windows", 0)
    assert (got[True] == oracle.strict_many(m, p, s)).all()
    assert (got[False] == oracle.leaf_many(m, p, s)).all()
    assert 0.6 * n < got[True].sum() < 0.9 * n
