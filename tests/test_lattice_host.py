"""CPU tests of the half-size scalar reduction (narwhal_amd/csrc/lattice.h, host build).

Property checked for every k: ok -> d odd, 0 < d < 2^146, |c| < 2^146 and d*k = c (mod 8l);
the kernels rely on exactly this.  Failure (ok == 0) is allowed only rarely;
such lanes are re-verified by the full-length ladder.
"""
import ctypes
import os
import random
import subprocess

import pytest

from tests.conftest import ROOT

L = 2**252 + 27742317777372353535851937790883648493
N = 8 * L
SO = os.path.join(ROOT, "tests", "cpp", "build", "liblattice_host.so")


@pytest.fixture(scope="module")
def lat():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-I" + os.path.join(ROOT, "narwhal_amd", "csrc"),
                    "-o", SO, os.path.join(ROOT, "tests", "cpp", "lattice_host.cpp")], check=True)
    lib = ctypes.CDLL(SO)
    return lib


def run(lib, k, fn="lat_reduce"):
    kw = (ctypes.c_uint32 * 8)(*[(k >> (32 * i)) & 0xFFFFFFFF for i in range(8)])
    c = (ctypes.c_uint32 * 5)()
    d = (ctypes.c_uint32 * 5)()
    cn, ok = ctypes.c_int(), ctypes.c_int()
    getattr(lib, fn)(kw, c, d, ctypes.byref(cn), ctypes.byref(ok))
    cv = sum(c[i] << (32 * i) for i in range(5))
    dv = sum(d[i] << (32 * i) for i in range(5))
    return (-cv if cn.value else cv), dv, bool(ok.value)


def check(k, c, d, ok):
    if not ok:
        return False
    assert d % 2 == 1 and 0 < d < 2**146, (k, d)
    assert abs(c) < 2**146
    assert (d * k - c) % N == 0, k
    return True


def test_random_k(lat):
    rng = random.Random(5)
    fails = 0
    for _ in range(20000):
        k = rng.randrange(L)
        c, d, ok = run(lat, k)
        fails += not check(k, c, d, ok)
    assert fails == 0, fails


def test_edge_k(lat):
    cases = [0, 1, 2, 3, 5, 2**64, 2**126, 2**127 - 1, 2**127, 2**127 + 1, 2**200, L - 1, L - 2, L // 2, L // 3,
             L // 7, 4 * L // 9, (N - 1) // 2 % L, 2**252, 2**252 + 12345]
    for k in cases:
        k %= L
        c, d, ok = run(lat, k)
        if ok:
            check(k, c, d, ok)
        # small k: (k, 1) is already short
        if k < 2**127:
            assert ok and d == 1 and c == k


def test_adversarial_structure(lat):
    """k close to rationals with small denominators force large partial quotients / short
    even vectors: results must still be correct when ok."""
    rng = random.Random(9)
    for _ in range(3000):
        num = rng.randrange(1, 2**20)
        den = rng.randrange(1, 2**20)
        k = (N * num // den + rng.randrange(-2**40, 2**40)) % L
        c, d, ok = run(lat, k)
        if ok:
            check(k, c, d, ok)


def test_lehmer_equals_single_steps(lat):
    """The Lehmer blocks certify every quotient and never step past the first r1 < 2^127, so
    the kernels' reduction returns exactly what one-step-at-a-time Euclid returns."""
    rng = random.Random(11)
    ks = [rng.randrange(L) for _ in range(20000)]
    ks += [(N * rng.randrange(1, 2**20) // rng.randrange(1, 2**20) + rng.randrange(-2**40, 2**40)) % L
           for _ in range(3000)]
    ks += [0, 1, 2**127 - 1, 2**127, 2**127 + 1, L - 1, L // 2, L // 3, 2**252]
    for k in ks:
        a, b = run(lat, k), run(lat, k, "lat_reduce_single")
        assert a[2] == b[2], k
        if a[2]:   # failed lanes (e.g. k = 2^252) go to the full-length ladder either way
            assert a == b, k
