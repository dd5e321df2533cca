"""Launch keys (narwhal_amd/csrc/launch_keys.h): a large batch-leaf launch without a committee
cache detects the keys it repeats, builds their flags and combs once, and runs the committee comb
kernel over them.  The verdicts must be exactly the per-vote leaves' (crypto/src/lib.rs:206-219 as
restated by the oracle) whichever kernel decides a vote: on the first launch (keys join, combs
built), on the next (steady state), with the set full, with the feature off, and for keys with
odd flags -- undecodable, small-order, torsion-bearing -- repeated often enough to join.
"""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _held(lib):
    h, cap = ctypes.c_uint32(), ctypes.c_uint32()
    from narwhal_amd import _lib
    _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), ctypes.byref(cap)))
    return h.value, cap.value


def _leaf(msgs, pks, sigs):
    from narwhal_amd import device
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    words = device.verify(t(msgs), t(pks), t(sigs), strict=False)
    torch.cuda.synchronize()
    return device.unpack_bits(words, len(msgs))


def _committee_workload(oracle, rng, nkeys, n, bad_rate=0.01, outsider_rate=0.02):
    """n votes by a committee of nkeys members (and a few one-off outsiders), bad_rate of them
    signed over another message."""
    seeds = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    who = rng.integers(0, nkeys, n)
    s = seeds[who].copy()
    out = rng.random(n) < outsider_rate
    s[out] = rng.integers(0, 256, (int(out.sum()), 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    signed = msgs.copy()
    bad = rng.random(n) < bad_rate
    signed[bad, 0] ^= 1
    pks, sigs = oracle.keygen_sign_many(s, signed)
    return msgs, pks, sigs


def test_committee_votes_vs_oracle(oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))   # empties the launch keys too
    rng = np.random.default_rng(71)
    n = 100_000
    msgs, pks, sigs = _committee_workload(oracle, rng, 100, n)
    exp = oracle.leaf_many(msgs, pks, sigs)
    assert 0.9 * n < exp.sum() < 0.995 * n
    assert _held(lib)[0] == 0
    first = _leaf(msgs, pks, sigs)               # keys join, combs built, then the comb kernel
    held, cap = _held(lib)
    assert held == 100 and cap >= 100, held       # the committee, not the one-off outsiders
    again = _leaf(msgs, pks, sigs)               # steady state: census only
    assert _held(lib)[0] == 100
    _lib.diag_set("launch_keys", 0)
    try:
        off = _leaf(msgs, pks, sigs)             # per-vote ladder for every vote
    finally:
        _lib.diag_set("launch_keys", 1)
    for got in (first, again, off):
        assert (got == exp).all(), np.nonzero(got != exp)[0][:10]


def test_set_fills_and_other_committees_take_the_ladder(oracle):
    """A second committee after the set is full: its votes are decided by the list-mode ladder,
    the first committee's by the comb kernel, in one launch; nwc_set_committee empties the set."""
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    rng = np.random.default_rng(72)
    m1 = _committee_workload(oracle, rng, 120, 80_000)
    _leaf(*m1)
    assert _held(lib)[0] == 120
    m2 = _committee_workload(oracle, rng, 40, 80_000)     # 8 fit (capacity 128), 32 do not
    both = tuple(np.concatenate([a, b]) for a, b in zip(m1, m2))
    perm = rng.permutation(len(both[0]))
    both = tuple(a[perm] for a in both)
    exp = oracle.leaf_many(*both)
    got = _leaf(*both)
    # the combs have room for the 120 held keys: this launch records the demand (128) ...
    assert _held(lib)[0] == 120
    got2 = _leaf(*both)
    # ... and the next one grows them first: 8 more join, the set is full
    assert _held(lib)[0] == 128
    for g in (got, got2):
        assert (g == exp).all(), np.nonzero(g != exp)[0][:10]
    _lib.check(lib.nwc_set_committee(None, 0))
    assert _held(lib)[0] == 0


def test_new_committee_replaces_the_set(oracle):
    """Two disjoint 100-key committees in turn (an epoch change): the second one's launch finds
    the held keys covering none of its repeated-key sample and no room for its own, so the set is
    emptied and the second committee's keys join; then the first committee comes back and takes
    the set again.  Verdicts equal the oracle's leaves throughout."""
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    rng = np.random.default_rng(74)
    c1 = _committee_workload(oracle, rng, 100, 80_000)
    c2 = _committee_workload(oracle, rng, 100, 80_000)
    keys1 = {bytes(k) for k in c1[1]}
    for work, name in ((c1, "first"), (c2, "second"), (c1, "first again")):
        exp = oracle.leaf_many(*work)
        got = _leaf(*work)
        held, cap = _held(lib)
        assert held == 100, (name, held)
        assert (got == exp).all(), (name, np.nonzero(got != exp)[0][:10])
        again = _leaf(*work)                      # steady state over the replaced set
        assert (again == exp).all() and _held(lib)[0] == 100, name
    assert len(keys1 & {bytes(k) for k in c2[1]}) == 0
    _lib.check(lib.nwc_set_committee(None, 0))


def test_golden_keys_repeated_join_with_their_flags(golden_verify, oracle):
    """Every golden strict/leaf case (undecodable keys, small-order keys, keys with an 8-torsion
    component, non-canonical encodings, s >= l, ...) tiled 600 times: their keys are frequent, so
    they join the set with the flags k_lk_keys computes, and each copy's verdict must still be the
    fixture's batch-leaf verdict."""
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    reps = 600
    idx = np.tile(np.arange(len(cases)), reps)
    np.random.default_rng(73).shuffle(idx)
    m = np.stack([np.frombuffer(bytes.fromhex(cases[i]["msg"]), np.uint8) for i in range(len(cases))])[idx]
    p = np.stack([np.frombuffer(bytes.fromhex(cases[i]["pk"]), np.uint8) for i in range(len(cases))])[idx]
    s = np.stack([np.frombuffer(bytes.fromhex(cases[i]["sig"]), np.uint8) for i in range(len(cases))])[idx]
    exp = np.array([bool(cases[i]["leaf"]) for i in idx])
    got = _leaf(m, p, s)
    held = _held(lib)[0]
    assert held >= min(len({c["pk"] for c in cases}), 128) - 2, held
    assert (got == exp).all(), [cases[idx[i]]["name"] for i in np.nonzero(got != exp)[0][:10]]
    again = _leaf(m, p, s)
    assert (again == exp).all()
    _lib.check(lib.nwc_set_committee(None, 0))
