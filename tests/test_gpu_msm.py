"""dalek's batch equation as a Pippenger MSM per group of votes on the GPU (k_verify_msm,
nwc_dev_verify_batch_msm / nwc_verify_batch_msm_many, narwhal_amd/csrc/msm.h), the exact leaves for
the groups it rejects: certificate verdicts and bad-vote sets against the golden batch fixtures
and the oracle (crypto/src/lib.rs:206-219).

As for the Straus entry: exact on the deterministic domain every run; on dalek's randomized
domain a group passes with probability ~1/ord (checked over repeated runs as neither always-Ok nor
always-Err).  Because a group is decided as a whole, the tests also read nwc_msm_stats to prove
that the equation -- not only the leaf fallback -- decided the clean groups."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(digests, offs, pks, sigs):
    from narwhal_amd import device
    m = len(offs) - 1
    nv = int(offs[-1])
    mi = np.repeat(np.arange(m, dtype=np.int32), np.diff(offs))
    t = lambda a, dt=torch.uint8: torch.from_numpy(np.ascontiguousarray(a)).to(dt).cuda()  # noqa: E731
    dd, do, dm = t(digests), t(offs.astype(np.int32), torch.int32), t(mi, torch.int32)
    dp = t(pks.reshape(max(nv, 1), 32) if nv else np.zeros((1, 32), np.uint8))
    ds = t(sigs.reshape(max(nv, 1), 64) if nv else np.zeros((1, 64), np.uint8))
    leaf = device.verify_batch_msm(dd, do, dm, dp[:nv], ds[:nv])
    cert, bad = device.cert_reduce(leaf, do, nv)
    torch.cuda.synchronize()
    return device.unpack_bits(cert, m), device.unpack_bits(bad, nv)


def _stats():
    from narwhal_amd import device
    return device.msm_stats()[:3]


@pytest.fixture(autouse=True)
def _every_group():
    """The exact group counts below need the equation on every group: the skip policy off (a
    test of its own turns it on)."""
    from narwhal_amd import _lib
    _lib.diag_set("msm_adapt", 0)
    yield
    _lib.diag_set("msm_adapt", 1)


def _committee_certs(oracle, rng, m, q=67, nkeys=100, bad_rate=0.0):
    kseeds = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    who = np.concatenate([rng.permutation(nkeys)[:q] for _ in range(m)])
    pks, sigs = oracle.keygen_sign_many(kseeds[who], np.repeat(dig, q, axis=0))
    bad = rng.random(m * q) < bad_rate
    sigs[bad, 33] ^= 1
    offs = (np.arange(m + 1) * q).astype(np.int64)
    return dig, offs, pks, sigs, bad


def test_golden_batches_msm(golden_batch):
    """Every golden batch as a call of its own (a group of its own), 30 times: the deterministic
    fixtures exactly, the randomized ones both ways."""
    batches = [b for b in golden_batch if len(bytes.fromhex(b["msg"])) == 32 and b["votes"]]
    runs = 30
    passes = {}
    for b in batches:
        dig = np.frombuffer(bytes.fromhex(b["msg"]), np.uint8)[None, :]
        offs = np.array([0, len(b["votes"])], np.int64)
        pks = np.frombuffer(b"".join(bytes.fromhex(p) for p, _ in b["votes"]), np.uint8)
        sigs = np.frombuffer(b"".join(bytes.fromhex(s) for _, s in b["votes"]), np.uint8)
        n = 0
        for _ in range(runs if b["class"] == "randomized" else 2):
            cert, bad = _run(dig, offs, pks, sigs)
            mine = sorted(int(v) for v in np.nonzero(bad)[0])
            if b["class"] == "randomized":
                n += int(cert[0])
                if cert[0]:
                    assert mine == [], b["name"]
                else:
                    assert mine and set(mine) <= set(b["bad"]), b["name"]
            else:
                assert bool(cert[0]) == bool(b["verdict"]), b["name"]
                assert mine == sorted(b["bad"]), b["name"]
        if b["class"] == "randomized":
            passes[b["name"]] = n
            assert n < runs, (b["name"], n)   # dalek's Err outcome occurs
    assert sum(passes.values()) > 0, passes   # and its Ok outcome


@pytest.mark.parametrize("group", [2048, 64, 4096])
def test_clean_committee_groups_pass_by_the_equation(oracle, group):
    """Config 3's clean variant in miniature: 300 certificates x 67 votes of a 100-key committee,
    every vote valid.  Every group must pass by the MSM equation itself (nwc_msm_stats: no group
    failed), and one corrupted vote then fails exactly its own group: verdicts and the bad set equal
    the oracle's."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(group)
    dig, offs, pks, sigs, _ = _committee_certs(oracle, rng, 300)
    nv = int(offs[-1])
    _lib.diag_set("msm_group", group)
    try:
        p0, f0, o0 = _stats()
        cert, bad = _run(dig, offs, pks, sigs)
        p1, f1, o1 = _stats()
        assert cert.all() and not bad.any()
        groups = (nv + group - 1) // group
        assert (p1 - p0, f1 - f0, o1 - o0) == (groups, 0, 0), (p1 - p0, f1 - f0, o1 - o0)
        v = int(rng.integers(0, nv))
        sigs2 = sigs.copy()
        sigs2[v, 40] ^= 4
        ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs2)
        cert, bad = _run(dig, offs, pks, sigs2)
        p2, f2, _ = _stats()
        assert (cert == ocert).all() and (bad == obad).all() and obad.sum() == 1 and bad[v]
        assert (p2 - p1, f2 - f1) == (groups - 1, 1), (p2 - p1, f2 - f1)
    finally:
        _lib.diag_set("msm_group", 0)


@pytest.mark.parametrize("group", [2048, 256])
def test_certificates_vs_oracle(oracle, group):
    """Honest and 1 %-bad certificates of many sizes (empty, single-vote, 383 and 1,600 votes) over
    150 keys: groups cut across certificates everywhere; verdicts and bad sets equal the oracle's."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(51)
    sizes = [0, 1, 2, 3, 24, 25, 48, 49, 67, 67, 67, 100, 200, 383, 1600] + [int(x) for x in rng.integers(1, 90, 150)]
    m = len(sizes)
    offs = np.zeros(m + 1, np.int64)
    offs[1:] = np.cumsum(sizes)
    nv = int(offs[-1])
    kseeds = rng.integers(0, 256, (150, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(kseeds[rng.integers(0, 150, nv)], np.repeat(dig, sizes, axis=0))
    bad = rng.random(nv) < 0.01
    sigs[bad, 33] ^= 1
    ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs)
    _lib.diag_set("msm_group", group)
    try:
        cert, gbad = _run(dig, offs, pks, sigs)
    finally:
        _lib.diag_set("msm_group", 0)
    assert (cert == ocert).all(), np.nonzero(cert != ocert)
    assert (gbad == obad).all()
    assert ocert.sum() > m // 3 and (~ocert).sum() > 3


def test_first_sight_keys_overflow_to_the_leaves(oracle):
    """Votes of distinct keys (first-sight: no repetition to aggregate): a group holds more keys
    than the LDS table (126) at 2,048 votes a group, so it is decided by the leaves -- verdicts still exact, and
    nwc_msm_stats counts the overflow."""
    rng = np.random.default_rng(53)
    m, q = 40, 67
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    seeds = rng.integers(0, 256, (m * q, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, np.repeat(dig, q, axis=0))
    sigs[[5, 700], 20] ^= 1
    offs = (np.arange(m + 1) * q).astype(np.int64)
    ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs)
    from narwhal_amd import _lib
    _lib.diag_set("msm_group", 2048)   # the automatic size would cut this small call into 64-vote groups
    try:
        _, f0, o0 = _stats()
        cert, bad = _run(dig, offs, pks, sigs)
        _, f1, o1 = _stats()
    finally:
        _lib.diag_set("msm_group", 0)
    assert (cert == ocert).all() and (bad == obad).all()
    assert o1 > o0 and f1 > f0


def test_host_entry_vs_oracle(oracle):
    """nwc_verify_batch_msm_many (host buffers): certificate verdicts and bad sets equal the
    oracle's, on a 1 %-bad mix and on clean committee traffic."""
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(57)
    for bad_rate in (0.01, 0.0):
        dig, offs, pks, sigs, _ = _committee_certs(oracle, rng, 150, bad_rate=bad_rate)
        m, nv = len(dig), int(offs[-1])
        offs32 = offs.astype(np.uint32)
        ocert, obad = oracle.batch_many(dig, offs32, pks, sigs)
        cert = ctypes.create_string_buffer((m + 7) // 8)
        badb = ctypes.create_string_buffer((nv + 7) // 8)
        _lib.check(lib.nwc_verify_batch_msm_many(_lib.buf(dig), _lib.buf(offs32), _lib.buf(pks), _lib.buf(sigs), m,
                                                 cert, badb))
        c = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:m].astype(bool)
        b = np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:nv].astype(bool)
        assert (c == ocert).all() and (b == obad).all(), bad_rate


def test_skip_policy_on_a_high_bad_rate(oracle):
    """A 2 %-bad mix (every group holds bad votes): after the first launch fails its groups, the
    next 7 skip the equation and pass every vote straight to the Straus sub-batches (nwc_msm_stats:
    skipped groups), the 8th runs it on every group again; verdicts stay the oracle's throughout,
    and on clean traffic the equation runs on every group from the next re-measuring launch on."""
    from narwhal_amd import _lib, device
    _lib.diag_set("msm_adapt", 1)
    _lib.diag_set("msm_group", 512)
    try:
        rng = np.random.default_rng(59)
        dig, offs, pks, sigs, _ = _committee_certs(oracle, rng, 400, bad_rate=0.02)
        ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs)
        groups = (int(offs[-1]) + 511) // 512
        per_call = []
        for _ in range(9):
            s0 = device.msm_stats()
            cert, bad = _run(dig, offs, pks, sigs)
            s1 = device.msm_stats()
            assert (cert == ocert).all() and (bad == obad).all()
            per_call.append((s1[1] - s0[1], s1[3] - s0[3]))   # (failed, skipped)
        assert per_call == [(groups, 0)] + [(0, groups)] * 7 + [(groups, 0)], per_call
        cdig, coffs, cpks, csigs, _ = _committee_certs(oracle, rng, 400)
        per_call = []
        for _ in range(9):
            s0 = device.msm_stats()
            cert, bad = _run(cdig, coffs, cpks, csigs)
            s1 = device.msm_stats()
            assert cert.all() and not bad.any()
            per_call.append((s1[0] - s0[0], s1[3] - s0[3]))   # (passed, skipped)
        assert per_call == [(0, groups)] * 7 + [(groups, 0)] * 2, per_call
    finally:
        _lib.diag_set("msm_group", 0)


def test_launches_above_the_cap_run_in_pieces():
    """NWC_VERIFY_MAX_LAUNCH (read once per process: a child) set to 65,536 votes: a 201k-vote call
    of the MSM and Straus entries runs as four consecutive launches, each with its own groups or
    sub-batches, fallback lists and leaf words; verdicts equal the construction (1 % of the votes
    signed over another digest)."""
    import os
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = r'''
import sys; sys.path.insert(0, %r)
import numpy as np, torch
from narwhal_amd import device
M, Q = 3000, 67
nv = M * Q
cdig = device.derive32(b"cap-cert", 0, M)
seeds = device.derive32(b"cap-seed", 0, 100)
g = torch.Generator(device="cuda"); g.manual_seed(7)
who = torch.randint(0, 100, (nv,), device="cuda", generator=g)
bad = torch.rand(nv, device="cuda", generator=g) < 0.01
mi = torch.arange(M, device="cuda", dtype=torch.int32).repeat_interleave(Q)
signed = cdig[mi.long()].clone(); signed[bad, 3] ^= 1
pks, sigs = device.keygen_sign(seeds[who], signed)
offs = torch.arange(M + 1, device="cuda", dtype=torch.int32) * Q
want_bad = bad.cpu().numpy(); want_cert = ~want_bad.reshape(M, Q).any(axis=1)
for f in (device.verify_batch_msm, device.verify_batch_straus):
    cw, bw = device.cert_reduce(f(cdig, offs, mi, pks, sigs), offs, nv)
    torch.cuda.synchronize()
    assert (device.unpack_bits(bw, nv) == want_bad).all(), f.__name__
    assert (device.unpack_bits(cw, M) == want_cert).all(), f.__name__
print("done", flush=True)
''' % ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=ROOT,
                       env=dict(os.environ, NWC_VERIFY_MAX_LAUNCH="65536"))
    assert r.returncode == 0 and "done" in r.stdout, (r.returncode, r.stdout[-500:], r.stderr[-3000:])


@pytest.mark.parametrize("nkeys", [126, 127])
def test_key_table_capacity_boundary(oracle, nkeys):
    """One group of 2,048 clean votes over exactly nkeys distinct keys: 126 (MSM_KMAX) fit the LDS
    key table and the group passes by the equation; 127 overflow it, and the group is decided by
    the fallback -- verdicts exact either way (nwc_msm_stats tells which)."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(61 + nkeys)
    n = 2048
    kseeds = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    who = np.concatenate([np.arange(nkeys), rng.integers(0, nkeys, n - nkeys)])
    m = 64
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    offs = (np.arange(m + 1) * (n // m)).astype(np.int64)
    pks, sigs = oracle.keygen_sign_many(kseeds[who], np.repeat(dig, n // m, axis=0))
    _lib.diag_set("msm_group", 2048)
    try:
        s0 = _stats()
        cert, bad = _run(dig, offs, pks, sigs)
        s1 = _stats()
    finally:
        _lib.diag_set("msm_group", 0)
    assert cert.all() and not bad.any()
    if nkeys <= 126:
        assert (s1[0] - s0[0], s1[1] - s0[1], s1[2] - s0[2]) == (1, 0, 0), (s0, s1)
    else:
        assert (s1[0] - s0[0], s1[1] - s0[1], s1[2] - s0[2]) == (0, 1, 1), (s0, s1)


def test_skip_policy_is_device_wide_and_verdicts_hold(oracle):
    """The skip policy's state is per device (include/nwc.h): one caller's high-bad-rate launch on
    its stream makes the next launch of another caller, on another stream with clean traffic, skip
    the equation (its groups go straight to the leaves) -- slower for it, with the same verdicts."""
    import torch
    from narwhal_amd import _lib, device
    _lib.diag_set("msm_adapt", 1)
    _lib.diag_set("msm_group", 512)
    try:
        rng = np.random.default_rng(63)
        bdig, boffs, bpks, bsigs, _ = _committee_certs(oracle, rng, 200, bad_rate=0.03)
        cdig, coffs, cpks, csigs, _ = _committee_certs(oracle, rng, 200)
        ocert, obad = oracle.batch_many(bdig, boffs.astype(np.uint32), bpks, bsigs)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        # the bad caller measures (the policy's re-measuring launch), fails its groups and arms the skip
        for _ in range(8):
            s0 = device.msm_stats()
            with torch.cuda.stream(s1):
                cert, bad = _run(bdig, boffs, bpks, bsigs)
            s1.synchronize()
            if device.msm_stats()[1] > s0[1]:
                break
        assert (cert == ocert).all() and (bad == obad).all()
        st0 = device.msm_stats()
        with torch.cuda.stream(s2):
            cert, bad = _run(cdig, coffs, cpks, csigs)
        s2.synchronize()
        st1 = device.msm_stats()
        assert cert.all() and not bad.any()
        groups = (int(coffs[-1]) + 511) // 512
        assert (st1[0] - st0[0], st1[3] - st0[3]) == (0, groups), (st0, st1)
    finally:
        _lib.diag_set("msm_group", 0)
        _lib.diag_set("msm_adapt", 0)
