"""Device memory per process and the digester's failure path (include/nwc.h nwc_memory_info,
nwc_trim, NWC_DIGEST_MAX_BYTES / NWC_DIGEST_KEEP_BYTES, NWC_DIGEST_FAIL_GROUP), and the build id
of the library the GPU runs.

The reference's Processor hashes one batch at a time (worker/src/processor.rs:35-55) and holds
nothing between batches; a primary and a worker may share one GPU, so the library must not keep a
large group's buffer resident, and a group that fails on the device must hand its batches back
(the caller holds them) instead of orphaning them."""
import hashlib
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

BATCH = 508_052   # BASELINE config 4's batch (977 txs of 512 B, bincode)


def _sha32(b) -> bytes:
    return hashlib.sha512(bytes(b)).digest()[:32]


def _digester_with_env(env, max_group, wait_us):
    """A Digester created with `env` set: the digester reads its NWC_DIGEST_* knobs at create."""
    from narwhal_amd.processor import Digester
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Digester(max_group, wait_us)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


def _drain(dg, n, timeout=120):
    got, t0 = [], time.time()
    while len(got) < n and time.time() - t0 < timeout:
        got += dg.poll(4096, 100_000)
    return got


def test_build_id_is_this_trees():
    """The library the GPU loads was compiled from the sources in this tree (a stale prebuilt
    .so would carry another hash)."""
    from narwhal_amd import _lib, build
    lib = _lib.load()
    assert lib.nwc_build_id().decode() == build.source_id()
    print("libnwc build id", build.source_id())


def test_large_group_is_released_and_small_one_fits():
    """A group above NWC_DIGEST_KEEP_BYTES leaves no device buffer behind; a later small group
    keeps only its own; digests equal hashlib throughout."""
    from narwhal_amd import _lib
    rng = np.random.default_rng(11)
    batch = rng.integers(0, 256, BATCH, dtype=np.uint8)
    want = _sha32(batch)
    dg = _digester_with_env({"NWC_DIGEST_KEEP_BYTES": str(256 << 20)}, 100_000, 200_000)
    try:
        n_big = 1200   # 610 MB of batches (the same borrowed buffer, one launch)
        for i in range(n_big):
            dg.submit(batch, i)
        got = _drain(dg, n_big)
        assert len(got) == n_big and all(d == want for _, d in got)
        assert _lib.memory_info()["digesters"] < (1 << 20), _lib.memory_info()
        small = [rng.integers(0, 256, int(k), dtype=np.uint8) for k in rng.integers(1, 50_000, 20)]
        for i, b in enumerate(small):
            dg.submit(b, n_big + i)
        got = _drain(dg, len(small))
        assert [d for _, d in got] == [_sha32(b) for b in small]
        held = _lib.memory_info()["digesters"]
        assert 0 < held < (64 << 20), held
        groups, nb, _ = dg.stats()
        assert nb == n_big + len(small)
    finally:
        dg.close()
    assert _lib.memory_info()["digesters"] == 0


def test_group_bytes_capped_per_launch():
    """NWC_DIGEST_MAX_BYTES cuts a group that would exceed it into several launches (in order)."""
    rng = np.random.default_rng(12)
    batches = [rng.integers(0, 256, BATCH, dtype=np.uint8) for _ in range(8)]
    dg = _digester_with_env({"NWC_DIGEST_MAX_BYTES": str(2 * BATCH + 64)}, 1000, 300_000)
    try:
        for i in range(40):
            dg.submit(batches[i % 8], i)
        got = _drain(dg, 40)
        assert [t for t, _ in got] == list(range(40))
        assert all(d == _sha32(batches[t % 8]) for t, d in got)
        groups, nb, _ = dg.stats()
        assert nb == 40 and groups >= 20, groups   # at most two batches per launch
    finally:
        dg.close()


def test_failed_group_returns_its_tags():
    """NWC_DIGEST_FAIL_GROUP=2: the second launch fails.  Its batches come back as tags with the
    error (DigestGroupError.tags), the groups before and after it as digests, in order; then
    submit refuses new batches and poll keeps reporting the error."""
    from narwhal_amd import _lib
    from narwhal_amd.processor import DigestGroupError
    rng = np.random.default_rng(13)
    batches = [rng.integers(0, 256, 1000 + 100 * i, dtype=np.uint8) for i in range(12)]
    dg = _digester_with_env({"NWC_DIGEST_FAIL_GROUP": "2"}, 4, 2_000_000)
    try:
        for i, b in enumerate(batches):
            dg.submit(b, 100 + i)
        ok, failed, t0 = [], [], time.time()
        while len(ok) + len(failed) < 12 and time.time() - t0 < 60:
            try:
                ok += dg.poll(4096, 100_000)
            except DigestGroupError as e:
                assert e.tags, "an error with no tags before every batch came back"
                failed += e.tags
        assert failed == [104, 105, 106, 107], failed
        assert [t for t, _ in ok] == [100, 101, 102, 103, 108, 109, 110, 111]
        assert all(d == _sha32(batches[t - 100]) for t, d in ok)
        with pytest.raises(_lib.DeviceError):
            dg.submit(batches[0], 999)
        with pytest.raises(DigestGroupError) as ei:
            dg.poll(16, 0)
        assert ei.value.tags == []
        assert not dg._held   # every batch was released back to the caller
    finally:
        with pytest.raises(_lib.DeviceError):
            dg.close()   # destroy reports the sticky error


def _tiled_triples(n: int, base: int = 1 << 14, tag: bytes = b"mem"):
    """n triples tiled from `base` GPU-signed ones, every 7th of the base corrupted (expected
    verdicts known by construction: equation i is valid iff (i mod base) % 7 != 0)."""
    from narwhal_amd import device
    msgs = device.derive32(tag + b"-msg", 0, base)
    pks, sigs = device.keygen_sign(device.derive32(tag + b"-seed", 0, base), msgs)
    sigs[::7, 40] ^= 1
    reps = (n + base - 1) // base
    t = lambda x: x.repeat(reps, 1)[:n].contiguous()  # noqa: E731
    return t(msgs), t(pks), t(sigs)


def test_trim_releases_scratch():
    """nwc_trim frees the on-demand scratch -- table slots, arenas, the per-launch lists and the
    launch-key set -- down to nothing; the next call re-allocates what it needs and verdicts hold."""
    import torch
    from narwhal_amd import _lib, device
    n = 1 << 17
    msgs, pks, sigs = _tiled_triples(n, 1 << 12, b"trim")
    first = device.unpack_bits(device.verify(msgs, pks, sigs, strict=True), n)
    leaf = device.unpack_bits(device.verify(msgs, pks, sigs, strict=False), n)   # launch keys join
    torch.cuda.synchronize()
    before = _lib.memory_info()
    assert before["scratch"] > 0 and before["tables"] > (2 << 30)
    _lib.check(_lib.load().nwc_trim())
    after = _lib.memory_info()
    assert after["scratch"] == 0, after
    assert after["tables"] == before["tables"] and after["auto_cache"] < before["auto_cache"]
    again = device.unpack_bits(device.verify(msgs, pks, sigs, strict=True), n)
    leaf2 = device.unpack_bits(device.verify(msgs, pks, sigs, strict=False), n)
    torch.cuda.synchronize()
    exp = (np.arange(n) % (1 << 12)) % 7 != 0
    assert (first == exp).all() and (again == exp).all() and (leaf == exp).all() and (leaf2 == exp).all()


def test_verify_memory_is_bounded_after_a_huge_launch():
    """A 64M-equation launch runs as launches of at most NWC_VERIFY_MAX_LAUNCH (16M) equations, so
    its lists are a 16M launch's; the next 1M launch shrinks lists above NWC_VERIFY_KEEP_BYTES
    (256 MB) back to its own size.  The per-lane table slots of the static grid (one per lane of
    NWC_VERIFY_GRID_MULT x the resident blocks, ~2.3 GB) do not depend on the launch size: they are
    measured after a 1M launch and the lists bounded above them.  Verdicts equal the construction."""
    import torch
    from narwhal_amd import _lib, device
    lib = _lib.load()
    # no committee cache (an earlier test may have left one): with one, strict launches take the
    # comb kernel, whose per-lane scratch is sized for its own resident grid
    _lib.check(lib.nwc_set_committee(None, 0))
    _lib.check(lib.nwc_trim())
    n = 64 << 20
    msgs, pks, sigs = _tiled_triples(n)
    exp_base = (np.arange(1 << 14) % 7) != 0
    m = 1 << 20
    small = device.unpack_bits(device.verify(msgs[:m], pks[:m], sigs[:m], strict=True), m)
    torch.cuda.synchronize()
    assert (small == np.tile(exp_base, m >> 14)).all()
    base = _lib.memory_info()["scratch"]   # table slots + a 1M launch's lists (~50 MB)
    words = device.verify(msgs, pks, sigs, strict=True)
    torch.cuda.synchronize()
    got = device.unpack_bits(words, n)
    assert (got.reshape(-1, 1 << 14) == exp_base).all()
    big = _lib.memory_info()["scratch"]
    # lists for one 16M launch: 12 B per listed slot (1.5 n + 4096) + 8 B per torsion hash slot
    # (2^26) = 0.84 GB; a single 64M launch's would be 3.3 GB
    assert big - base < (1000 << 20), (base, big)
    del words
    small = device.unpack_bits(device.verify(msgs[:m], pks[:m], sigs[:m], strict=True), m)
    torch.cuda.synchronize()
    assert (small == np.tile(exp_base, m >> 14)).all()
    after = _lib.memory_info()["scratch"]
    assert after < big and after - base < (256 << 20), (base, big, after)
    print("verify scratch: base %.0f MB, after 64M %.0f MB, after 1M again %.0f MB" % (base / 2**20, big / 2**20,
                                                                                  after / 2**20))


def test_stamped_clock_launch():
    """nwc_diag_verify_clock: the stamp build of the strict kernel returns a plausible shader
    clock and the same verdicts as the verdict kernel."""
    import torch
    from narwhal_amd import device
    n = 1 << 18
    msgs, pks, sigs = _tiled_triples(n, 1 << 12, b"clock")
    words = torch.empty(device.words_for(n), dtype=torch.int64, device="cuda")
    ghz, waves = device.verify_clock(msgs, pks, sigs, words)
    assert 0.5 < ghz < 3.0 and waves >= 1000, (ghz, waves)
    exp = (np.arange(n) % (1 << 12)) % 7 != 0
    assert (device.unpack_bits(words, n) == exp).all()
    print("in-kernel clock %.3f GHz over %d waves" % (ghz, waves))


def test_digest_only_process_holds_no_tables():
    """A worker process that only digests (worker/src/worker.rs:182-188: workers and a primary share
    the GPU) holds no verification tables: they are built by the first call that verifies.  A fresh
    process (the tables are per process): digests through the digester and the many-entry, then
    nwc_memory_info shows tables == 0 and no key caches; one verification builds them."""
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = r'''
import sys, hashlib; sys.path.insert(0, %r)
import numpy as np, torch
from narwhal_amd import _lib, crypto
from narwhal_amd.processor import Digester
lib = _lib.load()
assert _lib.memory_info()["tables"] == 0, _lib.memory_info()
rng = np.random.default_rng(5)
msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in rng.integers(0, 600000, 40)]
got = crypto.digest_many(msgs)
assert [g.to_vec() for g in got] == [hashlib.sha512(m).digest()[:32] for m in msgs]
dg = Digester(64, 1000)
for i, m in enumerate(msgs):
    dg.submit(m, i)
out = []
while len(out) < len(msgs):
    out += dg.poll(64, 100000)
assert [d for _, d in sorted(out)] == [hashlib.sha512(m).digest()[:32] for m in msgs]
mem = _lib.memory_info()
dg.close()
assert mem["tables"] == 0 and mem["auto_cache"] == 0 and mem["committee"] == 0, mem
print("digest-only", mem, flush=True)
import json
gold = json.load(open(%r))
c = [c for c in gold["cases"] if c["name"] == "ref-verify_valid_signature"][0]
assert lib.nwc_verify_strict(bytes.fromhex(c["msg"]), bytes.fromhex(c["pk"]), bytes.fromhex(c["sig"])) == 0
mem2 = _lib.memory_info()
assert mem2["tables"] > (2 << 30), mem2
print("after one verify", mem2, flush=True)
''' % (ROOT, os.path.join(ROOT, "tests", "golden", "ed25519_verify.json"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    print(r.stdout)


def test_batch_entry_buffers_above_keep_are_released():
    """The Straus tables (~3.8 GB at config-3 size) and the MSM groups' scratch (~1.3 GB) stay only
    while their entry runs: the next launch of another path frees them (NWC_VERIFY_KEEP_BYTES), so
    scratch returns to the leaf path's own; verdicts equal the construction throughout."""
    import torch
    from narwhal_amd import _lib, device
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    _lib.check(lib.nwc_trim())
    M, Q = 6000, 67
    nv = M * Q
    cdig = device.derive32(b"keep-cert", 0, M)
    seeds = device.derive32(b"keep-seed", 0, 100)
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    who = torch.randint(0, 100, (nv,), device="cuda", generator=g)
    bad = torch.rand(nv, device="cuda", generator=g) < 0.01
    mi = torch.arange(M, device="cuda", dtype=torch.int32).repeat_interleave(Q)
    signed = cdig[mi.long()].clone()
    signed[bad, 3] ^= 1
    pks, sigs = device.keygen_sign(seeds[who], signed)
    offs = torch.arange(M + 1, device="cuda", dtype=torch.int32) * Q
    want = bad.cpu().numpy()

    def leaves():
        return device.verify(cdig, pks, sigs, strict=False, msg_index=mi)

    _lib.diag_set("launch_keys", 0)
    _lib.diag_set("msm_adapt", 0)
    try:
        assert (~device.unpack_bits(leaves(), nv) == want).all()
        torch.cuda.synchronize()
        base = _lib.memory_info()["scratch"]
        for f in (device.verify_batch_straus, device.verify_batch_msm):
            w = f(cdig, offs, mi, pks, sigs)
            torch.cuda.synchronize()
            _, bw = device.cert_reduce(w, offs, nv)
            assert (device.unpack_bits(bw, nv) == want).all(), f.__name__
            held = _lib.memory_info()["scratch"]
            assert held - base > (256 << 20), (f.__name__, base, held)
            assert (~device.unpack_bits(leaves(), nv) == want).all()
            torch.cuda.synchronize()
            after = _lib.memory_info()["scratch"]
            assert after - base < (256 << 20), (f.__name__, base, held, after)
            print("%s: scratch base %.0f MB, with the entry's buffers %.0f MB, after a leaf launch %.0f MB"
                  % (f.__name__, base / 2**20, held / 2**20, after / 2**20))
    finally:
        _lib.diag_set("launch_keys", 1)
        _lib.diag_set("msm_adapt", 1)


def test_launch_key_combs_grow_as_keys_join():
    """Launch-key combs are allocated for the keys that join (20 MB each), not for 128 up front: a
    launch over 40 repeated keys reserves room for 40; a launch that brings 60 more runs them on the
    ladder (room for 40) and records the demand; the next grows the combs and they join.  Verdicts
    equal the construction at every step (launch_keys.h)."""
    import ctypes
    import torch
    from narwhal_amd import _lib, device
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    _lib.check(lib.nwc_trim())
    seeds = device.derive32(b"grow-seed", 0, 100)

    def launch(nkeys, n=1 << 17, tag=0):
        g = torch.Generator(device="cuda")
        g.manual_seed(100 + tag)
        who = torch.randint(0, nkeys, (n,), device="cuda", generator=g)
        msgs = device.derive32(b"grow-msg%d" % tag, 0, n)
        pks, sigs = device.keygen_sign(seeds[who], msgs)
        sigs[::97, 5] ^= 1
        got = device.unpack_bits(device.verify(msgs, pks, sigs, strict=False), n)
        torch.cuda.synchronize()
        exp = np.ones(n, bool)
        exp[::97] = False
        assert (got == exp).all()
        h = ctypes.c_uint32()
        _lib.check(lib.nwc_launch_keys_info(ctypes.byref(h), None))
        return h.value, _lib.memory_info()["auto_cache"]

    comb = 155648 * 128   # KeyComb: 19 windows x 8,192 entries of 128 B
    m0 = _lib.memory_info()["auto_cache"]   # the auto key cache alone (nwc_trim freed the launch keys)
    h1, m1 = launch(40, tag=1)
    h2, m2 = launch(100, tag=2)
    h3, m3 = launch(100, tag=3)
    assert (h1, h2, h3) == (40, 40, 100), (h1, h2, h3)
    assert m2 == m1 and m3 - m1 >= 60 * comb and m3 < m1 + 70 * comb, (m1, m2, m3)
    # (the first launch also builds the tables and the auto cache's first arrays if nothing had yet)
    assert 40 * comb <= m1 - m0 < 40 * comb + (400 << 20) or (m0 == 0 and m1 < 40 * comb + (400 << 20)), (m0, m1)
