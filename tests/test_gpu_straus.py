"""dalek's batch equation over sub-batches of votes on the GPU (k_verify_straus,
nwc_dev_verify_batch_straus), leaves for the sub-batches it rejects: certificate verdicts and exact
bad-vote sets against the golden batch fixtures and the oracle (crypto/src/lib.rs:206-219).

On the deterministic domain the outcome must be exact every run.  On dalek's randomized domain
(fixture class "randomized": pure-torsion residuals, torsion-bearing keys) this path IS dalek's
algorithm, so a certificate passes with probability ~1/ord and fails otherwise -- checked over
repeated runs (fresh z_i each launch) as neither always-Ok nor always-Err; when it fails, its bad
set is a non-empty part of the leaves' (the fixture's): a randomized vote whose sub-batch passed
is not in it."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests.conftest import GOLDEN, ROOT

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
    leaf = device.verify_batch_straus(dd, do, dm, dp[:nv], ds[:nv])
    cert, bad = device.cert_reduce(leaf, do, nv)
    torch.cuda.synchronize()
    return device.unpack_bits(cert, m), device.unpack_bits(bad, nv)


def _golden_arrays(batches):
    offs = np.zeros(len(batches) + 1, np.int64)
    offs[1:] = np.cumsum([len(b["votes"]) for b in batches])
    dig = np.stack([np.frombuffer(bytes.fromhex(b["msg"]), np.uint8) for b in batches])
    pks = np.frombuffer(b"".join(bytes.fromhex(p) for b in batches for p, _ in b["votes"]), np.uint8)
    sigs = np.frombuffer(b"".join(bytes.fromhex(s) for b in batches for _, s in b["votes"]), np.uint8)
    return dig, offs, pks, sigs


def test_golden_batches_straus(golden_batch):
    batches = [b for b in golden_batch if len(bytes.fromhex(b["msg"])) == 32]
    dig, offs, pks, sigs = _golden_arrays(batches)
    runs = 40
    passes = np.zeros(len(batches), int)
    for _ in range(runs):
        cert, bad = _run(dig, offs, pks, sigs)
        for c, b in enumerate(batches):
            mine = sorted(int(v - offs[c]) for v in np.nonzero(bad[offs[c]:offs[c + 1]])[0] + offs[c])
            if b["class"] == "randomized":
                passes[c] += int(cert[c])
                if cert[c]:
                    assert mine == [], b["name"]
                else:
                    assert mine and set(mine) <= set(b["bad"]), b["name"]
            else:
                assert bool(cert[c]) == bool(b["verdict"]), b["name"]
                assert mine == sorted(b["bad"]), b["name"]
    for c, b in enumerate(batches):
        if b["class"] == "randomized":
            assert passes[c] < runs, (b["name"], passes[c])   # dalek's Err outcome occurs
    assert passes[[c for c, b in enumerate(batches) if b["class"] == "randomized"]].sum() > 0   # and its Ok outcome


@pytest.mark.parametrize("big", [383, 1600])
def test_certificates_vs_oracle(oracle, big):
    """Honest and 1 %-bad certificates of many sizes (empty, single-vote, and 383 / 1,600 votes: the
    sub-batches cut across certificate boundaries everywhere).  Verdicts and bad sets equal the
    oracle's, at the default sub-batch size and at 1 and 16 votes per sub-batch (nwc_diag_set)."""
    rng = np.random.default_rng(41)
    sizes = [0, 1, 2, 3, 24, 25, 48, 49, 67, 67, 67, 100, 200, big] + [int(x) for x in rng.integers(1, 90, 120)]
    m = len(sizes)
    offs = np.zeros(m + 1, np.int64)
    offs[1:] = np.cumsum(sizes)
    nv = int(offs[-1])
    nkeys = 150
    kseeds = rng.integers(0, 256, (nkeys, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    who = rng.integers(0, nkeys, nv)
    vm = np.repeat(dig, sizes, axis=0)
    pks, sigs = oracle.keygen_sign_many(kseeds[who], vm)
    bad = rng.random(nv) < 0.01
    sigs[bad, 33] ^= 1
    ocert, obad = oracle.batch_many(dig, offs.astype(np.uint32), pks, sigs)
    from narwhal_amd import _lib
    for nq in (12, 1, 16):   # the default first
        _lib.diag_set("straus_nq", nq)
        try:
            cert, gbad = _run(dig, offs, pks, sigs)
        finally:
            _lib.diag_set("straus_nq", 12)
        assert (cert == ocert).all(), (nq, np.nonzero(cert != ocert))
        assert (gbad == obad).all(), nq
    assert ocert.sum() > m // 3 and (~ocert).sum() > 3


def test_without_basepoint_comb_takes_the_leaves():
    """NWC_COMB16=0 (no radix-2^22 basepoint comb for the -S B term): the entry runs the exact leaves
    instead; the oracle certificates must still match (a process of its own: the switch is read once)."""
    r = subprocess.run([sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_gpu_straus.py") + "::test_certificates_vs_oracle[383]"],
                       env=dict(os.environ, NWC_COMB16="0"), cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_host_entry_vs_oracle(oracle):
    """nwc_verify_batch_straus_many (host buffers, the Rust shim's `verify_batch_many(.., true)`):
    certificate verdicts and bad sets equal the oracle's and nwc_verify_batch_many's."""
    import ctypes
    from narwhal_amd import _lib
    lib = _lib.load()
    rng = np.random.default_rng(43)
    sizes = [0, 1, 3, 67, 67, 12, 13, 24, 100] + [int(x) for x in rng.integers(1, 90, 150)]
    m = len(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    nv = int(offs[-1])
    kseeds = rng.integers(0, 256, (120, 32), dtype=np.uint8)
    dig = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(kseeds[rng.integers(0, 120, nv)], np.repeat(dig, sizes, axis=0))
    bad = rng.random(nv) < 0.02
    sigs[bad, 50] ^= 8
    ocert, obad = oracle.batch_many(dig, offs, pks, sigs)
    out = {}
    for name in ("nwc_verify_batch_many", "nwc_verify_batch_straus_many"):
        cert = ctypes.create_string_buffer((m + 7) // 8)
        badb = ctypes.create_string_buffer((nv + 7) // 8)
        _lib.check(getattr(lib, name)(_lib.buf(dig), _lib.buf(offs), _lib.buf(pks), _lib.buf(sigs), m, cert, badb))
        out[name] = (np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:m].astype(bool),
                     np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:nv].astype(bool))
    for name, (c, b) in out.items():
        assert (c == ocert).all(), name
        assert (b == obad).all(), name
    assert ocert.sum() > 20 and (~ocert).sum() > 20
