"""BASELINE config 3 at its full size in the GPU suite (previously checked only inside bench.py):
100,000 certificates x 67 votes of a 100-node committee (quorum 2N/3 + 1, config/src/lib.rs:181-186),
each vote invalid with p = 0.01 (signed over another digest), built as bench.py's bench_cfg3 builds
them.  Certificate::verify's batch check (primary/src/messages.rs:189-215 -> crypto/src/lib.rs:
206-219) runs through every entry that decides it:

- the uncached per-vote leaves (launch keys off): nwc_dev_verify + nwc_dev_cert_reduce;
- dalek's batch equation over sub-batches (nwc_dev_verify_batch_straus), and as Pippenger MSM
  groups (nwc_dev_verify_batch_msm) through its skip policy's first calls;
- the launch keys (no nwc_set_committee): the first call, where the keys join and their combs are
  built, and the steady state;
- the crate's host entry nwc_verify_batch_many from pageable host buffers.

Each must give a bad-vote bitmap equal to the construction and certificate bits equal to the AND
of each certificate's votes; 2,000 random certificates are also checked against the oracle's
batch_many (the CPU restatement of dalek verify_batch, bisection leaves included)."""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

N, Q, M = 100, 67, 100_000


@pytest.fixture(scope="module")
def cfg3():
    from narwhal_amd import device
    nv = M * Q
    cseeds = device.derive32(b"nw-committee", 0, N)
    cdig = device.derive32(b"nw-cert", 0, M)
    g = torch.Generator(device="cuda")
    g.manual_seed(0x4E57)
    voters = torch.rand((M, N), device="cuda", generator=g).argsort(dim=1)[:, :Q].reshape(-1)
    bad = torch.rand(nv, device="cuda", generator=g) < 0.01
    msg_index = torch.arange(M, device="cuda", dtype=torch.int32).repeat_interleave(Q)
    signed = cdig[msg_index.long()].clone()
    signed[bad, 0] ^= 1
    pks, sigs = device.keygen_sign(cseeds[voters], signed)
    offs = torch.arange(M + 1, device="cuda", dtype=torch.int32) * Q
    torch.cuda.synchronize()
    want_bad = bad.cpu().numpy()
    want_cert = ~want_bad.reshape(M, Q).any(axis=1)
    assert 0.4 < 1 - want_cert.mean() < 0.6   # ~1 - 0.99^67 of certificates fail
    return dict(cdig=cdig, msg_index=msg_index, pks=pks, sigs=sigs, offs=offs, want_bad=want_bad,
                want_cert=want_cert)


def _check(cw, bw, w):
    from narwhal_amd import device
    got_bad = device.unpack_bits(bw, M * Q)
    got_cert = device.unpack_bits(cw, M)
    assert (got_bad == w["want_bad"]).all(), np.nonzero(got_bad != w["want_bad"])[0][:10]
    assert (got_cert == w["want_cert"]).all(), np.nonzero(got_cert != w["want_cert"])[0][:10]


def test_cfg3_device_entries(cfg3):
    from narwhal_amd import _lib, device
    lib = _lib.load()
    w = cfg3
    _lib.check(lib.nwc_set_committee(None, 0))   # no committee cache, launch keys emptied
    try:
        _lib.diag_set("launch_keys", 0)
        leaf = device.verify(w["cdig"], w["pks"], w["sigs"], strict=False, msg_index=w["msg_index"])
        _check(*device.cert_reduce(leaf, w["offs"], M * Q), w)
        straus = device.verify_batch_straus(w["cdig"], w["offs"], w["msg_index"], w["pks"], w["sigs"])
        _check(*device.cert_reduce(straus, w["offs"], M * Q), w)
        # the Pippenger groups: every group holds bad votes at 1 %, so the first call fails them all
        # into the Straus sub-batches and the next ones skip the equation (the policy's cycle)
        for call in range(3):
            s0 = device.msm_stats()
            msm = device.verify_batch_msm(w["cdig"], w["offs"], w["msg_index"], w["pks"], w["sigs"])
            _check(*device.cert_reduce(msm, w["offs"], M * Q), w)
            s1 = device.msm_stats()
            assert s1[0] == s0[0], (call, s0, s1)   # no group passes with a bad vote in it
        _lib.diag_set("launch_keys", 1)
        for call in ("first", "steady"):
            lk = device.verify(w["cdig"], w["pks"], w["sigs"], strict=False, msg_index=w["msg_index"])
            _check(*device.cert_reduce(lk, w["offs"], M * Q), w)
            held = ctypes.c_uint32()
            _lib.check(lib.nwc_launch_keys_info(ctypes.byref(held), None))
            assert held.value == N, (call, held.value)
    finally:
        _lib.diag_set("launch_keys", 1)
        _lib.check(lib.nwc_set_committee(None, 0))


def test_cfg3_host_entry_and_oracle_sample(cfg3, oracle):
    from narwhal_amd import _lib
    lib = _lib.load()
    w = cfg3
    d, o, p, s = (np.ascontiguousarray(t.cpu().numpy()) for t in (w["cdig"], w["offs"], w["pks"], w["sigs"]))
    nv = M * Q
    for call in ("first", "steady"):
        cert = ctypes.create_string_buffer((M + 7) // 8)
        badb = ctypes.create_string_buffer((nv + 7) // 8)
        _lib.check(lib.nwc_verify_batch_many(_lib.buf(d), _lib.buf(o), _lib.buf(p), _lib.buf(s), M, cert, badb))
        got_bad = np.unpackbits(np.frombuffer(badb.raw, np.uint8), bitorder="little")[:nv].astype(bool)
        got_cert = np.unpackbits(np.frombuffer(cert.raw, np.uint8), bitorder="little")[:M].astype(bool)
        assert (got_bad == w["want_bad"]).all(), call
        assert (got_cert == w["want_cert"]).all(), call
    _lib.check(lib.nwc_set_committee(None, 0))
    # 2,000 random certificates against the CPU restatement (bisection leaves included)
    rng = np.random.default_rng(0xC3)
    pick = np.sort(rng.choice(M, 2000, replace=False))
    vid = (pick[:, None] * Q + np.arange(Q)[None, :]).reshape(-1)
    so = (np.arange(len(pick) + 1) * Q).astype(np.uint32)
    ocert, obad = oracle.batch_many(d[pick], so, p[vid], s[vid], threads=16)
    assert (ocert == w["want_cert"][pick]).all()
    assert (obad == w["want_bad"][vid]).all()
