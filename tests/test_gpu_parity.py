"""GPU parity: the HIP path (through the C ABI) against the golden fixtures and the oracle.

Bar: bit-exact verdicts, bad-vote sets and digests.  Small sizes are compared with the oracle
element by element; full BASELINE sizes are checked through size-independent properties
(all-valid sets verify, exactly the corrupted indices fail, digests of cycled batches match).
"""
import ctypes
import hashlib
import os
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


@pytest.fixture(scope="module")
def lib():
    from narwhal_amd import _lib
    return _lib.load()


@pytest.fixture(scope="module")
def torch_dev():
    import torch
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return torch


def _bits(raw: bytes, n: int) -> np.ndarray:
    return np.unpackbits(np.frombuffer(raw, dtype=np.uint8), bitorder="little")[:n].astype(bool)


def _strict_many(lib, msgs: np.ndarray, pks: np.ndarray, sigs: np.ndarray) -> np.ndarray:
    n = pks.shape[0]
    out = ctypes.create_string_buffer((n + 7) // 8)
    from narwhal_amd import _lib
    _lib.check(lib.nwc_verify_strict_many(_lib.buf(msgs), _lib.buf(pks), _lib.buf(sigs), n, out))
    return _bits(out.raw, n)


# ----------------------------------------------------------------------------- digests
def test_digest_golden_small(lib, golden_sha):
    from narwhal_amd import crypto
    for c in golden_sha["small"]:
        m = bytes.fromhex(c["msg"])
        assert crypto.digest_bytes(m).to_vec().hex() == c["digest32"], c["name"]
    got = crypto.digest_many([bytes.fromhex(c["msg"]) for c in golden_sha["small"]])
    assert [g.to_vec().hex() for g in got] == [c["digest32"] for c in golden_sha["small"]]


def test_digest_cfg4_batches(lib, golden_sha):
    import make_golden
    from narwhal_amd import crypto
    batches = [make_golden.cfg4_batch(int(c["recipe"].split("(")[1].rstrip(")"))) for c in golden_sha["cfg4"]]
    got = crypto.digest_many(batches)
    assert [g.to_vec().hex() for g in got] == [c["digest32"] for c in golden_sha["cfg4"]]


def test_digest_random_lengths_vs_hashlib(lib):
    from narwhal_amd import crypto
    rng = np.random.default_rng(11)
    lens = list(range(0, 300)) + list(rng.integers(0, 5000, 200))
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    got = crypto.digest_many(msgs)
    for m, g in zip(msgs, got):
        assert g.to_vec() == hashlib.sha512(m).digest()[:32], len(m)


def _sched_count(torch):
    """Messages per launch above which launch_digest takes the McNaughton-scheduled kernel."""
    return 64 * 4 * torch.cuda.get_device_properties(0).multi_processor_count


def test_digest_scheduled_ragged_vs_hashlib(lib, torch_dev):
    """k_sha512_digest32_sched: > one wave per SIMD of ragged messages (short, long, empty,
    unaligned), so lane segments cut messages and hand chaining values over between lanes."""
    torch = torch_dev
    from narwhal_amd import device
    rng = np.random.default_rng(21)
    n = _sched_count(torch) + 4321
    lens = rng.integers(0, 2500, n)
    lens[rng.integers(0, n, 40)] = rng.integers(20_000, 300_000, 40)   # a few long ones set T
    lens[rng.integers(0, n, 200)] = 0
    blob = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    data = torch.from_numpy(blob).cuda()
    out = device.sha512_trunc32(data, torch.from_numpy(offs).cuda())
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    raw = blob.tobytes()
    bad = [i for i in range(n) if o[i].tobytes() != hashlib.sha512(raw[offs[i]:offs[i + 1]]).digest()[:32]]
    assert not bad, (len(bad), bad[:10])


def test_digest_scheduled_cfg4_shape(lib, torch_dev):
    """Config-4 shape through the scheduled kernel: > one wave per SIMD of 508,052-B batches
    (a pool of 48 distinct aligned batches cycled by range), every digest checked."""
    torch = torch_dev
    import make_golden
    from narwhal_amd import device
    pool = 48
    batches = [make_golden.cfg4_batch(i) for i in range(pool)]
    stride = (len(batches[0]) + 255) & ~255
    blob = np.zeros(stride * pool, dtype=np.uint8)
    for i, b in enumerate(batches):
        blob[i * stride:i * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
    want = [hashlib.sha512(b).digest()[:32] for b in batches]
    n = _sched_count(torch) + 1000
    idx = (np.arange(n) * 7) % pool
    starts = torch.from_numpy((idx * stride).astype(np.int64)).cuda()
    ends = starts + len(batches[0])
    out = device.sha512_trunc32_ranges(torch.from_numpy(blob).cuda(), starts, ends)
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    bad = [i for i in range(n) if o[i].tobytes() != want[idx[i]]]
    assert not bad, (len(bad), bad[:10])


def test_digest_device_resident_unaligned(lib, torch_dev):
    """nwc_dev_sha512_trunc32 on contiguous (unaligned) offsets, the reference's own layout."""
    torch = torch_dev
    from narwhal_amd import device
    rng = np.random.default_rng(12)
    lens = rng.integers(0, 3000, 500)
    msgs = [rng.integers(0, 256, int(n), dtype=np.uint8).tobytes() for n in lens]
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    data = torch.from_numpy(np.frombuffer(b"".join(msgs) + bytes(16), dtype=np.uint8).copy()).cuda()
    out = device.sha512_trunc32(data, torch.from_numpy(offs).cuda())
    torch.cuda.synchronize()
    o = out.cpu().numpy()
    for i, m in enumerate(msgs):
        assert o[i].tobytes() == hashlib.sha512(m).digest()[:32]


# ----------------------------------------------------------------------------- fixtures
def test_strict_golden_cases(lib, golden_verify):
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    assert len(cases) > 100
    m = np.stack([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in cases])
    p = np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in cases])
    s = np.stack([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in cases])
    got = _strict_many(lib, m, p, s)
    exp = np.array([c["strict"] for c in cases])
    bad = [cases[i]["name"] for i in np.nonzero(got != exp)[0]]
    assert not bad, bad


def test_leaf_golden_cases(lib, golden_verify, torch_dev):
    torch = torch_dev
    from narwhal_amd import device
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    m = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in cases])).cuda()
    p = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in cases])).cuda()
    s = torch.tensor(np.stack([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in cases])).cuda()
    words = device.verify(m, p, s, strict=False)
    got = device.unpack_bits(words, len(cases))
    exp = np.array([c["leaf"] for c in cases])
    bad = [cases[i]["name"] for i in np.nonzero(got != exp)[0]]
    assert not bad, bad


def test_reference_crypto_tests(lib, golden_verify, golden_batch):
    """crypto/src/tests/crypto_tests.rs:49-115 through the crate mirror."""
    from narwhal_amd.crypto import CryptoError, Digest, PublicKey, Signature
    by = {c["name"]: c for c in golden_verify["cases"]}
    ok = by["ref-verify_valid_signature"]
    Signature.from_bytes(bytes.fromhex(ok["sig"])).verify(Digest(bytes.fromhex(ok["msg"])),
                                                          PublicKey(bytes.fromhex(ok["pk"])))
    bad = by["ref-verify_invalid_signature"]
    with pytest.raises(CryptoError):
        Signature.from_bytes(bytes.fromhex(bad["sig"])).verify(Digest(bytes.fromhex(bad["msg"])),
                                                               PublicKey(bytes.fromhex(bad["pk"])))
    bb = {b["name"]: b for b in golden_batch}
    for name in ("ref-verify_valid_batch", "ref-verify_invalid_batch"):
        b = bb[name]
        votes = [(PublicKey(bytes.fromhex(p)), Signature.from_bytes(bytes.fromhex(s))) for p, s in b["votes"]]
        if b["verdict"]:
            Signature.verify_batch(Digest(bytes.fromhex(b["msg"])), votes)
        else:
            with pytest.raises(CryptoError):
                Signature.verify_batch(Digest(bytes.fromhex(b["msg"])), votes)


def test_batch_golden_cases(lib, golden_batch):
    """Signature::verify_batch verdicts and the exact bad-vote sets (bisection result, A.5);
    'randomized' cases (torsion-only residuals) must come back Err deterministically."""
    from narwhal_amd.crypto import CryptoError, Digest, PublicKey, Signature
    for b in golden_batch:
        votes = [(PublicKey(bytes.fromhex(p)), Signature.from_bytes(bytes.fromhex(s))) for p, s in b["votes"]]
        bad = []
        try:
            Signature.verify_batch(Digest(bytes.fromhex(b["msg"])), votes, bad=bad)
            verdict = True
        except CryptoError:
            verdict = False
        assert verdict == b["verdict"], b["name"]
        assert bad == b["bad"], b["name"]


def test_signing_matches_reference_keys(lib, golden_verify):
    """crypto_tests.rs keys()/Signature::new reproduced on the GPU signer (32-byte digests)."""
    from narwhal_amd.crypto import Digest, SecretKey, Signature, generate_keypair
    ref = golden_verify["reference_keys"]
    digest = Digest(bytes.fromhex(golden_verify["hello_digest"]))
    seed3 = bytes.fromhex(ref["seeds"][3])
    stream = iter([seed3])

    class Rng:
        def fill_bytes(self, n):
            return next(stream)

    pk, sk = generate_keypair(Rng())
    assert bytes(pk) == bytes.fromhex(ref["pks"][3])
    sig = Signature.new(digest, sk)
    exp = [c for c in golden_verify["cases"] if c["name"] == "ref-verify_valid_signature"][0]["sig"]
    assert sig.flatten().hex() == exp


# ----------------------------------------------------------------------------- random vs oracle
def test_keygen_sign_matches_oracle(lib, oracle, torch_dev):
    torch = torch_dev
    from narwhal_amd import device
    n = 2048
    seeds = device.derive32(b"nw-seed", 0, n)
    msgs = device.derive32(b"nw-msg", 0, n)
    pks, sigs = device.keygen_sign(seeds, msgs)
    torch.cuda.synchronize()
    s, m = seeds.cpu().numpy(), msgs.cpu().numpy()
    # derive32 == SHA-512(tag || u64le(i))[..32]
    for i in (0, 1, n - 1):
        assert s[i].tobytes() == hashlib.sha512(b"nw-seed" + i.to_bytes(8, "little")).digest()[:32]
    opk, osig = oracle.keygen_sign_many(s, m)
    assert (pks.cpu().numpy() == opk).all()
    assert (sigs.cpu().numpy() == osig).all()


def _random_triples(torch, device, n, tag=b"t"):
    seeds = device.derive32(b"nw-seed" + tag, 0, n)
    msgs = device.derive32(b"nw-msg" + tag, 0, n)
    pks, sigs = device.keygen_sign(seeds, msgs)
    return msgs, pks, sigs


def test_strict_random_mutations_vs_oracle(lib, oracle, torch_dev):
    torch = torch_dev
    from narwhal_amd import device
    n = 20000
    msgs, pks, sigs = _random_triples(torch, device, n)
    torch.cuda.synchronize()
    m, p, s = msgs.cpu().numpy(), pks.cpu().numpy(), sigs.cpu().numpy()
    rng = np.random.default_rng(5)
    kind = rng.integers(0, 8, n)
    for i in np.nonzero(kind == 1)[0]:
        s[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))      # flip a signature bit
    for i in np.nonzero(kind == 2)[0]:
        p[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))      # flip a key bit
    for i in np.nonzero(kind == 3)[0]:
        m[i, rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))      # wrong message
    for i in np.nonzero(kind == 4)[0]:
        s[i, 63] |= np.uint8(0x10 << rng.integers(0, 4))                     # s >= l region
    got = _strict_many(lib, m, p, s)
    exp = oracle.strict_many(m, p, s)
    diff = np.nonzero(got != exp)[0]
    assert diff.size == 0, diff[:20]
    assert exp[kind == 0].all() and exp.sum() < n


def test_leaf_and_certificates_vs_oracle(lib, oracle, torch_dev):
    """nwc_verify_batch_many: committee certificates with invalid votes (config 3 shape)."""
    torch = torch_dev
    from narwhal_amd import _lib, device
    N, Q, m = 100, 67, 300
    seeds = device.derive32(b"nw-committee", 0, N)
    rng = np.random.default_rng(9)
    digests = np.stack([np.frombuffer(hashlib.sha512(b"nw-cert" + c.to_bytes(8, "little")).digest()[:32], np.uint8)
                        for c in range(m)])
    voter = np.stack([rng.permutation(N)[:Q] for _ in range(m)])
    vs = seeds[torch.from_numpy(voter.reshape(-1)).cuda()]
    vm = torch.from_numpy(np.repeat(digests, Q, axis=0)).cuda()
    bad_mask = rng.random(m * Q) < 0.01
    vm_signed = vm.clone()
    vm_signed[torch.from_numpy(bad_mask).cuda(), 0] ^= 1          # invalid vote: signs another digest
    pks, sigs = device.keygen_sign(vs, vm_signed)
    torch.cuda.synchronize()
    p, s = pks.cpu().numpy(), sigs.cpu().numpy()
    offs = (np.arange(m + 1) * Q).astype(np.uint32)
    cert = ctypes.create_string_buffer((m + 7) // 8)
    badb = ctypes.create_string_buffer((m * Q + 7) // 8)
    _lib.check(lib.nwc_verify_batch_many(_lib.buf(digests), _lib.buf(offs), _lib.buf(p), _lib.buf(s), m, cert, badb))
    ocert, obad = oracle.batch_many(digests, offs, p, s)
    assert (_bits(cert.raw, m) == ocert).all()
    assert (_bits(badb.raw, m * Q) == obad).all()
    assert (obad == bad_mask).all()
    # device-resident path: leaf equations + cert reduction
    lw = device.verify(torch.from_numpy(digests).cuda(), pks, sigs, strict=False,
                       msg_index=torch.from_numpy(np.repeat(np.arange(m), Q).astype(np.int32)).cuda())
    cw, bw = device.cert_reduce(lw, torch.from_numpy(offs.astype(np.int32)).cuda(), m * Q)
    torch.cuda.synchronize()
    assert (device.unpack_bits(cw, m) == ocert).all()
    assert (device.unpack_bits(bw, m * Q) == obad).all()


def test_broadcast_digest_batch_with_bad_votes(lib, oracle):
    """Signature::verify_batch with one digest for all votes (certificate, config 1 shape)."""
    from narwhal_amd import _lib
    import make_golden  # noqa: F401
    rng = np.random.default_rng(3)
    n = 67
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    digest = rng.integers(0, 256, 32, dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, np.tile(digest, (n, 1)))
    sigs[[3, 40], 33] ^= 1
    bad = ctypes.create_string_buffer((n + 7) // 8)
    rc = lib.nwc_verify_batch(_lib.buf(digest), _lib.buf(pks), _lib.buf(sigs), n, bad)
    assert rc == _lib.NWC_INVALID
    assert list(np.nonzero(_bits(bad.raw, n))[0]) == [3, 40]
    assert lib.nwc_verify_batch(_lib.buf(digest), None, None, 0, None) == _lib.NWC_OK  # empty -> Ok


# ----------------------------------------------------------------------------- full size
@pytest.mark.slow
def test_full_size_1m_all_valid_and_exact_failures(lib, oracle, torch_dev):
    """BASELINE config 2 size (1M triples): all valid verify; then exactly the corrupted
    indices fail (size-independent property), cross-checked with the oracle on those."""
    torch = torch_dev
    from narwhal_amd import device
    n = 1 << 20
    msgs, pks, sigs = _random_triples(torch, device, n, tag=b"")
    words = device.verify(msgs, pks, sigs, strict=True)
    torch.cuda.synchronize()
    assert device.unpack_bits(words, n).all()
    rng = np.random.default_rng(1)
    idx = np.sort(rng.choice(n, 257, replace=False))
    ti = torch.from_numpy(idx).cuda()
    sigs[ti, 45] ^= 0x20
    words = device.verify(msgs, pks, sigs, strict=True)
    torch.cuda.synchronize()
    got = device.unpack_bits(words, n)
    assert list(np.nonzero(~got)[0]) == list(idx)
    sub = [t[ti].cpu().numpy() for t in (msgs, pks, sigs)]
    assert not oracle.strict_many(*sub).any()


def test_host_calls_pipelined_chunks_vs_oracle(lib, oracle, torch_dev):
    """Host-memory calls of 2+ chunks (NWC_HOST_CHUNK = 131,072 equations) copy chunk k+1 while
    chunk k verifies: strict triples (per-triple digests) and certificates (msg_index into the
    digests; a certificate may straddle a chunk cut) with corrupted entries, against the oracle."""
    torch = torch_dev
    from narwhal_amd import _lib, device
    n = 2 * 131072 + 12345
    msgs, pks, sigs = _random_triples(torch, device, n, tag=b"chunks")
    m, p, s = (t.cpu().numpy().copy() for t in (msgs, pks, sigs))
    rng = np.random.default_rng(21)
    bad = np.sort(rng.choice(n, 997, replace=False))
    s[bad[::2], 40] ^= 4
    m[bad[1::2], 7] ^= 1
    got = _strict_many(lib, m, p, s)
    assert (got == oracle.strict_many(m, p, s)).all()
    assert list(np.nonzero(~got)[0]) == list(bad)
    # certificates of 67 votes over one digest each, the votes signed by device keys
    Q, mc = 67, n // 67
    digests = rng.integers(0, 256, (mc, 32), dtype=np.uint8)
    vm = torch.from_numpy(np.repeat(digests, Q, axis=0)).cuda()
    pk2, sg2 = device.keygen_sign(device.derive32(b"chunks-seed", 0, mc * Q), vm)
    p2, s2 = pk2.cpu().numpy().copy(), sg2.cpu().numpy().copy()
    s2[rng.choice(mc * Q, 500, replace=False), 33] ^= 1
    offs = (np.arange(mc + 1) * Q).astype(np.uint32)
    cert = ctypes.create_string_buffer((mc + 7) // 8)
    badb = ctypes.create_string_buffer((mc * Q + 7) // 8)
    _lib.check(lib.nwc_verify_batch_many(_lib.buf(digests), _lib.buf(offs), _lib.buf(p2), _lib.buf(s2), mc, cert, badb))
    ocert, obad = oracle.batch_many(digests, offs, p2, s2)
    assert (_bits(cert.raw, mc) == ocert).all()
    assert (_bits(badb.raw, mc * Q) == obad).all()
