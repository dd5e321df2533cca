"""GPU parity of the cold kernel (narwhal_amd/csrc/kernels.hip, k_verify_cold): calls of at most
NWC_COLD_MAX (3072) equations whose keys no cache holds run one limb-sliced block per equation,
with the batch leaf's torsion test (l A = [2^252] A + [l - 2^252] A) inside the same block.  Every
golden verify case (torsion keys, small-order A and R, non-canonical encodings, s >= l) goes
through it in both modes against the fixture's `strict` / `leaf` verdicts, and random triples with
corruptions against the oracle (dalek verify_strict / the batch leaf restated)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _verify(m, p, s, strict):
    import torch
    from narwhal_amd import device
    tm, tp, ts = (torch.from_numpy(np.ascontiguousarray(x)).cuda() for x in (m, p, s))
    w = device.verify(tm, tp, ts, strict=strict)
    torch.cuda.synchronize()
    return device.unpack_bits(w, p.shape[0])


def test_cold_golden_cases(golden_verify):
    from narwhal_amd import _lib
    lib = _lib.load()
    _lib.check(lib.nwc_set_committee(None, 0))
    cases = [c for c in golden_verify["cases"] if len(c["msg"]) == 64]
    arr = lambda k: np.stack([np.frombuffer(bytes.fromhex(c[k]), np.uint8) for c in cases])  # noqa: E731
    m, p, s = arr("msg"), arr("pk"), arr("sig")
    rng = np.random.default_rng(11)
    for n in (1, 3, 64, 1000, 3000):
        idx = rng.integers(0, len(cases), n) if n < len(cases) else np.resize(rng.permutation(len(cases)), n)
        for strict in (True, False):
            got = _verify(m[idx], p[idx], s[idx], strict)
            exp = np.array([cases[i]["strict" if strict else "leaf"] for i in idx])
            bad = [cases[idx[k]]["name"] for k in np.nonzero(got != exp)[0][:6]]
            assert not bad, (n, strict, bad)


def test_cold_random_triples(oracle):
    import torch
    from narwhal_amd import device
    n = 1000
    msgs = device.derive32(b"cold-msg", 0, n)
    pks, sigs = device.keygen_sign(device.derive32(b"cold-seed", 0, n), msgs)
    m, p, s = (t.cpu().numpy().copy() for t in (msgs, pks, sigs))
    rng = np.random.default_rng(5)
    for i in np.nonzero(rng.random(n) < 0.3)[0]:
        col = rng.integers(0, 96)
        if col < 64:
            s[i, col] ^= 1 << rng.integers(0, 8 if col < 63 else 4)
        else:
            m[i, col - 64] ^= 1 << rng.integers(0, 8)
    assert torch.cuda.is_available()
    got_s = _verify(m, p, s, True)
    got_l = _verify(m, p, s, False)
    assert (got_s == oracle.strict_many(m, p, s)).all()
    assert (got_l == oracle.leaf_many(m, p, s)).all()
    assert 0.6 * n < got_s.sum() < 0.8 * n
