"""The library's multi-device host paths on a one-GPU box: NWC_VIRTUAL_DEVICES=k (3, and 8 = one
node's width) makes nwc_init open k contexts on the GPU, so nwc_verify_strict_many's shard threads and bitmap merge,
nwc_verify_batch_many's, nwc_verify_batch_straus_many's and nwc_verify_batch_msm_many's certificate cuts
and nwc_sha512_trunc32_many's
split all run as with three
GPUs.  Outputs must equal the oracle's bit for bit, including verdicts that
straddle the shard boundaries."""
import hashlib
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("contexts", [3, 8])
def test_contexts_match_oracle(oracle, tmp_path, contexts):
    rng = np.random.default_rng(31)
    n = 9001                                        # > 4096: sharded; 9001 = not a multiple of 64
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    flip = rng.random(n) < 0.05
    flip[[0, 63, 64, 3000, 3007, 3008, 6015, 6016, n - 1]] = True   # around the 64-aligned cuts
    sigs[flip, 40] ^= 2
    # certificates over the same votes: 1..90 votes each (a few empty), one digest per certificate
    sizes = []
    while sum(sizes) < n:
        sizes.append(int(rng.integers(0, 91)))
    sizes[-1] -= sum(sizes) - n
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    dig = np.zeros((len(sizes), 32), np.uint8)
    vm = msgs.copy()
    for c in range(len(sizes)):
        dig[c] = msgs[offs[c]] if sizes[c] else 0
        vm[offs[c]:offs[c + 1]] = dig[c]
    vp, vs = oracle.keygen_sign_many(seeds, vm)
    vs[flip, 41] ^= 4
    lens = rng.integers(0, 3000, 5000)
    blob = rng.integers(0, 256, int(lens.sum()) + 16, dtype=np.uint8)
    boffs = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    np.savez(tmp_path / "in.npz", m=msgs, p=pks, s=sigs, offs=offs, dig=dig, blob=blob, boffs=boffs)
    env = dict(os.environ, NWC_VIRTUAL_DEVICES=str(contexts))
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "multidev_helper.py"), str(tmp_path / "in.npz"),
                    str(tmp_path / "out.npz"), ROOT], env=env, check=True, timeout=300)
    got = np.load(tmp_path / "out.npz")
    assert int(got["devices"][0]) == contexts
    bits = lambda raw, k: np.unpackbits(raw, bitorder="little")[:k].astype(bool)  # noqa: E731
    assert (bits(got["strict"], n) == oracle.strict_many(msgs, pks, sigs)).all()
    # batch: certificates over (vp, vs) -- rerun the helper's call shape against the oracle
    np.savez(tmp_path / "in2.npz", m=msgs, p=vp, s=vs, offs=offs, dig=dig, blob=blob[:16], boffs=np.zeros(2, np.uint64))
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "multidev_helper.py"), str(tmp_path / "in2.npz"),
                    str(tmp_path / "out2.npz"), ROOT], env=env, check=True, timeout=300)
    got2 = np.load(tmp_path / "out2.npz")
    ocert, obad = oracle.batch_many(dig, offs, vp, vs)
    assert (bits(got2["cert"], len(sizes)) == ocert).all()
    assert (bits(got2["bad"], n) == obad).all() and obad.sum() >= flip.sum()
    # the Straus host entry over the same certificate cuts (honest keys: the deterministic domain)
    assert (bits(got2["cert_straus"], len(sizes)) == ocert).all()
    assert (bits(got2["bad_straus"], n) == obad).all()
    # and the Pippenger host entry (its groups fall back to the sub-batches, then the leaves)
    assert (bits(got2["cert_msm"], len(sizes)) == ocert).all()
    assert (bits(got2["bad_msm"], n) == obad).all()
    raw = blob.tobytes()
    for i in range(len(lens)):
        assert got["digests"][i].tobytes() == hashlib.sha512(raw[boffs[i]:boffs[i + 1]]).digest()[:32], i


def test_contexts_device_vote_index(tmp_path):
    """Ragged certificates (0..130 votes, empty ones included) over 3 contexts with ~280k votes per
    context: every shard takes the pipelined path and builds its vote -> certificate index on the
    device (k_cert_index) from a range starting at a certificate boundary lo > 0.
    Votes reuse a table of 100 keys x 40 digests; expected verdicts come from the construction."""
    from tests.conftest import ROOT as root
    from tests.oracle_lib import load_oracle
    oracle = load_oracle()
    rng = np.random.default_rng(37)
    K, D = 100, 40
    seeds = rng.integers(0, 256, (K, 32), dtype=np.uint8)
    dtab = rng.integers(0, 256, (D, 32), dtype=np.uint8)
    pk_t, sig_t = oracle.keygen_sign_many(np.repeat(seeds, D, axis=0), np.tile(dtab, (K, 1)))
    m = 13000
    counts = rng.integers(0, 131, m)
    counts[[0, 4333, 8666, m - 1]] = 0
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    nv = int(offs[-1])
    dc = rng.integers(0, D, m)
    vote_cert = np.repeat(np.arange(m), counts)
    rows = rng.integers(0, K, nv) * D + dc[vote_cert]
    vp, vs = pk_t[rows], sig_t[rows].copy()
    bad = rng.random(nv) < 0.01
    vs[bad, 9] ^= 0x20
    dig = np.ascontiguousarray(dtab[dc])
    np.savez(tmp_path / "in.npz", m=np.zeros((nv, 32), np.uint8), p=vp, s=vs, offs=offs, dig=dig,
             blob=np.zeros(16, np.uint8), boffs=np.zeros(2, np.uint64))
    env = dict(os.environ, NWC_VIRTUAL_DEVICES="3")
    subprocess.run([sys.executable, os.path.join(root, "tests", "multidev_helper.py"), str(tmp_path / "in.npz"),
                    str(tmp_path / "out.npz"), root], env=env, check=True, timeout=300)
    got = np.load(tmp_path / "out.npz")
    assert int(got["devices"][0]) == 3
    bits = lambda raw, k: np.unpackbits(raw, bitorder="little")[:k].astype(bool)  # noqa: E731
    exp_cert = np.bincount(vote_cert[bad], minlength=m) == 0
    for c, b in (("cert", "bad"), ("cert_straus", "bad_straus"), ("cert_msm", "bad_msm")):
        assert (bits(got[b], nv) == bad).all(), (b, np.nonzero(bits(got[b], nv) != bad)[0][:10])
        assert (bits(got[c], m) == exp_cert).all(), (c, np.nonzero(bits(got[c], m) != exp_cert)[0][:10])
