"""The half-size (lattice) path, the full-length path and the fallback kernel give identical
verdicts (each in its own process; libnwc reads the path switches once)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT, GOLDEN

pytestmark = pytest.mark.gpu


def _inputs(oracle, tmp_path):
    import json
    rng = np.random.default_rng(21)
    n = 6000
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    kind = rng.integers(0, 5, n)
    for i in np.nonzero(kind == 1)[0]:
        sigs[i, rng.integers(0, 64)] ^= np.uint8(1 << rng.integers(0, 8))
    for i in np.nonzero(kind == 2)[0]:
        msgs[i, rng.integers(0, 32)] ^= 1
    g = json.load(open(os.path.join(GOLDEN, "ed25519_verify.json")))["cases"]
    g = [c for c in g if len(c["msg"]) == 64]
    gm = np.stack([np.frombuffer(bytes.fromhex(c["msg"]), np.uint8) for c in g])
    gp = np.stack([np.frombuffer(bytes.fromhex(c["pk"]), np.uint8) for c in g])
    gs = np.stack([np.frombuffer(bytes.fromhex(c["sig"]), np.uint8) for c in g])
    m, p, s = np.concatenate([msgs, gm]), np.concatenate([pks, gp]), np.concatenate([sigs, gs])
    path = str(tmp_path / "in.npz")
    np.savez(path, m=m, p=p, s=s)
    return path, m, p, s


def _run(inp, out, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "gpu_verify_helper.py"), inp, out, ROOT],
                   env=env, check=True, timeout=600)
    return np.load(out)


def test_half_full_fallback_agree_with_oracle(oracle, tmp_path):
    inp, m, p, s = _inputs(oracle, tmp_path)
    exp_strict = oracle.strict_many(m, p, s)
    exp_leaf = oracle.leaf_many(m, p, s)
    for tag, env in (("half", {}), ("full", {"NWC_VERIFY_PATH": "full"}),
                     ("fallback", {"NWC_FORCE_FALLBACK_EVERY": "3"})):
        r = _run(inp, str(tmp_path / ("out_%s.npz" % tag)), env)
        assert (r["strict"] == exp_strict).all(), (tag, np.nonzero(r["strict"] != exp_strict)[0][:10])
        assert (r["leaf"] == exp_leaf).all(), (tag, np.nonzero(r["leaf"] != exp_leaf)[0][:10])
