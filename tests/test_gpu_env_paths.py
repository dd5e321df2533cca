"""Small-call paths selected by process-wide switches, each in its own process (libnwc reads them
once): NWC_ZERO_COPY=0 (staged H2D/D2H copies instead of the zero-copy latency launch),
NWC_SPIN_WAIT=0 (the zero-copy launch waited on its stream instead of polled), NWC_AUTO_KEYS=2
(an auto key cache that fills up after two keys), NWC_COLD=0 (first-sight calls on the one-lane
ladder with the torsion test beside it instead of k_verify_cold) and NWC_FORCE_FALLBACK_EVERY=2
(every other equation treated as a failed reduction: the zero-copy cold launch hands the call back
to the staged path, whose fallback kernel decides those equations).  Verdicts and bad-vote sets
must equal the golden fixtures on every path, with and without the committee cache."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("env", [{"NWC_ZERO_COPY": "0"}, {"NWC_SPIN_WAIT": "0"}, {"NWC_AUTO_KEYS": "2"},
                                 {"NWC_AUTO_KEYS": "0"}, {"NWC_COLD": "0"}, {"NWC_FORCE_FALLBACK_EVERY": "2"}])
def test_small_call_paths_match_fixtures(env, golden_verify, golden_batch, tmp_path):
    out = tmp_path / "out.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tests", "env_paths_helper.py"), str(out), ROOT],
                   env=dict(os.environ, **env), check=True, timeout=600)
    got = json.load(open(out))
    exp_b = {b["name"]: b for b in golden_batch}
    for name, rc, bad in got["batch"]:
        assert rc == (0 if exp_b[name]["verdict"] else 1), (env, name)
        assert bad == exp_b[name]["bad"], (env, name)
    exp_s = {c["name"]: c for c in golden_verify["cases"]}
    for name, rc in got["strict"]:
        assert rc == (0 if exp_s[name]["strict"] else 1), (env, name)
    auto = [a for _, a in got["stats"]]
    if env.get("NWC_AUTO_KEYS") == "2":
        assert max(auto) == 2          # filled up, never beyond its capacity
    if env.get("NWC_AUTO_KEYS") == "0":
        assert max(auto) == 0
