"""BASELINE config 3 at world > 1 (whole certificates, balanced by votes): bench.py
under torch.distributed.run with the gloo backend, 2 and 4 ranks sharing this box's one GPU (the
driver's 8-GPU node runs the same code with RCCL, one GPU per rank).  Each rank verifies its
certificates' votes through the production batch-leaf path (launch keys), the certificate and
bad-vote words are all-gathered, and rank 0 compares the whole set with the construction
(primary/src/messages.rs:189-215: a certificate passes iff every vote verifies)."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4])
def test_cfg3_sharded_gloo(world):
    port = 31500 + (os.getpid() * 11 + world) % 2000
    certs = 4001   # uneven whole-certificate shards, each >= LK_MIN_EQUATIONS (65,536) votes at world 4
    env = dict(os.environ, NWC_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "2", "--warmup", "1", "--triples", "65536", "--digest-batches", "0",
           "--cpu-budget", "0", "--cfg3-certs", str(certs), "--cfg1-calls", "0", "--wire-certs", "0",
           "--cfg5-total", "0", "--clock-s", "0"]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240 + 40 * world)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    c3 = line["configs"]["cfg3"]
    assert c3["parity_ok"], c3
    assert c3["verdict_allgather_ms"] is not None and c3["allgather_needed"] is False
    assert c3["launch_keys"]["launch_keys_held"] == 100, c3
    assert abs(c3["votes_per_gpu"] - certs * 67 / world) <= 67, c3
