"""BASELINE config 5: 64M mixed signatures -- 99 % honest, 1 % edge
cases spread over the golden edge classes (small-order / non-canonical A and R, s >= l, ...) --
verified with verify_strict, sharded over ranks, verdict words all-gathered.

* full size on one GPU, in process, through bench.bench_cfg5 (the bench's own leg);
* the sharded form over 2, 4 and 8 ranks (config 5's full width): bench.py under torch.distributed.run with the gloo
  backend, every rank on this box's one GPU (the driver's 8-GPU node runs the same code with RCCL,
  one GPU per rank).  Each rank generates its contiguous shard, verifies it, and the verdict words
  are all-gathered and compared with each rank's own; expected verdicts come from the golden
  fixtures (oracle-pinned, tests/test_oracle_golden.py).
"""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def test_cfg5_full_size_one_gpu():
    sys.path.insert(0, ROOT)
    import bench
    from narwhal_amd import _lib
    out = bench.bench_cfg5(_lib.load(), 0, 1, 64 << 20, 1)
    assert out["parity_ok"], out
    assert out["per_gpu"] == 64 << 20 and out["edge_slots_per_gpu"] > 600000


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg5_sharded_gloo(world):
    port = 29500 + (os.getpid() * 7 + world) % 2000
    env = dict(os.environ, NWC_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", "1", "--warmup", "1", "--triples", "65536", "--digest-batches", "0",
           "--cpu-budget", "0", "--cfg3-certs", "0", "--cfg1-calls", "0", "--wire-certs", "0",
           "--cfg5-total", str(3 * (1 << 20) + 4096 * world)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=240 + 40 * world)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == world and line["config"]["verdicts_ok"]
    c5 = line["configs"]["cfg5"]
    assert c5["parity_ok"], c5
    assert c5["per_gpu"] == (3 * (1 << 20) + 4096 * world) // world
    assert c5["verdict_allgather_ms"] is not None
