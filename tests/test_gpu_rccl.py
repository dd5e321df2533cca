"""RCCL on the box: the "nccl" process group initialises with one GPU per rank (device_id) and
the collectives of bench.py's N > 1 path -- all_gather_into_tensor of verdict words, all_reduce
MAX of step times, barrier -- return the right values (world size 1 here; the driver's 8-GPU
runs make the same calls).  In a subprocess, so the process group does not outlive the test."""
import os
import random
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def test_rccl_collectives_world1():
    port = str(random.randint(20000, 40000))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "rccl_helper.py"), port],
                       capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=port))
    assert r.returncode == 0, (r.stdout[-500:], r.stderr[-2000:])
    assert "RCCL_OK" in r.stdout, (r.stdout[-500:], r.stderr[-2000:])
