import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs the HIP path through the C ABI")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden_verify():
    with open(os.path.join(GOLDEN, "ed25519_verify.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_batch():
    with open(os.path.join(GOLDEN, "ed25519_batch.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_sha():
    with open(os.path.join(GOLDEN, "sha512.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    from tests.oracle_lib import load_oracle
    return load_oracle()
