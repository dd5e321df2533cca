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


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    """Name the library this session tested: the build id libnwc.so embeds and the hash of the
    sources in this tree (narwhal_amd/build.py), so the run's output proves which binary ran."""
    try:
        from narwhal_amd import build
        lib_id = build.embedded_id()
        terminalreporter.write_line("libnwc.so build id %s; sources in this tree %s%s" % (
            lib_id, build.source_id(), "" if lib_id == build.source_id() else "  (MISMATCH: stale library)"))
    except Exception as e:  # noqa: BLE001
        terminalreporter.write_line("libnwc.so build id unavailable: %r" % (e,))
