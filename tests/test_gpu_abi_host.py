"""The C ABI from a plain C host (tests/cpp/abi_host.c): no Python or torch in the verifying
process, as in the Rust `crypto` shim of INTEGRATION.md.  Golden strict verdicts, the reference
batch cases with their bad-vote bitmaps, and SHA-512 digests, through nwc_verify_strict /
nwc_verify_batch / nwc_sha512_trunc32_many."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tests", "cpp", "build", "abi_host")


def build_abi_host() -> str:
    """gcc, linked against the in-tree libnwc.so (rpath relative to the binary)."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "abi_host.c"), "-L" + os.path.join(ROOT, "narwhal_amd"),
                    "-l:libnwc.so", "-Wl,-rpath,$ORIGIN/../../../narwhal_amd", "-o", BIN], check=True)
    return BIN


def test_c_host_golden(golden_verify, golden_batch, golden_sha):
    if not os.path.exists(BIN):
        build_abi_host()
    lines, want = [], []
    for c in golden_verify["cases"]:
        if len(c["msg"]) != 64:   # the crate surface always passes 32-byte digests
            continue
        lines.append("S %s %s %s" % (c["msg"], c["pk"], c["sig"]))
        want.append("S %d" % (0 if c["strict"] else 1))
    for b in golden_batch:
        n = len(b["votes"])
        lines.append("B %s %d %s" % (b["msg"], n, " ".join("%s %s" % (p, s) for p, s in b["votes"])))
        bits = bytearray((n + 7) // 8)
        for i in b["bad"]:
            bits[i >> 3] |= 1 << (i & 7)
        want.append(("B %d %s" % (0 if b["verdict"] else 1, bits.hex())).rstrip())
    for c in golden_sha["small"]:
        lines.append("D %s" % c["msg"])
        want.append("D %s" % c["digest32"])
    r = subprocess.run([BIN], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout[-500:], r.stderr[-500:])
    got = [l.rstrip() for l in r.stdout.splitlines()]
    assert len(got) == len(want), (len(got), len(want))
    bad = [(i, g, w) for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, bad[:5]
