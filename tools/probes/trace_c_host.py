#!/usr/bin/env python3
"""The plain C host (tests/cpp/build/abi_host: gcc, libnwc.so, no torch or Python in the process)
under rocprofv3's kernel + memory-copy trace, on golden batches, a sharded strict request,
certificates, the wire-message pipeline and a digester group: does the tracer report memory
copies whose completions HSA never delivered (round-4 review, "what's weak" #6)?

    python tools/probes/trace_c_host.py OUTDIR
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    out = os.path.abspath(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "c_host_trace"))
    os.makedirs(out, exist_ok=True)
    from asan_exit_probe import requests
    from tests.test_gpu_abi_host import BIN, _message_requests
    mlines, _ = _message_requests()
    inp = requests().rstrip("\n").split("\n")
    inp = inp[:-1] + mlines + inp[-1:]
    env = dict(os.environ, TMPDIR="/tmp", NWC_HOST_EXIT="return")   # _exit would skip the tracer's own finalisation
    r = subprocess.run(["rocprofv3", "--kernel-trace", "--memory-copy-trace", "--output-format", "csv", "-d", out,
                        "-o", "run", "--", BIN], input="\n".join(inp) + "\n", capture_output=True, text=True,
                       timeout=300, env=env, cwd="/tmp")
    open(os.path.join(out, "stderr.txt"), "w").write(r.stderr)
    lines = r.stdout.splitlines()
    warn = [l for l in r.stderr.splitlines() if "completion callbacks" in l or "dangling" in l]
    print("rc %d, %d response lines, %d tracer warnings" % (r.returncode, len(lines), len(warn)))
    for w in warn[:12]:
        print("  " + w[w.find("]") + 1:].strip())


if __name__ == "__main__":
    main()
