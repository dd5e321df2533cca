"""The C ABI from a plain C host (tests/cpp/abi_host.c): no Python or torch in the verifying
process, as in the Rust `crypto` shim of INTEGRATION.md.  Golden strict verdicts, the reference
batch cases with their bad-vote bitmaps, and SHA-512 digests, through nwc_verify_strict /
nwc_verify_batch / nwc_sha512_trunc32_many; and, in the AddressSanitizer + UBSan build, every
host entry with threads or queues behind it: sharded strict and certificate calls, the Straus and
MSM batch entries, the message pipeline, the worker digester (stages, receive arena, a failing group)
and a digester streaming while other threads verify on the same device."""
import hashlib
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tests", "cpp", "build", "abi_host")
ASAN_BIN = os.path.join(ROOT, "tests", "cpp", "build", "abi_host_asan")
ASAN_LIB = os.path.join(ROOT, "tests", "cpp", "build", "libnwc_asan.so")


def _stale(out, srcs):
    return not os.path.exists(out) or any(os.path.getmtime(x) > os.path.getmtime(out) for x in srcs)


def build_abi_host() -> str:
    """gcc, linked against the in-tree libnwc.so (rpath relative to the binary); and the sanitized
    pair: libnwc's HOST code under AddressSanitizer + UBSan (`-Xarch_host -fsanitize=...`; the
    gfx950 device code is built as usual) with the same C host built by ROCm's clang."""
    os.makedirs(os.path.dirname(BIN), exist_ok=True)
    src = os.path.join(ROOT, "tests", "cpp", "abi_host.c")
    inc = "-I" + os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", inc, src, "-L" + os.path.join(ROOT, "narwhal_amd"),
                    "-l:libnwc.so", "-lpthread", "-Wl,-rpath,$ORIGIN/../../../narwhal_amd", "-o", BIN], check=True)
    from narwhal_amd import build as nb
    if _stale(ASAN_LIB, nb.sources()):
        subprocess.run([nb.HIPCC, "--offload-arch=gfx950", "-O2", "-g", "-std=c++20", "-fPIC", "-shared",
                        "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
                        "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer",
                        inc, "-I" + nb.CSRC,
                        "-o", ASAN_LIB + ".tmp", os.path.join(nb.CSRC, "nwc_api.hip")], check=True)
        os.replace(ASAN_LIB + ".tmp", ASAN_LIB)
    if _stale(ASAN_BIN, [src, ASAN_LIB]):
        # compiled as C, linked by clang++: the sanitizer runtime's own operator new / delete then
        # serve libnwc's C++ allocations, so a leak report's stack (fast frame-pointer unwind)
        # reaches libnwc's frames instead of stopping inside libstdc++'s operator new
        obj = ASAN_BIN + ".o"
        subprocess.run(["/opt/rocm/llvm/bin/clang", "-c", "-O1", "-g", "-fno-omit-frame-pointer",
                        "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", inc, src, "-o", obj],
                       check=True)
        subprocess.run(["/opt/rocm/llvm/bin/clang++", "-fsanitize=address,undefined", obj,
                        "-L" + os.path.dirname(ASAN_LIB), "-l:" + os.path.basename(ASAN_LIB), "-lpthread",
                        "-Wl,-rpath,$ORIGIN", "-o", ASAN_BIN], check=True)
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


def _report_head(err):
    """The sanitizer report's first lines (error kind, access, the faulting stack), not its tail."""
    i = err.find("==ERROR")
    if i < 0:
        i = err.find("runtime error")
    return err[max(0, i - 200):i + 4000] if i >= 0 else err[-3000:]


def _keep_report(name, r):
    """A failing sanitizer run's whole stdout/stderr, kept where a GPU-box run's outputs come back."""
    import os
    from tests.conftest import ROOT
    d = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, name + ".stderr"), "w") as f:
            f.write(r.stderr)
        with open(os.path.join(d, name + ".stdout"), "w") as f:
            f.write(r.stdout)
    except OSError:
        pass


def asan_env(**extra):
    """The sanitized host's environment: leak checking on (the C host calls
    __lsan_do_recoverable_leak_check after nwc_shutdown; suppressions for the ROCm runtime's frames
    only, tests/cpp/lsan.supp), UBSan fatal with stacks, three virtual device contexts."""
    supp = os.path.join(ROOT, "tests", "cpp", "lsan.supp")
    return dict(os.environ, NWC_VIRTUAL_DEVICES="3", ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:malloc_context_size=40",
                LSAN_OPTIONS="suppressions=%s:print_suppressions=1" % supp,
                UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1", **extra)


def test_c_host_under_asan(oracle, golden_verify, golden_batch):
    """libnwc's host code (small-call staging, zero-copy path, auto key cache, shard threads and
    bitmap merges over NWC_VIRTUAL_DEVICES=3 contexts, certificate cuts, concurrent callers)
    under AddressSanitizer + UBSan: no report, and every output equal to the oracle's."""
    import numpy as np
    if _stale(ASAN_BIN, [ASAN_LIB]):
        build_abi_host()
    rng = np.random.default_rng(41)
    lines, want = [], []
    for b in golden_batch:
        n = len(b["votes"])
        lines.append("B %s %d %s" % (b["msg"], n, " ".join("%s %s" % (p, s) for p, s in b["votes"])))
        bits = bytearray((n + 7) // 8)
        for i in b["bad"]:
            bits[i >> 3] |= 1 << (i & 7)
        want.append(("B %d %s" % (0 if b["verdict"] else 1, bits.hex())).rstrip())
    # sharded strict verification: 9001 triples over three contexts, flips around the cuts
    n = 9001
    seeds = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    msgs = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    pks, sigs = oracle.keygen_sign_many(seeds, msgs)
    flip = rng.random(n) < 0.03
    flip[[0, 63, 64, 3000, 3007, 3008, 6015, 6016, n - 1]] = True
    sigs[flip, 40] ^= 2
    lines.append("V %d" % n)
    lines += ["%s %s %s" % (m.tobytes().hex(), p.tobytes().hex(), s.tobytes().hex()) for m, p, s in zip(msgs, pks, sigs)]
    exp = oracle.strict_many(msgs, pks, sigs)
    want.append("V 0 " + np.packbits(exp, bitorder="little").tobytes().hex())
    # the same triples tiled 90x (810k, 270k per virtual device): pipelined chunks, input copies
    # through the pinned stages
    lines.append("W 90")
    want.append("W 0")
    # certificates: 0..40 votes each over one digest per certificate
    sizes = [int(x) for x in rng.integers(0, 41, 200)]
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint32)
    nv = int(offs[-1])
    dig = rng.integers(0, 256, (len(sizes), 32), dtype=np.uint8)
    vm = np.repeat(dig, sizes, axis=0)
    vp, vs = oracle.keygen_sign_many(seeds[:nv], vm)
    bad = rng.random(nv) < 0.05
    vs[bad, 50] ^= 8
    lines.append("C %d %s" % (len(sizes), " ".join(str(int(o)) for o in offs)))
    lines += ["%s %s" % (p.tobytes().hex(), s.tobytes().hex()) for p, s in zip(vp, vs)]
    lines += [d.tobytes().hex() for d in dig]
    ocert, obad = oracle.batch_many(dig, offs, vp, vs)
    want.append("C 0 %s %s" % (np.packbits(ocert, bitorder="little").tobytes().hex(),
                               np.packbits(obad, bitorder="little").tobytes().hex()))
    # the same certificates through dalek's batch equation (Straus sub-batches + leaves): the
    # deterministic domain (honest keys, corrupted signatures), so exactly the oracle's answer
    lines.append("T %d %s" % (len(sizes), " ".join(str(int(o)) for o in offs)))
    lines += ["%s %s" % (p.tobytes().hex(), s.tobytes().hex()) for p, s in zip(vp, vs)]
    lines += [d.tobytes().hex() for d in dig]
    want.append("T" + want[-1][1:])
    # and as Pippenger groups (their failing groups through the sub-batches, then the leaves)
    lines.append("P %d %s" % (len(sizes), " ".join(str(int(o)) for o in offs)))
    lines += ["%s %s" % (p.tobytes().hex(), s.tobytes().hex()) for p, s in zip(vp, vs)]
    lines += [d.tobytes().hex() for d in dig]
    want.append("P" + want[-1][1:])
    lines.append("X 4 3")
    want.append("X 0")
    # Core::sanitize_* from wire bytes on the reference's fixtures and the restated negatives
    mlines, mwant = _message_requests()
    lines += mlines
    want += mwant
    # the worker digester from malloc'd batches (stage path) and from its receive arena, then
    # one digester streaming while four threads verify on the same device
    batches = [rng.integers(0, 256, int(k), dtype=np.uint8).tobytes() for k in
               [0, 1, 111, 112, 127, 128, 129, 255, 256] + [int(x) for x in rng.integers(0, 150_000, 40)]]
    for max_group, wait, arena in ((7, 0, 0), (64, 200_000, 0), (4096, 100_000, 1)):
        lines.append("G %d %d %d %d" % (max_group, wait, arena, len(batches)))
        lines += [b.hex() or "-" for b in batches]
        want += ["g %d %s" % (i, hashlib.sha512(b).digest()[:32].hex()) for i, b in enumerate(batches)]
        want.append("G 0")
    lines.append("Y 4 2")
    want.append("Y 0")
    env = asan_env()
    r = subprocess.run([ASAN_BIN], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=600, env=env)
    if r.returncode != 0:
        _keep_report("abi_host_asan", r)
    assert r.returncode == 0, (r.returncode, r.stdout[-500:], _report_head(r.stderr))
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-3000:]
    assert "LeakSanitizer" not in r.stderr and "leaks after nwc_shutdown" not in r.stderr, _report_head(r.stderr)
    # the leak check ran: LSan prints the suppressions it matched (the ROCm runtime's, if any)
    print(r.stderr[-2000:])
    got = [l.rstrip() for l in r.stdout.splitlines()]
    assert len(got) == len(want), (len(got), len(want), r.stderr[-1000:])
    mism = [(i, g[:80], str(w)[:80]) for i, (g, w) in enumerate(zip(got, want)) if not _same(g, w)]
    assert not mism, mism[:5]
    # a digest group that fails on the device (NWC_DIGEST_FAIL_GROUP=2, the second launch): its
    # tags come back with the error, the groups around it as digests, destroy reports the error
    small = [rng.integers(0, 256, 1000 + 10 * i, dtype=np.uint8).tobytes() for i in range(12)]
    fl = ["G 4 2000000 0 12"] + [b.hex() for b in small]
    fw = ["g %d %s" % (i, hashlib.sha512(b).digest()[:32].hex()) if not 4 <= i < 8 else "g %d ERR -1" % i
          for i, b in enumerate(small)] + ["G -1"]
    r = subprocess.run([ASAN_BIN], input="\n".join(fl) + "\n", capture_output=True, text=True, timeout=300,
                       env=dict(env, NWC_DIGEST_FAIL_GROUP="2"))
    assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, (r.returncode, r.stderr[-3000:])
    assert [l.rstrip() for l in r.stdout.splitlines()] == fw, r.stdout[-2000:]
    # the sanitizer is live in this process layout: an out-of-bounds heap read is reported
    r = subprocess.run([ASAN_BIN], input="Z\n", capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "heap-buffer-overflow" in r.stderr, (r.returncode, r.stderr[-500:])
    # the whole exit path -- main's return: the atexit handlers, libnwc's static destructors, the
    # HIP/HSA runtime's own teardown -- with ASan's quarantine off.  With it on, ASan recycles a
    # quarantined device-allocator chunk inside libamdhip64's __cxa_finalize and aborts on its
    # CHECK "dev_runtime_unloaded_" (no libnwc frame on that stack; 2 of 2 runs abort with the
    # quarantine, 0 of 3 without: profiles/r05/asan_exit.md)
    r = subprocess.run([ASAN_BIN], input="\n".join(lines[:len(golden_batch)] + ["Y 4 2"]) + "\n", capture_output=True,
                       text=True, timeout=300,
                       env=dict(env, NWC_HOST_EXIT="return", ASAN_OPTIONS=env["ASAN_OPTIONS"] + ":quarantine_size_mb=0"))
    if r.returncode != 0:
        _keep_report("abi_host_asan_exit", r)
    assert r.returncode == 0, (r.returncode, _report_head(r.stderr))
    assert "AddressSanitizer" not in r.stderr and "CHECK failed" not in r.stderr, r.stderr[-3000:]
    assert [l.rstrip() for l in r.stdout.splitlines()] == want[:len(golden_batch)] + ["Y 0"], r.stdout[-1000:]


def _same(got: str, want) -> bool:
    """A line equal to the expected text, or an M line matching a checker function."""
    return want(got) if callable(want) else got == want


def _message_requests():
    """Q (committee config) + one M request per (gc_round, target) group of the golden message
    fixtures (tests/golden/messages.json), with a checker per M line: codes always, the digest and
    kind where the fixture has them."""
    import json
    from tests.conftest import GOLDEN
    g = json.load(open(os.path.join(GOLDEN, "messages.json")))
    c = g["committee"]
    lines = ["Q %d" % len(c["keys"])]
    lines += ["%s %d %d %s" % (k, st, len(w), " ".join(str(x) for x in w)) for k, st, w in
              zip(c["keys"], c["stakes"], c["workers"])]
    want = ["Q 0"]
    groups = {}
    for case in g["cases"]:
        groups.setdefault((case["gc_round"], json.dumps(case["target"])), []).append(case)
    for (gc, tj), cases in groups.items():
        t = json.loads(tj)
        target = "-" if t is None else t[0] + int(t[1]).to_bytes(8, "little").hex() + t[2]
        lines.append("M %d %d %s" % (len(cases), gc, target))
        lines += [x["msg"] or "-" for x in cases]

        def check(line, cases=cases):
            parts = line.split()
            if parts[:2] != ["M", "0"] or len(parts) != 2 + len(cases):
                return False
            for case, item in zip(cases, parts[2:]):
                code, kind, dg = item.split(",")
                if int(code) != case["code"]:
                    return False
                if case["kind"] >= 0 and case["kind"] != 3 and (int(kind) != case["kind"] or dg != case["digest"]):
                    return False
            return True
        want.append(check)
    return lines, want
