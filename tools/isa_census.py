#!/usr/bin/env python3
"""ISA census of the hot kernels: VALU instructions by issue class, static counts x trip counts.

On gfx950 a wave64 VALU instruction issues over 2 cycles of its SIMD in the VOP1 / VOP2 / VOPC
encodings (printed with an _e32, _dpp or _sdwa suffix) and over 4 cycles in the VOP3 / VOP3P
encodings (no suffix, or _e64): DESIGN.md §3 (tools/microbench/int_rates.hip).  A kernel's true
issue fraction therefore prices each instruction at its own class:

    frac_issue = sum over classes (dynamic wave-instructions x cycles) / (4 SIMDs x 256 CUs x clock x time)

The dynamic class counts come from the kernel's assembly (hipcc -S of nwc_api.hip): the kernel
and the functions it calls are cut into basic blocks, natural loops are found from the back edges,
and every loop's trip count per invocation comes from TRIPS below -- the loop structure of the
source (window counts, doublings per window, exponentiation chains), matched to the loops by
their order and size.  The census is calibrated against the measured SQ_INSTS_VALU per lane of
the same build (profiles/<round>/summary.json): the model's total must agree within a few %.

    python tools/isa_census.py [--asm FILE.s] [--out profiles/r05/isa_census.json]

Only the class SHARES enter bench.py (roofline.frac_issue): the instruction total stays the
measured counter.
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

KERNELS = {
    "k_verify": "_ZN3nwc8k_verifyILb1ELb0ELb0ELb0EEEvNS_10VerifyArgsENS_8CombArgsE",
    "k_verify_comb": "_ZN3nwc13k_verify_combENS_10VerifyArgsENS_8CombArgsE",
    "k_verify_straus": "_ZN3nwc15k_verify_strausILb0EEEvNS_10StrausArgsE",
    "k_sha512_digest32_sched": "_ZN3nwc23k_sha512_digest32_schedEPKhPKmS3_mPh",
}


def cycles(mn: str) -> int:
    """Issue cycles of one wave64 VALU instruction of mnemonic `mn` on gfx950."""
    if mn.endswith("_e32") or mn.endswith("_dpp") or mn.endswith("_sdwa"):
        return 2
    return 4


def gen_asm(path):
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(ROOT, "narwhal_amd", "csrc")]
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++20", "-fPIC",
                    "--offload-device-only", "-S", *inc, "-o", path,
                    os.path.join(ROOT, "narwhal_amd", "csrc", "nwc_api.hip")], check=True)


def functions(asm: str):
    """name -> list of (label, [lines]) basic blocks, in program order."""
    out = {}
    for m in re.finditer(r"^([A-Za-z_][\w.$]*):[^\n]*\n(.*?)^\.Lfunc_end\d+:", asm, re.S | re.M):
        name, body = m.group(1), m.group(2)
        blocks, cur, lines = [], name, []
        for line in body.splitlines():
            lm = re.match(r"^(\.LBB\d+_\d+):", line)
            if lm:
                blocks.append((cur, lines))
                cur, lines = lm.group(1), []
            else:
                lines.append(line)
        blocks.append((cur, lines))
        out[name] = blocks
    return out


def block_info(lines):
    valu = defaultdict(int)
    succ, calls = [], []
    for line in lines:
        t = line.strip()
        if not t or t.startswith(";") or t.startswith("."):
            continue
        mn = t.split()[0]
        if mn.startswith("v_"):
            valu[cycles(mn)] += 1
        bm = re.match(r"s_(cbranch_\w+|branch)\s+(\.LBB\d+_\d+)", t)
        if bm:
            succ.append((bm.group(1), bm.group(2)))
        cm = re.search(r"([A-Za-z_][\w.$]*)@rel32@lo", t)
        if cm:
            calls.append(cm.group(1))
    return dict(valu), succ, calls


def loops(blocks):
    """Natural loops approximated by back edges: a branch from block j to an earlier label i makes
    blocks [i, j] a loop (nested loops are contained intervals)."""
    index = {lab: k for k, (lab, _) in enumerate(blocks)}
    out = []
    for j, (lab, lines) in enumerate(blocks):
        _, succ, _ = block_info(lines)
        for kind, tgt in succ:
            i = index.get(tgt)
            if i is not None and i <= j:
                out.append((i, j))
    return sorted(set(out))


def census(asm_path, trips):
    asm = open(asm_path).read()
    fns = functions(asm)
    res = {}
    for short, mangled in KERNELS.items():
        if mangled not in fns:
            res[short] = {"error": "kernel not found in the assembly"}
            continue
        t = trips.get(short, {})

        def count(fname, depth=0):
            """Dynamic class counts of one invocation of fname (trip-weighted)."""
            blocks = fns.get(fname)
            if blocks is None or depth > 6:
                return defaultdict(float), []
            lp = loops(blocks)
            # trips keyed by the loop's static VALU size ("size", or "size#k" for the k-th loop of
            # that size in program order): stable across builds that leave the loop bodies alone
            ftrips = t.get(fname if fname != mangled else "kernel", {})
            mult = [1.0] * len(blocks)
            desc = []
            seen = defaultdict(int)
            for k, (i, j) in enumerate(lp):
                size = sum(sum(block_info(blocks[b][1])[0].values()) for b in range(i, j + 1))
                key = "%d#%d" % (size, seen[size])
                seen[size] += 1
                tr = float(ftrips.get(key, ftrips.get(str(size), 1.0)))
                for b in range(i, j + 1):
                    mult[b] *= tr
                desc.append({"loop": k, "key": key, "blocks": [i, j], "static_valu": size, "trips": tr})
            tot = defaultdict(float)
            only = t.get("only_blocks") if fname == mangled else None
            for b, (lab, lines) in enumerate(blocks):
                if only and not only[0] <= b <= only[1]:
                    continue
                valu, _, calls = block_info(lines)
                for c, v in valu.items():
                    tot[c] += v * mult[b]
                for callee in calls:
                    sub, _ = count(callee, depth + 1)
                    cm = float(t.get("call_mult", {}).get(callee, 1.0))   # invocations per call site pass
                    for c, v in sub.items():
                        tot[c] += v * mult[b] * cm
            return tot, desc

        tot, desc = count(mangled)
        n = sum(tot.values())
        cal = t.get("calibration", {})
        model_unit = n / cal.get("units_per_invocation", 1) if n else None
        res[short] = {"mangled": mangled, "valu_per_lane_model": n, "by_cycles": {str(k): v for k, v in tot.items()},
                      "valu_per_unit_model": model_unit, "valu_per_unit_measured": cal.get("measured_valu_per_unit"),
                      "model_over_measured": model_unit / cal["measured_valu_per_unit"] if cal.get("measured_valu_per_unit") and model_unit else None,
                      "calibration_source": cal.get("source"),
                      "share_4cycle": tot.get(4, 0.0) / n if n else None,
                      "avg_issue_cycles": sum(k * v for k, v in tot.items()) / n if n else None,
                      "loops": desc}
    return res


# Trip counts per invocation of each natural loop, in program order of its back edge, for the
# kernel body ("kernel") and the functions it calls.  Filled from the source's loop structure; a
# loop missing from a list runs once.  tools/isa_census.py --show lists the loops it finds.
TRIPS = os.path.join(ROOT, "tools", "census_trips.json")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--asm")
    ap.add_argument("--out")
    ap.add_argument("--show", action="store_true")
    a = ap.parse_args()
    asm = a.asm
    if not asm:
        asm = os.path.join(tempfile.mkdtemp(), "nwc.s")
        gen_asm(asm)
    trips = json.load(open(TRIPS)) if os.path.exists(TRIPS) else {}
    res = census(asm, trips)
    if a.show:
        for k, v in res.items():
            print(k, {x: v[x] for x in ("valu_per_lane_model", "share_4cycle", "avg_issue_cycles") if x in v})
            for l in v.get("loops", []):
                print("   ", l)
    if a.out:
        json.dump({"method": __doc__.strip().splitlines()[0], "trips": trips, "kernels": res}, open(a.out, "w"), indent=1)
    print(json.dumps({k: {x: v.get(x) for x in ("model_over_measured", "share_4cycle", "avg_issue_cycles")}
                      for k, v in res.items()}))


if __name__ == "__main__":
    main()
