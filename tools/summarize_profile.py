#!/usr/bin/env python3
"""Condenses a round's rocprofv3 output (tools/profile_round.sh) into profiles/<tag>/:
kernel_stats.csv (as produced), pmc_*.csv filtered to the nwc:: kernels, and summary.json with
per-kernel average duration, VALU instructions per lane, VALU lane-op rate, FETCH_SIZE bytes.

    python tools/summarize_profile.py gpurun_out/prof_r01 profiles/r01
"""
import collections
import csv
import json
import os
import shutil
import sys

VALU_PEAK = 128 * 256 * 2.4e9  # wave64 VALU issue, 2 cycles/SIMD (MI355X_MICROARCH.md)
VOP3_RATE = 64 * 256 * 2.4e9   # measured 4-cycle VOP3 integer issue


def kname(full):
    """'void nwc::k_verify<true, false>(nwc::VerifyArgs)' -> 'nwc::k_verify<true, false>'; None if not ours."""
    n = full[5:] if full.startswith("void ") else full
    return n.split("(")[0] if n.startswith("nwc::") else None


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    if os.path.exists(os.path.join(src, "build_id.txt")):
        shutil.copy(os.path.join(src, "build_id.txt"), os.path.join(dst, "build_id.txt"))
    c3 = os.path.join(src, "trace_cfg3", "run_kernel_stats.csv")
    if os.path.exists(c3):
        shutil.copy(c3, os.path.join(dst, "kernel_stats_cfg3.csv"))
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    summary = {}
    for name, r in stats.items():
        if kname(name) is None:
            continue
        summary[kname(name)] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                       "min_ns": float(r["MinNs"]), "max_ns": float(r["MaxNs"])}
    for pmc in ("pmc_sq", "pmc_fetch", "pmc_write", "pmc_clk"):
        path = os.path.join(src, pmc, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        rows = [r for r in csv.DictReader(open(path)) if kname(r["Kernel_Name"]) is not None]
        with open(os.path.join(dst, pmc + ".csv"), "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        agg = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in rows:
            agg[kname(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, cs in agg.items():
            d = summary.setdefault(k, {})
            for c, v in cs.items():
                d[c] = sum(v) / len(v)
            d["VGPR"] = int(rows[[kname(r["Kernel_Name"]) for r in rows].index(k)]["VGPR_Count"])
            d["AGPR"] = int(rows[[kname(r["Kernel_Name"]) for r in rows].index(k)]["Accum_VGPR_Count"])
            d["scratch_per_lane"] = int(rows[[kname(r["Kernel_Name"]) for r in rows].index(k)]["Scratch_Size"])
    for k, d in summary.items():
        if "SQ_INSTS_VALU" in d and "avg_ns" in d and d.get("SQ_WAVES"):
            d["valu_insts_per_lane"] = d["SQ_INSTS_VALU"] / d["SQ_WAVES"]
            d["valu_lane_ops_per_s"] = d["SQ_INSTS_VALU"] * 64 / (d["avg_ns"] * 1e-9)
            d["valu_issue_frac"] = d["valu_lane_ops_per_s"] / VALU_PEAK
            d["valu_frac_vop3_rate"] = d["valu_lane_ops_per_s"] / VOP3_RATE
        if "FETCH_SIZE" in d:
            d["fetch_bytes_reported"] = d["FETCH_SIZE"] * 1024
            d["fetch_bytes_x2_gfx950"] = d["FETCH_SIZE"] * 1024 * 2
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            # MI355X_MICROARCH.md "HBM [CDNA4]": FETCH_SIZE (KB) x2 on gfx950 for 16-B/lane reads,
            # WRITE_SIZE (KB) exact for 16-B/lane stores; per launch (counters are per dispatch)
            d["write_bytes"] = d["WRITE_SIZE"] * 1024
            d["hbm_traffic_bytes_per_launch"] = d["fetch_bytes_x2_gfx950"] + d["write_bytes"]
        if "GRBM_GUI_ACTIVE" in d and "avg_ns" in d:
            # GRBM_GUI_ACTIVE comes back summed over the 8 XCD instances
            d["gui_active_clk_ghz_per_xcd"] = d["GRBM_GUI_ACTIVE"] / 8 / d["avg_ns"]
    json.dump(summary, open(os.path.join(dst, "summary.json"), "w"), indent=1)
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
