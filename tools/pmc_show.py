#!/usr/bin/env python3
"""Prints per-kernel averages of the counters collected by tools/pmc_quick.sh (development aid)."""
import collections
import csv
import glob
import os
import sys

src = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"]
        if "nwc::" not in n:
            continue
        agg[n.split("(")[0].replace("void ", "")][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = {}
p = os.path.join(src, "trace", "run_kernel_stats.csv")
if os.path.exists(p):
    for r in csv.DictReader(open(p)):
        dur[r["Name"].split("(")[0].replace("void ", "")] = (int(r["Calls"]), float(r["AverageNs"]))
for k, cs in agg.items():
    c = {n: sum(v) / len(v) for n, v in cs.items()}
    calls, ns = dur.get(k, (0, 0.0))
    print("%s  calls=%d avg_ms=%.3f" % (k, calls, ns / 1e6))
    for n in sorted(c):
        print("   %-22s %.4g" % (n, c[n]))
    if c.get("SQ_WAVES") and c.get("SQ_INSTS_VALU"):
        print("   valu/wave=%.0f" % (c["SQ_INSTS_VALU"] / c["SQ_WAVES"]))
    if c.get("GRBM_GUI_ACTIVE") and ns:
        print("   eff_clock_GHz=%.3f" % (c["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9) / 1e9))
