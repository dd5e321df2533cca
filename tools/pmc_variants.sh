#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES per kernel for A/B library builds (one --pmc pass per build, cfg-2 leg).
#   tools/pmc_variants.sh lib1.so lib2.so ...      -> gpurun_out/pmc_<name>/ + pmc_variants.txt
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --digest-batches 0"
for lib in "$@"; do
  name=$(basename $lib .so)
  export NWC_LIB_PATH=$R/$lib
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_$name -o run -- python3 $R/bench.py $ARGS > $R/gpurun_out/pmc_$name.log 2>&1
  python3 - $R/gpurun_out/pmc_$name $name <<'PY' | tee -a $R/gpurun_out/pmc_variants.txt
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "k_verify" not in k: continue
        acc[(k, row.get("Dispatch_Id"))][row["Counter_Name"]].append(float(row["Counter_Value"]))
per = collections.defaultdict(list)
for (k, d), c in acc.items():
    v = {n: sum(x) for n, x in c.items()}
    if v.get("SQ_WAVES", 0) >= 16000:
        per[k].append(v)
for k, vs in per.items():
    valu = sum(v["SQ_INSTS_VALU"] for v in vs) / len(vs); waves = sum(v["SQ_WAVES"] for v in vs) / len(vs)
    salu = sum(v.get("SQ_INSTS_SALU", 0) for v in vs) / len(vs)
    gui = sum(v.get("GRBM_GUI_ACTIVE", 0) for v in vs) / len(vs)
    print("%-10s %-40s VALU/wave %9.0f  SALU/wave %7.0f  waves %6.0f  GUI_ACTIVE %.4g" % (sys.argv[2], k[:40], valu / waves, salu / waves, waves, gui))
PY
done
