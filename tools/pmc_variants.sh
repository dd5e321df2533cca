#!/bin/bash
# Per-wave counters of k_verify for A/B library builds (cfg-2 leg of bench.py), one --pmc pass per
# build and counter set.
#   tools/pmc_variants.sh lib1.so lib2.so ...      -> gpurun_out/pmc_<name>_<set>/ + pmc_variants.txt
# PMC_SETS: ';'-separated counter sets (default: instruction mix, then wait/active cycles, then bytes)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --digest-batches 0"
SETS=${PMC_SETS:-"SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE;SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM SQ_INSTS_LDS;SQ_WAVES FETCH_SIZE;SQ_WAVES WRITE_SIZE"}
IFS=';' read -ra SETARR <<< "$SETS"
for lib in "$@"; do
  name=$(basename $lib .so)
  export NWC_LIB_PATH=$R/$lib
  si=0
  for set in "${SETARR[@]}"; do
    out=$R/gpurun_out/pmc_${name}_$si
    timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $out -o run -- python3 $R/bench.py $ARGS > $out.log 2>&1
    python3 - $out $name <<'PY' | tee -a $R/gpurun_out/pmc_variants.txt
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
    waves = sum(v["SQ_WAVES"] for v in vs) / len(vs)
    names = sorted(n for n in vs[0] if n != "SQ_WAVES")
    cols = "  ".join("%s/wave %.4g" % (n, sum(v[n] for v in vs) / len(vs) / waves) for n in names)
    print("%-10s %-28s waves %6.0f  %s" % (sys.argv[2], k[:28], waves, cols))
PY
    si=$((si + 1))
  done
done
