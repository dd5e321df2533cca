#!/bin/bash
# Sub-batch size sweep of the Straus batch path (k_verify_straus) on config 3 (100k certificates x
# 67 votes, uncached; 1 % and 0 % bad), then one SQ-counter pass at the default size.
# Run through gpurun from the repo root: bash tools/straus_ab.sh [NQ list]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/straus_ab
mkdir -p $OUT
ARGS="--steps 3 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --wire-certs 0 --e2e-reps 0 --cfg3-certs ${CFG3_CERTS:-100000}"
for nq in ${1:-4 8 12 16}; do
  NWC_STRAUS_NQ=$nq timeout -k 10 300 python3 $R/bench.py $ARGS > $OUT/bench_nq$nq.json 2> $OUT/bench_nq$nq.err
  python3 - $OUT/bench_nq$nq.json $nq <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))["configs"]["cfg3"]
print("nq", sys.argv[2], {k: round(v["votes_per_s"] / 1e6, 1) for k, v in d.items() if isinstance(v, dict) and "votes_per_s" in v},
      "parity", all(v.get("parity_ok", True) for v in d.values() if isinstance(v, dict)), flush=True)
EOF
done
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_sq.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
  timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_clk -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_clk.log 2>&1
fi
echo done
