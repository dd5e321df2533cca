#!/bin/bash
# rocprofv3 of the config-3 batch-equation legs (Straus sub-batches and the Pippenger MSM, clean
# traffic): kernel trace + stats, then one PMC pass (VALU instructions, waves, busy cycles).
#   tools/profile_msm.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/msm_prof}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
export NWC_BENCH_CFG3_LEGS=${NWC_BENCH_CFG3_LEGS:-no_cache_straus,no_cache_msm,clean_no_cache_straus,clean_no_cache_msm}
ARGS="--steps 4 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --wire-certs 0 --clock-s 0 --host-digest-group 0"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/bench_trace.json 2> $OUT/trace.err
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- python3 $R/bench.py $ARGS > $OUT/bench_pmc.json 2> $OUT/pmc.err
echo done
