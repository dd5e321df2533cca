#!/bin/bash
# rocprofv3 evidence of BASELINE config 3's kernels (run through gpurun from the repo root):
# bench.py with only the config-3 legs -- per-vote leaves (k_verify), Straus sub-batches
# (k_verify_straus), launch keys and the committee cache (k_verify_comb) -- under a kernel trace
# and one PMC pass per counter group (SQ, FETCH_SIZE, WRITE_SIZE, GRBM clock), each in its own run.
#   bash tools/profile_cfg3.sh <tag>   ->  gpurun_out/prof_cfg3_<tag>/{trace,pmc_sq,pmc_fetch,pmc_write,pmc_clk}
set -e
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_cfg3_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --wire-certs 0 --e2e-reps 0 --cfg3-certs ${CFG3_CERTS:-100000}"
P="timeout -k 10 300 rocprofv3"
$P --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
$P --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_sq.log 2>&1
$P --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
$P --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_write.log 2>&1
$P --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_clk -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_clk.log 2>&1
echo done
