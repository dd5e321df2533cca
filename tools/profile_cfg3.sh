#!/bin/bash
# rocprofv3 passes over the cfg-3 legs alone (leaves, Straus, clean, committee comb): kernel trace,
# SQ counters, FETCH_SIZE, clock.
# Each --pmc pass in its own run (no sys/runtime traces).
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof3_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --wire-certs 0 --e2e-reps 0 --cfg3-certs ${CFG3_CERTS:-30000}"
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
$P --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_sq.log 2>&1
$P --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
$P --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_clk -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_clk.log 2>&1
echo done
