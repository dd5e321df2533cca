#!/bin/bash
# Collects the round's rocprofv3 evidence on the GPU box (run through gpurun from the repo root).
#   pass 1: kernel trace + stats (durations)            -> gpurun_out/prof_<tag>/trace
#   pass 2: SQ counters (VALU instructions, waves)       -> gpurun_out/prof_<tag>/pmc_sq
#   pass 3: TCC FETCH_SIZE (HBM read bytes, digest leg)  -> gpurun_out/prof_<tag>/pmc_fetch
# PMC passes use --pmc alone (no sys/runtime traces), each in its own run.
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --cpu-budget 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
echo done
