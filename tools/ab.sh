#!/bin/bash
# A/B of library builds on one GPU box: the cfg-2 headline leg of bench.py, alternating the
# builds for ROUNDS rounds (the box's clock drifts; only interleaved pairs decide a change).
#   tools/ab.sh ROUNDS lib1.so lib2.so ...        (paths relative to the repo root)
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 10 --warmup 2 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --digest-batches 0 ${AB_ARGS:-}"
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    NWC_LIB_PATH=$R/$lib timeout -k 10 180 python3 $R/bench.py $ARGS > $R/gpurun_out/ab_last.json 2> $R/gpurun_out/ab_last.err
    python3 -c "
import json,sys
d=json.loads(open('$R/gpurun_out/ab_last.json').read().strip().splitlines()[-1])
print('%-40s %8.2f M/s  step %.3f ms  kernel %.3f ms  ok=%s' % ('$lib', d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms'], d['config'].get('verdicts_ok')))
" | tee -a $R/gpurun_out/ab.txt
  done
done
