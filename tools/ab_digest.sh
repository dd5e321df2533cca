#!/bin/bash
# A/B of library builds on the config-4 digest leg (100k x 508,052-B batches resident in HBM),
# alternating the builds for ROUNDS rounds.   tools/ab_digest.sh ROUNDS lib1.so lib2.so ...
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 2 --warmup 1 --triples 65536 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --digest-steps 3"
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    NWC_LIB_PATH=$R/$lib timeout -k 10 240 python3 $R/bench.py $ARGS > $R/gpurun_out/abd_last.json 2> $R/gpurun_out/abd_last.err
    python3 -c "
import json
d=json.loads(open('$R/gpurun_out/abd_last.json').read().strip().splitlines()[-1])['digest']
print('%-40s %8.1f GB/s  kernel %.3f ms  ok=%s' % ('$lib', d['value'], d['kernel_ms'], d['parity_ok']))
" | tee -a $R/gpurun_out/ab_digest.txt
  done
done
