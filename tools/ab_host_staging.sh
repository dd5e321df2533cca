#!/bin/bash
# Interleaved A/B of NWC_HOST_STAGING (pinned-stage copies vs hipMemcpyAsync from pageable
# memory) on the host-buffer legs: config 2 through nwc_verify_strict_many and config 3 through
# nwc_verify_batch_many.   tools/ab_host_staging.sh ROUNDS
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --wire-certs 0 --cfg5-total 0 --digest-batches 0 --host-digest-group 0 --e2e-reps 3"
for r in $(seq 1 ${1:-3}); do
  for st in 1 0; do
    NWC_HOST_STAGING=$st timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abh_last.json 2> $R/gpurun_out/abh_last.err
    python3 -c "
import json
d=json.loads(open('$R/gpurun_out/abh_last.json').read().strip().splitlines()[-1])['configs']
h=d['cfg3']['host_abi_launch_keys']
print('staging=%s  cfg2 host %.1f M/s  cfg3 host %.1f M votes/s (%.1f ms)  ok=%s/%s' % ('$st', d['cfg2_host_abi']['verifies_per_s']/1e6, h['votes_per_s']/1e6, h['ms_per_call'], d['cfg2_host_abi']['verdicts_ok'], h['parity_ok']))
" | tee -a $R/gpurun_out/ab_host_staging.txt
  done
done
