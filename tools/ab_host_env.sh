#!/bin/bash
# Interleaved A/B of a libnwc environment switch on the host-buffer legs (config 2 through
# nwc_verify_strict_many, config 3 through nwc_verify_batch_many).
#   tools/ab_host_env.sh ROUNDS VAR VALUE_A VALUE_B      e.g. tools/ab_host_env.sh 3 NWC_HOST_STAGING 1 0
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; VAR=$2; A=$3; B=$4
mkdir -p $R/gpurun_out
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --wire-certs 0 --cfg5-total 0 --digest-batches 0 --host-digest-group 0 --e2e-reps 3"
for r in $(seq 1 $ROUNDS); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abe_last.json 2> $R/gpurun_out/abe_last.err
    python3 -c "
import json
d=json.loads(open('$R/gpurun_out/abe_last.json').read().strip().splitlines()[-1])['configs']
h=d['cfg3']['host_abi_launch_keys']
print('$VAR=%s  cfg2 host %.1f M/s  cfg3 host %.1f M votes/s (%.1f ms)  ok=%s/%s' % ('$v', d['cfg2_host_abi']['verifies_per_s']/1e6, h['votes_per_s']/1e6, h['ms_per_call'], d['cfg2_host_abi']['verdicts_ok'], h['parity_ok']))
" | tee -a $R/gpurun_out/ab_host_env.txt
  done
done
