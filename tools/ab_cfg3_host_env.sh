#!/bin/bash
# Interleaved A/B of environment variants on config 3 through nwc_verify_batch_many from pageable
# host memory (the bench's host_abi_launch_keys leg): votes/s and parity.
#   bash tools/ab_cfg3_host_env.sh ROUNDS "name:ENV=V ..." ...  ->  gpurun_out/ab_cfg3_host.txt
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 64 --clock-s 0 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --wire-certs 0 --host-digest-group 0"
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs NWC_BENCH_CFG3_LEGS=host_abi_launch_keys NWC_HOST_TIMING=1 timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abc3_last.json 2> $R/gpurun_out/abc3_last.err
    grep "nwc host call" $R/gpurun_out/abc3_last.err | tail -1 >> $R/gpurun_out/ab_cfg3_host_timing.txt || true
    python3 -c "
import json
c=json.loads(open('$R/gpurun_out/abc3_last.json').read().strip().splitlines()[-1])['configs']['cfg3']['host_abi_launch_keys']
print('%-8s %.1f M votes/s  %.2f ms  parity=%s  [%s]' % ('$name', c['votes_per_s']/1e6, c['ms_per_call'], c['parity_ok'], '$envs'))
" | tee -a $R/gpurun_out/ab_cfg3_host.txt
  done
done
