#!/bin/bash
# Interleaved A/B of environment variants on the config-3 wire leg (nwc_dev_sanitize_messages
# device-resident and nwc_sanitize_messages from host memory): certificates/s and parity.
#   bash tools/ab_wire_env.sh ROUNDS "name:ENV=V ..." ...  ->  gpurun_out/ab_wire_env.txt
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 6 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --host-digest-group 0 --clock-s 0"
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs NWC_HOST_TIMING=1 timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abwe_last.json 2> $R/gpurun_out/abwe_last.err
    grep "nwc sanitize:" $R/gpurun_out/abwe_last.err | tail -2 >> $R/gpurun_out/ab_wire_env_timing.txt || true
    python3 -c "
import json
w=json.loads(open('$R/gpurun_out/abwe_last.json').read().strip().splitlines()[-1])['configs']['cfg3_wire']
print('%-10s device %.2f M certs/s  host ABI %.2f M certs/s  parity=%s  [%s]' % ('$name', w['certs_per_s']/1e6, w['host_abi_certs_per_s']/1e6, w['parity_ok'], '$envs'))
" | tee -a $R/gpurun_out/ab_wire_env.txt
  done
done
