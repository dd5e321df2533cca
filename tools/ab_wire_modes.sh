#!/bin/bash
# Interleaved A/B of the host sanitize pipeline's environment knobs on the config-3 wire leg: each
# argument is a comma-separated list of VAR=VALUE (empty: the defaults), e.g.
#   tools/ab_wire_modes.sh 2 "" NWC_HOST_STAGING_THREADS=16 NWC_MSG_CHUNK=16777216,NWC_LEAF_ROUNDS=1
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 6 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --host-digest-group 0 --clock-s 0"
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    env ${v//,/ } timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abm_last.json 2> $R/gpurun_out/abm_last.err
    python3 -c "
import json
w=json.loads(open('$R/gpurun_out/abm_last.json').read().strip().splitlines()[-1])['configs']['cfg3_wire']
print('%-60s device %.2f M certs/s  host ABI %.2f M certs/s  parity=%s' % ('${v:-defaults}', w['certs_per_s']/1e6, w['host_abi_certs_per_s']/1e6, w['parity_ok']))
" | tee -a $R/gpurun_out/ab_wire_modes.txt
  done
done
