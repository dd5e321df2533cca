#!/bin/bash
# Interleaved A/B of NWC_MSG_CHUNK (bytes per pipelined chunk of nwc_sanitize_messages from host
# memory) on the config-3 wire leg: device-resident and host-ABI certificates/s.
#   tools/ab_wire_host.sh ROUNDS VALUE...      e.g. tools/ab_wire_host.sh 2 0 33554432 67108864
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 6 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --host-digest-group 0"
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    NWC_MSG_CHUNK=$v timeout -k 10 300 python3 $R/bench.py $ARGS > $R/gpurun_out/abw_last.json 2> $R/gpurun_out/abw_last.err
    python3 -c "
import json
w=json.loads(open('$R/gpurun_out/abw_last.json').read().strip().splitlines()[-1])['configs']['cfg3_wire']
print('NWC_MSG_CHUNK=%-10s device %.2f M certs/s  host ABI %.2f M certs/s  parity=%s' % ('$v', w['certs_per_s']/1e6, w['host_abi_certs_per_s']/1e6, w['parity_ok']))
" | tee -a $R/gpurun_out/ab_wire_host.txt
  done
done
