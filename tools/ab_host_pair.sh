#!/bin/bash
# A/B of the strict host pipeline (nwc_verify_strict_many, config-2 inputs in pageable host memory):
# the paired pipeline (two compute streams, halves of the table slots) against the single-stream
# chunks (NWC_HOST_PAIR=0), interleaved; extra variants of the paired schedule as "NAME=ENV ..." args.
#   bash tools/ab_host_pair.sh ROUNDS [variant ...]  ->  gpurun_out/ab_host_pair.txt
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
ROUNDS=${1:-3}; shift || true
VARIANTS=("single:NWC_HOST_PAIR=0" "paired:NWC_HOST_PAIR=1" "$@")
for r in $(seq 1 $ROUNDS); do
  for v in "${VARIANTS[@]}"; do
    name=${v%%:*}; envs=${v#*:}
    env $envs NWC_HOST_TIMING=1 timeout -k 10 180 python3 $R/tools/host_abi_rate.py --reps 7 > $R/gpurun_out/abp_last.json 2> $R/gpurun_out/abp_last.err
    tail -1 $R/gpurun_out/abp_last.err >> $R/gpurun_out/ab_host_pair_timing.txt
    python3 -c "
import json; d=json.load(open('$R/gpurun_out/abp_last.json'))
print('%-10s median %.2f M/s  best %.2f M/s  %.3f ms  ok=%s  [%s]' % ('$name', d['verifies_per_s_median']/1e6, d['verifies_per_s_best']/1e6, d['ms_median'], d['all_valid'], '$envs'))
" | tee -a $R/gpurun_out/ab_host_pair.txt
  done
done
