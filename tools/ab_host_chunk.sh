#!/bin/bash
# A/B of the pipelined host path's chunk schedule (nwc_verify_strict_many, config-2 inputs in
# pageable host memory): equal 131,072-equation chunks (growth 1) vs geometric growth (x3).
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p $R/gpurun_out
for r in $(seq 1 ${1:-3}); do
  for g in 1 3; do
    NWC_HOST_CHUNK_GROWTH=$g timeout -k 10 180 python3 $R/tools/host_abi_rate.py --reps 7 > $R/gpurun_out/abh_last.json 2> $R/gpurun_out/abh_last.err
    python3 -c "
import json; d=json.load(open('$R/gpurun_out/abh_last.json'))
print('growth $g  median %.2f M/s  best %.2f M/s  %.3f ms  ok=%s' % (d['verifies_per_s_median']/1e6, d['verifies_per_s_best']/1e6, d['ms_median'], d['all_valid']))
" | tee -a $R/gpurun_out/ab_host_chunk.txt
  done
done
