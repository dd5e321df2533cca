#!/bin/bash
# Interleaved A/B of library builds on config-1 latency (tools/lat_cfg1.py: the reference's 3-vote
# certificate, committee cached, host ABI).   tools/ab_cfg1.sh ROUNDS CALLS lib1.so lib2.so ...
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; CALLS=$2; shift 2
mkdir -p $R/gpurun_out
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    NWC_LIB_PATH=$R/$lib timeout -k 10 120 python3 $R/tools/lat_cfg1.py $CALLS > $R/gpurun_out/abc_last.json 2> $R/gpurun_out/abc_last.err
    python3 -c "
import json
d=json.loads(open('$R/gpurun_out/abc_last.json').read().strip().splitlines()[-1])
print('%-34s p50 %.1f us  p99 %.1f us' % ('$lib', d['p50_us'], d['p99_us']))
" | tee -a $R/gpurun_out/ab_cfg1.txt
  done
done
