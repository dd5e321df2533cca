#!/bin/bash
# Timeline of nwc_verify_strict_many from host memory (config-2 inputs): kernel and memory-copy
# traces of tools/host_abi_rate.py, one directory per variant ("NAME:ENV ..." args).
#   bash tools/trace_strict_host.sh "paired:NWC_HOST_PAIR=1" ...  ->  gpurun_out/strict_trace_NAME/
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  OUT=$R/gpurun_out/strict_trace_$name
  mkdir -p $OUT
  for kv in $envs; do export "$kv"; done
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 $R/tools/host_abi_rate.py --reps 3 > $OUT/rate.json 2> $OUT/rate.err
  for kv in $envs; do unset "${kv%%=*}"; done
  python3 $R/tools/strict_trace_timeline.py $OUT > $OUT/timeline.txt
done
echo done
