#!/bin/bash
# Timeline of nwc_sanitize_messages from host memory (config-3 wire leg): kernel and memory-copy
# traces of the wire bench, for the copy / parse / leaves overlap.
#   tools/trace_wire_host.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/wire_trace}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --host-digest-group 0 --clock-s 0"
cd /tmp && export TMPDIR=/tmp
NWC_HOST_TIMING=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
echo done
