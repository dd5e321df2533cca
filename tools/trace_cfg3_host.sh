#!/bin/bash
# Timeline of nwc_verify_batch_many from host memory (config 3, launch keys): kernel and
# memory-copy traces of the bench's host_abi_launch_keys leg.
#   bash tools/trace_cfg3_host.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/cfg3_host_trace}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 64 --clock-s 0 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --wire-certs 0 --host-digest-group 0"
cd /tmp && export TMPDIR=/tmp
export NWC_BENCH_CFG3_LEGS=host_abi_launch_keys NWC_HOST_TIMING=1
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT -o run -- python3 $R/bench.py $ARGS > $OUT/bench.json 2> $OUT/bench.err
echo done
