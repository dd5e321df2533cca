#!/bin/bash
# Counters of the message pipeline's kernels on the device-resident config-3 wire leg (20k
# certificates): kernel trace, then one SQ pass (VALU / SALU / LDS / memory instructions, busy and
# waiting cycles) -- is k_parse_messages issue-bound or waiting?
#   tools/profile_wire_dev.sh OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/wire_dev}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 4 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --host-digest-group 0 --clock-s 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- python3 $R/bench.py $ARGS > $OUT/pmc.json 2> $OUT/pmc.err
echo done
