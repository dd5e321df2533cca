#!/bin/bash
# tools/probes/copy_trace_probe.sh OUTDIR: the copy probe of each mode under rocprofv3's
# memory-copy trace; one line per mode with the tracer's undelivered-completion warning, if any.
# Extra environment (e.g. HSA_ENABLE_SDMA=0: every copy as a blit kernel) applies to all modes.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
OUT=${1:-$R/gpurun_out/copy_probe}
mkdir -p "$OUT" && OUT=$(cd "$OUT" && pwd)
cd /tmp && export TMPDIR=/tmp
for m in pageable_d2h pageable_h2d pinned_d2h pinned_h2d big_pinned_h2d coherent_d2h coherent_h2d; do
  timeout -k 10 120 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $OUT/$m -o run -- $R/tools/probes/build/copy_trace_probe $m > $OUT/$m.out 2> $OUT/$m.err
  w=$(grep -o "waiting for [0-9]* completion callbacks" $OUT/$m.err || true)
  echo "$m: $(cat $OUT/$m.out) | tracer: ${w:-no undelivered completions}"
done
