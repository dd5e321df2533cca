#!/bin/bash
# A/B of library builds on the config-3 legs (100k certificates x 67 votes: leaves, Straus sub-batches,
# clean, committee comb), interleaved for ROUNDS rounds.   tools/ab_cfg3.sh ROUNDS lib1.so lib2.so ...
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ROUNDS=$1; shift
mkdir -p $R/gpurun_out
ARGS="--steps 4 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --digest-batches 0 --triples 65536"
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    NWC_LIB_PATH=$R/$lib timeout -k 10 240 python3 $R/bench.py $ARGS > $R/gpurun_out/ab3_last.json 2> $R/gpurun_out/ab3_last.err
    python3 -c "
import json
d=json.loads(open('$R/gpurun_out/ab3_last.json').read().strip().splitlines()[-1])['configs']['cfg3']
print('%-34s ' % '$lib' + '  '.join('%s %.1f%s' % (k, v['votes_per_s'] / 1e6, '' if v.get('parity_ok') else ' PARITY-FAIL') for k, v in d.items() if isinstance(v, dict) and 'votes_per_s' in v))
" | tee -a $R/gpurun_out/ab3.txt
  done
done
