#!/bin/bash
# SQ_INSTS_VALU / SQ_WAVES / SQ_BUSY_CYCLES of k_verify_msm per library (the phase-cut builds of
# tools/msm_phases.sh), clean config-3 MSM leg, skip policy off: the instruction split by phase.
#   tools/msm_phases_pmc.sh LIB...
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/msm_phases_pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export NWC_BENCH_CFG3_LEGS=clean_no_cache_msm NWC_MSM_ADAPT=0
ARGS="--steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --wire-certs 0 --clock-s 0 --host-digest-group 0"
for v in "$@"; do
  n=$(basename $v .so)
  NWC_LIB_PATH=$R/$v timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/$n -o run -- python3 $R/bench.py $ARGS > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "
import csv, collections
d = collections.defaultdict(float); n = 0
for x in csv.DictReader(open('$OUT/$n/run_counter_collection.csv')):
    if 'k_verify_msm' in x['Kernel_Name']:
        d[x['Counter_Name']] += float(x['Counter_Value']); n += 1
disp = n / 3
print('$n', 'dispatches %.0f' % disp, ' '.join('%s %.3g' % (k, v / disp) for k, v in sorted(d.items())))
"
done
