#!/bin/bash
# k_verify_msm kernel time per variant (phase-cut builds made by tools/build_variant.sh with
# -DNWC_MSM_CUT=1 / 2), clean config-3 MSM leg, skip policy off; VGPRs and scratch per lane too.
#   tools/msm_phases.sh [ROUNDS] [LIB...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/msm_phases
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export NWC_BENCH_CFG3_LEGS=clean_no_cache_msm NWC_MSM_ADAPT=0
ARGS="--steps 4 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 --wire-certs 0 --clock-s 0 --host-digest-group 0"
ROUNDS=${1:-2}; shift || true
LIBS=${@:-narwhal_amd/libnwc.so narwhal_amd/variants/msm_cut1.so narwhal_amd/variants/msm_cut2.so}
for r in $(seq 1 $ROUNDS); do
for v in $LIBS; do
  n=$(basename $v .so)_$r
  NWC_LIB_PATH=$R/$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 $R/bench.py $ARGS > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "
import csv
for x in csv.DictReader(open('$OUT/$n/run_kernel_stats.csv')):
    if 'msm' in x['Name'] and 'policy' not in x['Name']: print('$n', x['Name'][:24], x['Calls'], '%.3f ms' % (float(x['AverageNs'])/1e6), end=' ')
for x in csv.DictReader(open('$OUT/$n/run_kernel_trace.csv')):
    if 'k_verify_msm' in x['Kernel_Name']: print('vgpr', x['VGPR_Count'], 'agpr', x['Accum_VGPR_Count'], 'scratch', x['Scratch_Size'], 'lds', x['LDS_Block_Size']); break
"
done
done
