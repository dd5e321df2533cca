#!/bin/bash
# Quick counter passes for one bench configuration (development aid; the round's committed
# evidence comes from tools/profile_round.sh).  Usage: tools/pmc_quick.sh TAG "<bench args>"
set -e
TAG=$1
ARGS=$2
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcq_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 120 rocprofv3"
$P --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
$P --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM --output-format csv -d $OUT/pmc1 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc1.log 2>&1
$P --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc2 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc2.log 2>&1
$P --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o run -- python3 $R/bench.py $ARGS > $OUT/pmc3.log 2>&1
echo done
