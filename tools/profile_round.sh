#!/bin/bash
# Collects the round's rocprofv3 evidence on the GPU box (run through gpurun from the repo root).
# Headline passes run bench.py with only the cfg-2 verify leg and the cfg-4 digest leg, so the
# per-kernel averages are those of the headline launches (cfg-1/cfg-3 legs launch k_verify with
# other sizes and would mix into its average).
#   trace   : kernel trace + stats (durations)                      -> prof_<tag>/trace
#   pmc_sq  : SQ counters (VALU instructions, waves, cycle buckets)  -> prof_<tag>/pmc_sq
#   pmc_fetch / pmc_write : TCC FETCH_SIZE / WRITE_SIZE (HBM bytes)  -> prof_<tag>/pmc_fetch, pmc_write
#   pmc_clk : GRBM_GUI_ACTIVE (effective clock)                      -> prof_<tag>/pmc_clk
#   trace_cfg3 : kernel trace of the cfg-3 (committee) leg alone     -> prof_<tag>/trace_cfg3
# Every PMC pass uses --pmc alone (no sys/runtime traces), each in its own run.
set -e
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
# the library these passes profile (narwhal_amd/build.py embeds a hash of its sources)
(cd $R && python3 -c "from narwhal_amd import build; print(build.embedded_id())") > $OUT/build_id.txt
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 5 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0"
P="timeout -k 10 240 rocprofv3"
$P --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py $ARGS > $OUT/trace.log 2>&1
$P --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_sq.log 2>&1
$P --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_fetch.log 2>&1
$P --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_write.log 2>&1
$P --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_clk -o run -- python3 $R/bench.py $ARGS > $OUT/pmc_clk.log 2>&1
$P --kernel-trace --stats --output-format csv -d $OUT/trace_cfg3 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --triples 65536 --digest-batches 0 --cfg5-total 0 --e2e-reps 0 > $OUT/trace_cfg3.log 2>&1
# instruction-rate microbenchmarks (the VOP3 4-cycle issue rate the roofline quotes beside the
# guide's 2-cycle peak), built in-tree by `make -C tools/microbench` / hipcc before the call
mkdir -p $OUT/microbench
for mb in int_rates sha_ops lattice_cost; do
  if [ -x $R/tools/microbench/$mb ]; then timeout -k 10 120 $R/tools/microbench/$mb > $OUT/microbench/$mb.txt 2>&1; fi
done
echo done
