#!/bin/bash
# Round-6 rocprofv3 evidence (run through gpurun from the repo root): one kernel trace and three PMC
# passes (SQ + GRBM clock, FETCH_SIZE, WRITE_SIZE -- each pass its own run, --pmc alone) for each
# workload whose number the bench line reports:
#   head  : config 2 verify (k_verify) + config 4 digest (k_sha512_digest32_sched)
#   c3lk  : config 3, launch keys (k_verify_comb; the production batch-leaf path)
#   c3dk  : config 3, dalek's batch semantics with launch keys (k_verify_comb + k_vote_resolve)
#   c3msm : config 3 clean, Pippenger groups without keys (k_verify_msm)
#   c5    : config 5, 64M mixed signatures (k_verify over 16M launches)
# The non-headline runs shrink the headline leg to 64 triples (the cold kernel, not k_verify), so
# each kernel's averages are its own workload's.
#   bash tools/profile_r06.sh [only-tags...]  ->  gpurun_out/prof6_<tag>/{trace,pmc_sq,pmc_fetch,pmc_write}
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P="timeout -k 10 300 rocprofv3"
SMALL="--triples 64 --clock-s 0 --digest-batches 0 --cpu-budget 0 --cfg1-calls 0 --wire-certs 0 --e2e-reps 0"
run_tag() {
  local tag=$1; shift
  local OUT=$R/gpurun_out/prof6_$tag
  mkdir -p $OUT
  (cd $R && python3 -c "from narwhal_amd import build; print(build.embedded_id())") > $OUT/build_id.txt
  echo "[profile] $tag: $*"
  $P --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py "$@" > $OUT/trace.log 2>&1
  $P --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_sq -o run -- python3 $R/bench.py "$@" > $OUT/pmc_sq.log 2>&1
  $P --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/bench.py "$@" > $OUT/pmc_fetch.log 2>&1
  $P --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/bench.py "$@" > $OUT/pmc_write.log 2>&1
}
want() { [ $# -eq 0 ] || [[ " $ONLY " == *" $1 "* ]]; }
ONLY="$*"
if [ -z "$ONLY" ] || want head; then
  run_tag head --steps 5 --warmup 1 --cpu-budget 0 --cfg1-calls 0 --cfg3-certs 0 --wire-certs 0 --cfg5-total 0 --e2e-reps 0 --clock-s 0
fi
if [ -z "$ONLY" ] || want c3lk; then
  export NWC_BENCH_CFG3_LEGS=launch_keys
  run_tag c3lk --steps 8 --warmup 1 $SMALL --cfg5-total 0 --cfg3-certs 100000
fi
if [ -z "$ONLY" ] || want c3dk; then
  export NWC_BENCH_CFG3_LEGS=dalek_launch_keys
  run_tag c3dk --steps 8 --warmup 1 $SMALL --cfg5-total 0 --cfg3-certs 100000
fi
if [ -z "$ONLY" ] || want c3msm; then
  export NWC_BENCH_CFG3_LEGS=clean_no_cache_msm
  run_tag c3msm --steps 8 --warmup 1 $SMALL --cfg5-total 0 --cfg3-certs 100000
fi
unset NWC_BENCH_CFG3_LEGS
if [ -z "$ONLY" ] || want c5; then
  run_tag c5 --steps 2 --warmup 1 $SMALL --cfg3-certs 0 --cfg5-total 67108864
fi
echo done
