#!/bin/bash
# The VALU breakdown of k_prilen (r05 verdict item 6): the default iso kernel
# and its measurement variants (PMX_PRILEN_EXP=1 no length, 2 no shell
# rotation, 3 neither; results wrong by design), each with its own
# SQ_INSTS_VALU / SQ_WAVES pass and the bench's own timing.
#   tools/prilen_breakdown.sh <tag> [bench_stats args...]
tag="$1"; shift
args="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prilen_$tag
mkdir -p $out
for x in ${PRILEN_VARIANTS:-0 1 2 3 4}; do
  PMX_EXPERIMENTS=1 PMX_PRILEN_EXP=$x timeout -k 10 200 python3 tools/bench_stats.py --reps 5 $args \
    > $out/time_x$x.json 2> $out/time_x$x.err || { echo "time x$x failed"; exit 2; }
  PMX_EXPERIMENTS=1 PMX_PRILEN_EXP=$x timeout -s KILL 150 rocprofv3 --kernel-trace \
    --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY \
    --kernel-include-regex "k_prilen" -f csv -d $out/pmc_x$x -o run -- \
    python3 tools/bench_stats.py --reps 1 $args > $out/pmc_x$x.log 2>&1
  rc=$?
  echo "x$x pmc rc=$rc"
  [ $rc -eq 0 ] || exit 3
done
echo breakdown done
