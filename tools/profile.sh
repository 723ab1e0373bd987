#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: kernel trace + stats (csv), then one --pmc
# pass per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on
# gfx950; at most 4 TCC slots per pass).  Each pass has its own time limit and
# the script stops at the first pass that does not exit cleanly.  The bench
# runs without its host-staged legs (--no-pcie): those run the walk beside the
# residency topology build, which would skew the per-launch averages.
tag="$1"; shift
args="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- \
  python3 bench.py --no-cpu --no-pcie $args > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 2; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp -f csv -d $out/pmc$i -o run -- \
    python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 1 $args > $out/pmc$i.log 2>&1
  rc=$?
  echo "pmc$i [$grp] rc=$rc"
  [ $rc -eq 0 ] || exit 3
done
echo profile done
