#!/bin/bash
# rocprofv3 collection for the statistics kernels (run on the GPU box).
#   tools/profile_stats.sh <tag> [bench_stats args...]
# Kernel trace + stats, then one --pmc pass per counter group restricted to the
# k_qual / k_prilen kernels, each under its own hard time limit; stops at the
# first pass that does not exit cleanly.
tag="$1"; shift
args="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/pstats_$tag
mkdir -p $out
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- \
  python3 tools/bench_stats.py $args > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 2; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
  "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "k_qual|k_prilen|k_pb_" -f csv -d $out/pmc$i -o run -- \
    python3 tools/bench_stats.py --reps 2 $args > $out/pmc$i.log 2>&1
  rc=$?
  echo "pmc$i [$grp] rc=$rc"
  [ $rc -eq 0 ] || exit 3
done
echo profile done
