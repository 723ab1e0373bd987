#!/bin/bash
# Issue / memory-pipeline counters of the volume walk kernel (GPU box).
#   tools/profile_diag.sh <tag> [bench args...]
# One --pmc pass per group, each under its own hard time limit; the script
# stops at the first pass that does not exit cleanly.
tag="$1"; shift
args="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/diag_$tag
mkdir -p $out
i=0
for grp in \
  "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU" \
  "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU" \
  "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
  "TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
  "SQ_WAVES SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex "k_walk|k_locate_vol|k_hint" -f csv -d $out/pmc$i -o run -- \
    python3 bench.py --no-cpu --steps 3 --warmup 1 $args > $out/pmc$i.log 2>&1
  rc=$?
  echo "pmc$i [$grp] rc=$rc"
  [ $rc -eq 0 ] || exit 3
done
echo diag done
