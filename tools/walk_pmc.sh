#!/bin/bash
# Line accounting of the volume walk by variant (GPU box):
#   tools/walk_pmc.sh <tag> <config> <flags values...>
# One rocprofv3 --pmc pass per counter group and variant (tools/sweep.py with
# a single value), k_walk* kernels only; stops at the first failing pass.
tag="$1"; cfg="$2"; shift 2
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/wpmc_$tag
mkdir -p $out
for v in "$@"; do
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_REGEX:-k_walk}" -f csv -d $out/v${v}_p$i -o run -- \
      python3 tools/sweep.py --config $cfg --rounds 1 --reps 2 --opt flags=$v > $out/v${v}_p$i.log 2>&1
    rc=$?
    echo "variant $v pmc$i [$grp] rc=$rc"
    [ $rc -eq 0 ] || exit 3
  done
done
echo walk_pmc done
