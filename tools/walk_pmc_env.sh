#!/bin/bash
# PMC rows of the FRESH step by layout switch (GPU box), the r05 verdict's
# item 5 ("the PMC row for each attempt"):
#   tools/walk_pmc_env.sh <tag> <name>=<ENV=VAL[,ENV=VAL]> ...
# e.g. default= compact=PMX_WALK_RECORDS=compact owner=PMX_HINT_SAMPLE_ORDER=2
# One rocprofv3 --pmc pass per counter group and variant over a short
# bench.py run (C3, FRESH steps), the step's kernels only; stops at the
# first failing pass.  Summarise with tools/pmc_ab_summary.py.
tag="$1"; shift
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/wpmce_$tag
mkdir -p $out
i=0
for spec in "$@"; do
  i=$((i+1))
  name="${spec%%=*}"; envs="${spec#*=}"
  vars=()
  [ -n "$envs" ] && IFS=',' read -r -a vars <<< "$envs"
  echo "variant $i: $name [${vars[*]}]" >> $out/variants.txt
  timeout -k 10 240 env "${vars[@]}" python3 -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 \
    > $out/v${i}_time.json 2> $out/v${i}_time.err || { echo "time $name failed"; exit 2; }
  p=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES"; do
    p=$((p+1))
    env "${vars[@]}" timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_REGEX:-k_}" -f csv \
      -d $out/v${i}_p$p -o run -- python3 bench.py --no-cpu --no-pcie --no-seq --steps 3 --warmup 1 \
      > $out/v${i}_p$p.log 2>&1
    rc=$?
    echo "variant $name pmc$p [$grp] rc=$rc"
    [ $rc -eq 0 ] || exit 3
  done
done
echo walk_pmc_env done
