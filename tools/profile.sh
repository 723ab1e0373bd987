#!/bin/bash
# rocprofv3 collection for the bench workload (run on the GPU box).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/: kernel trace + stats, then one --pmc pass per
# counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
set -e
tag="$1"; shift
args="$@"
out=gpurun_out/prof_$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 bench.py --no-cpu $args > $out/trace.log 2>&1
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  name=$(echo $grp | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $out/pmc_$name -o run -- python3 bench.py --no-cpu $args > $out/pmc_$name.log 2>&1 || echo "pmc $grp failed rc=$?"
done
echo profile done
