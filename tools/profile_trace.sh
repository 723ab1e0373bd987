#!/bin/bash
# rocprofv3 kernel trace + stats only (no counters) of the bench workload.
#   tools/profile_trace.sh <tag> [bench args...]
tag="$1"; shift
args="$@"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
out=gpurun_out/prof_$tag
mkdir -p $out
timeout -k 10 280 rocprofv3 --kernel-trace --stats -f csv -d $out/trace -o run -- \
  python3 bench.py --no-cpu --no-pcie $args > $out/trace.log 2>&1 || { echo "trace failed rc=$?"; exit 2; }
echo trace done
