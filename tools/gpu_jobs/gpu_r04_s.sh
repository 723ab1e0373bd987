set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/c2_prof -o run -- python3 bench.py --config C2 --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/c2_prof.log 2>&1
