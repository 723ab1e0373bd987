set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_topology.py -m gpu > gpurun_out/t_topo.log 2>&1
PMX_TOPO_MATCH=global timeout -k 10 300 python3 tools/bench_topo.py --n 255 --reps 3 > gpurun_out/topo_global.log 2>&1
timeout -k 10 300 python3 tools/bench_topo.py --n 255 --reps 3 > gpurun_out/topo_lds.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/topo_prof -o run -- python3 tools/bench_topo.py --n 255 --reps 3 > gpurun_out/topo_prof.log 2>&1
