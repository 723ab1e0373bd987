tools/gpu_job.sh \
 "adapter:300:python -u -m pytest tests/test_adapter.py -x -v --timeout 240 --timeout-method thread" \
 "tests:800:python -u -m pytest tests -m gpu -x -q -s --timeout 1100 --timeout-method thread --deselect tests/test_adapter.py" \
 "bench:240:python bench.py --no-cpu --no-pcie --steps 20 --warmup 3" \
 "prof:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r03b -o run -- python3 bench.py --no-cpu --no-pcie --steps 10 --warmup 2"
