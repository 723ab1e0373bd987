tools/gpu_job.sh \
 "r5t_test:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_edge_cases.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5t_lex:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5t_lex2:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5t_c2:300:python -u bench.py --config C2 --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5t_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_t -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2"
