tools/gpu_job.sh \
 "r5s_test:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_wrec.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5s_lex:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5s_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_s -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2"
