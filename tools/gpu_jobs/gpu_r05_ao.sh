tools/gpu_job.sh \
 "r5ao_test:600:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5ao_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_ao -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2" \
 "r5ao_bench:300:python -u bench.py --steps 20 --warmup 5"
