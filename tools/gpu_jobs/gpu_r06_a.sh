tools/gpu_job.sh \
 "r6a_tests:700:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r6a_bench:400:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r6a_prof:300:bash tools/profile_trace.sh r6a"
