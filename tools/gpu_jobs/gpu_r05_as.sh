tools/gpu_job.sh \
 "r5as_test:600:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5as_bench:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5"
