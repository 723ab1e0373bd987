tools/gpu_job.sh \
 "r6c_seq:600:python -u -m pytest tests/test_gpu_seq_surface.py tests/test_gpu_edge_cases.py -x -v -s --timeout 280 --timeout-method thread" \
 "r6c_b0:400:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r6c_b23:300:python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 5 --run-exp 23"
