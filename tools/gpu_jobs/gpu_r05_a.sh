tools/gpu_job.sh \
 "r5a_tests:600:python -u -m pytest tests/test_gpu_edge_cases.py tests/test_adapter.py tests/test_gpu_stats.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread"
