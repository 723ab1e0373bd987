tools/gpu_job.sh \
 "r5b_tests:700:python -u -m pytest tests/test_gpu_edge_cases.py tests/test_adapter.py tests/test_gpu_stats.py -m gpu -v --timeout 120 --timeout-method thread"
