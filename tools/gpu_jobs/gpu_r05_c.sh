tools/gpu_job.sh \
 "r5c_tests:700:python -u -m pytest tests/test_gpu_stats.py tests/test_adapter.py -m gpu -v --timeout 120 --timeout-method thread"
