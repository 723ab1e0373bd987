tools/gpu_job.sh \
 "r5aj_parity:900:python -u -m pytest tests/test_gpu_configs.py -m gpu -v -s --timeout 600 --timeout-method thread"
