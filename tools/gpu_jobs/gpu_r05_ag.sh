tools/gpu_job.sh \
 "r5ag_test:400:python -u -m pytest tests/test_gpu_wrec.py -m gpu -x -v --timeout 280 --timeout-method thread"
