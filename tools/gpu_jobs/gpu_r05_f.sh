tools/gpu_job.sh \
 "r5f_tests:600:python -u -m pytest tests/test_gpu_stats.py -m gpu -v --timeout 120 --timeout-method thread" \
 "r5f_pmc:1000:PMC_REGEX='k_walk|k_hint|k_bg_derive' bash tools/walk_pmc.sh r5_ab C3 16 851984 917520 983056"
