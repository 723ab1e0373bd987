tools/gpu_job.sh \
 "r5d_tests:600:python -u -m pytest tests/test_gpu_stats.py tests/test_adapter.py -m gpu -v --timeout 120 --timeout-method thread" \
 "r5d_sweep_c3:600:python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --check --opt flags=16,851984,917520,983056"
