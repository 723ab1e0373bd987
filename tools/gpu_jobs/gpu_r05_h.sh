tools/gpu_job.sh \
 "r5h_sweep_c3:500:python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --check --opt flags=16,1048592" \
 "r5h_sweep_c2:300:python -u tools/sweep.py --config C2 --rounds 5 --reps 5 --check --opt flags=16,1048592" \
 "r5h_parity:600:python -u -m pytest tests/test_gpu_configs.py -m gpu -x -v -s -k full_size --timeout 500 --timeout-method thread"
