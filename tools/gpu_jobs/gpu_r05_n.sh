tools/gpu_job.sh \
 "r5n_test:200:python -u -m pytest tests/test_gpu_wrec.py -m gpu -x -v --timeout 180 --timeout-method thread" \
 "r5n_b_app:300:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5n_b_app2:300:PMX_HINT_SAMPLE_ORDER=2 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5n_b_lex:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5n_b_lex2:200:PMX_HINT_SAMPLE_ORDER=2 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5n_sw_lex:300:python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --check --opt flags=16,393232" \
 "r5n_sw_app:300:python -u tools/sweep.py --config C3 --numbering appended --rounds 5 --reps 5 --check --opt flags=16,1179664"
