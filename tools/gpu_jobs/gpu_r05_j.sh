tools/gpu_job.sh \
 "r5j_test:300:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5j_sw_app:400:python -u tools/sweep.py --config C3 --numbering appended --rounds 5 --reps 5 --check --opt flags=16,1114128,393232" \
 "r5j_sw_lex:400:python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --check --opt flags=16,1114128" \
 "r5j_b_lex:300:python -u bench.py --steps 20 --warmup 5" \
 "r5j_b_app:300:python -u bench.py --steps 20 --warmup 5 --numbering appended"
