tools/gpu_job.sh \
 "r5ab_sw_c3:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,589840" \
 "r5ab_sw_c4:400:python -u tools/sweep.py --config C4 --rounds 7 --reps 5 --check --opt flags=16,589840" \
 "r5ab_sw_c2:300:python -u tools/sweep.py --config C2 --rounds 7 --reps 5 --check --opt flags=16,589840"
