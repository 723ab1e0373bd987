tools/gpu_job.sh \
 "r5v_sw_c3:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,1245200" \
 "r5v_sw_c2:300:python -u tools/sweep.py --config C2 --rounds 7 --reps 5 --check --opt flags=16,1245200" \
 "r5v_sw_c4:300:python -u tools/sweep.py --config C4 --rounds 7 --reps 5 --check --opt flags=16,1245200"
