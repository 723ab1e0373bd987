tools/gpu_job.sh \
 "r5ap_sw15:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,983056" \
 "r5ap_sw15c2:300:python -u tools/sweep.py --config C2 --rounds 7 --reps 5 --check --opt flags=16,983056"
