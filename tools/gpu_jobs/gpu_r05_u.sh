tools/gpu_job.sh \
 "r5u_ab_cus:400:python -u tools/ab_env.py --config C3 --env PMX_SIDE_CUS=0,8,16,32 --rounds 5 --reps 5" \
 "r5u_ab_cus_c2:300:python -u tools/ab_env.py --config C2 --env PMX_SIDE_CUS=0,8,16 --rounds 5 --reps 5"
