tools/gpu_job.sh \
 "r5i_test:300:python -u -m pytest tests/test_gpu_stats.py -m gpu -x -v -k buckets --timeout 280 --timeout-method thread" \
 "r5i_rot:200:python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5i_pb:200:PMX_PRILEN_BUCKETS=1 python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5i_rot2:200:python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5i_pb2:200:PMX_PRILEN_BUCKETS=1 python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5i_prof_rot:500:bash tools/profile_stats.sh r5_rot --metric graded" \
 "r5i_prof_pb:500:PMX_PRILEN_BUCKETS=1 bash tools/profile_stats.sh r5_pb --metric graded"
