tools/gpu_job.sh \
 "r5ah_wrec:300:python -u -m pytest tests/test_gpu_wrec.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5ah_stats:500:python -u -m pytest tests/test_gpu_stats.py tests/test_adapter.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5ah_pf1:200:python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5ah_pf0:200:PMX_QUAL_PF=0 python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5ah_pf1b:200:python -u tools/bench_stats.py --metric graded --reps 10" \
 "r5ah_pf0b:200:PMX_QUAL_PF=0 python -u tools/bench_stats.py --metric graded --reps 10"
