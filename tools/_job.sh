tools/gpu_job.sh \
 "dbg:200:md5sum parmmg_amd/libpmx_transfer.so; PMX_EXP_PRILEN=2 python -u tools/bench_stats.py --n 60 --metric graded --reps 2" \
 "tests:900:python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread" \
 "bench:300:python bench.py --no-cpu --no-pcie --steps 20 --warmup 3" \
 "pb1024:150:PMX_EXP_PRILEN_BLOCKS=1024 python -u tools/bench_stats.py --metric graded --reps 10" \
 "pb2048:150:PMX_EXP_PRILEN_BLOCKS=2048 python -u tools/bench_stats.py --metric graded --reps 10" \
 "pe1:150:PMX_EXP_PRILEN=1 python -u tools/bench_stats.py --metric graded --reps 10" \
 "pe2:150:PMX_EXP_PRILEN=2 python -u tools/bench_stats.py --metric graded --reps 10"
