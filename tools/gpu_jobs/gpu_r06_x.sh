tools/gpu_job.sh \
 "r6x_bench:480:python -u bench.py --no-seq" \
 "r6x_tr:300:bash tools/profile_trace.sh r6x --steps 3 --warmup 1 --no-seq"
