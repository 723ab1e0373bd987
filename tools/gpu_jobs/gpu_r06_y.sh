tools/gpu_job.sh \
 "r6y_bench:480:python -u bench.py --no-seq"
