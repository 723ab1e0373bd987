tools/gpu_job.sh \
 "r5am_shuf:300:python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3 --numbering shuffle"
