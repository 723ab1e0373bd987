tools/gpu_job.sh \
 "r6k_bench:420:python -u bench.py" \
 "r6k_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie" \
 "r6k_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie"
