tools/gpu_job.sh \
 "r6ad_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie" \
 "r6ad_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie"
