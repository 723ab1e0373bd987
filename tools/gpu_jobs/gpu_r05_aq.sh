tools/gpu_job.sh \
 "r5aq_b1:200:python -u bench.py --no-cpu --no-pcie --steps 50 --warmup 5" \
 "r5aq_b2:200:python -u bench.py --no-cpu --no-pcie --steps 50 --warmup 5" \
 "r5aq_b3:200:python -u bench.py --no-cpu --no-pcie --steps 50 --warmup 5" \
 "r5aq_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie --steps 50 --warmup 5" \
 "r5aq_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie --steps 50 --warmup 5"
