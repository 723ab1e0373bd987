tools/gpu_job.sh \
 "r6ae_q4:300:python -u bench.py --config C4 --no-cpu --no-pcie --no-seq" \
 "r6ae_q8:300:GPU_MAX_HW_QUEUES=8 python -u bench.py --config C4 --no-cpu --no-pcie --no-seq"
