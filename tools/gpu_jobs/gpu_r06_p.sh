tools/gpu_job.sh \
 "r6p_a0:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6p_a1:200:PMX_STREAM_PRIO=1 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6p_b0:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6p_b1:200:PMX_STREAM_PRIO=1 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6p_c41:200:PMX_STREAM_PRIO=1 python -u bench.py --config C4 --no-cpu --no-pcie --no-seq" \
 "r6p_c21:200:PMX_STREAM_PRIO=1 python -u bench.py --config C2 --no-cpu --no-pcie --no-seq" \
 "r6p_c20:200:python -u bench.py --config C2 --no-cpu --no-pcie --no-seq"
