tools/gpu_job.sh \
 "r6m_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie --no-seq" \
 "r6m_c4t:250:bash tools/profile_trace.sh r6m_c4 --config C4 --no-seq" \
 "r6m_c3:300:python -u bench.py --no-cpu --no-pcie --no-seq"
