tools/gpu_job.sh \
 "r6ag_t:400:PMX_MARK_TPT=4 python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
 "r6ag_2a:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6ag_4a:200:PMX_MARK_TPT=4 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6ag_2b:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6ag_4b:200:PMX_MARK_TPT=4 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6ag_tr4:250:PMX_MARK_TPT=4 bash tools/profile_trace.sh r6ag --no-seq --steps 5 --warmup 2"
