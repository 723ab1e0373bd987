tools/gpu_job.sh \
 "r6o_edge:600:python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py -x -q --timeout 500 --timeout-method thread" \
 "r6o_c3:300:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6o_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie --no-seq" \
 "r6o_tr:250:bash tools/profile_trace.sh r6o --no-seq"
