tools/gpu_job.sh \
 "r6h_t:300:python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py -x -q --timeout 280 --timeout-method thread" \
 "r6h_f1a:200:PMX_HINT_FILT=1 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6h_f0a:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6h_f1b:200:PMX_HINT_FILT=1 python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6h_f0b:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6h_t2:300:PMX_HINT_FILT=1 python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py tests/test_gpu_wrec.py -x -q --timeout 280 --timeout-method thread"
