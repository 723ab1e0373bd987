tools/gpu_job.sh \
 "r5m_test:300:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5m_b_app:300:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5m_b_app0:300:PMX_HINT_SAMPLE_ORDER=0 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5m_b_lex:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5m_b_app2:300:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5m_b_lex2:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie"
