tools/gpu_job.sh \
 "r5l_tests:900:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5l_b_lex:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5l_b_lex0:200:PMX_HINT_SAMPLE_ORDER=0 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5l_b_app:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5l_b_app0:200:PMX_HINT_SAMPLE_ORDER=0 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended" \
 "r5l_b_lex2:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie" \
 "r5l_b_app2:200:python -u bench.py --steps 20 --warmup 5 --no-cpu --no-pcie --numbering appended"
