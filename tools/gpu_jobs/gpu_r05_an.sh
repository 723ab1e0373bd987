tools/gpu_job.sh \
 "r5an_test:400:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py tests/test_gpu_resident.py tests/test_gpu_edge_cases.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5an_ab_lex:300:python -u tools/ab_env.py --config C3 --env PMX_HINT_SAMPLE_ORDER=1,2" \
 "r5an_ab_app:300:python -u tools/ab_env.py --config C3 --numbering appended --env PMX_HINT_SAMPLE_ORDER=1,2" \
 "r5an_ab_shuf:400:python -u tools/ab_env.py --config C3 --numbering shuffle --rounds 3 --env PMX_HINT_SAMPLE_ORDER=1,2" \
 "r5an_ab_c2:300:python -u tools/ab_env.py --config C2 --env PMX_HINT_SAMPLE_ORDER=1,2"
