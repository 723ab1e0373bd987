tools/gpu_job.sh \
 "r5q_test:300:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5q_ab_lex:300:python -u tools/ab_env.py --config C3 --env PMX_HINT_SAMPLE_ORDER=0,1,2" \
 "r5q_ab_app:300:python -u tools/ab_env.py --config C3 --numbering appended --env PMX_HINT_SAMPLE_ORDER=0,1,2" \
 "r5q_prof:600:bash tools/profile.sh r5final2"
