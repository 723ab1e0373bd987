tools/gpu_job.sh \
 "r5af_test:400:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py tests/test_gpu_resident.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5af_ab_lex:300:python -u tools/ab_env.py --config C3 --env PMX_HINT_SAMPLE_ORDER=0,1" \
 "r5af_ab_app:300:python -u tools/ab_env.py --config C3 --numbering appended --env PMX_HINT_SAMPLE_ORDER=0,1" \
 "r5af_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_af -o run -- python3 tools/sweep.py --config C3 --numbering appended --rounds 1 --reps 3 --opt flags=16"
