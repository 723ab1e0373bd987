tools/gpu_job.sh \
 "r5aa_test:400:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5aa_sw_c3:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,1376272" \
 "r5aa_sw_c2:300:python -u tools/sweep.py --config C2 --rounds 7 --reps 5 --check --opt flags=16,1376272" \
 "r5aa_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_aa -o run -- python3 tools/sweep.py --config C3 --rounds 1 --reps 3 --opt flags=16"
