tools/gpu_job.sh \
 "r5ae_test:400:python -u -m pytest tests/test_gpu_edge_cases.py tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5ae_sw:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,1507344" \
 "r5ae_sw2:300:python -u tools/sweep.py --config C2 --rounds 7 --reps 5 --check --opt flags=16,1507344" \
 "r5ae_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_ae -o run -- python3 tools/sweep.py --config C3 --rounds 1 --reps 3 --opt flags=16,1507344"
