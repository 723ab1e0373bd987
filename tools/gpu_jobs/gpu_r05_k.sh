tools/gpu_job.sh \
 "r5k_test:200:python -u -m pytest tests/test_gpu_wrec.py -m gpu -x -v --timeout 180 --timeout-method thread" \
 "r5k_tr_app:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_app -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2 --numbering appended" \
 "r5k_tr_lex:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_lex -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2" \
 "r5k_ser_app:300:python -u tools/sweep.py --config C3 --numbering appended --rounds 3 --reps 5 --opt flags=16,24" \
 "r5k_ser_lex:300:python -u tools/sweep.py --config C3 --rounds 3 --reps 5 --opt flags=16,24" \
 "r5k_f02:300:python -u tools/sweep.py --config C3 --numbering appended:0.02 --rounds 3 --reps 5 --opt flags=1179664,393232" \
 "r5k_f05:300:python -u tools/sweep.py --config C3 --numbering appended:0.05 --rounds 3 --reps 5 --opt flags=1179664,393232"
