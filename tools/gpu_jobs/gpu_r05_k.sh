tools/gpu_job.sh \
 "r5k_ser_app:400:python -u tools/sweep.py --config C3 --numbering appended --rounds 3 --reps 5 --opt flags=16,24" \
 "r5k_ser_lex:400:python -u tools/sweep.py --config C3 --rounds 3 --reps 5 --opt flags=16,24" \
 "r5k_tr_app:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_app -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2 --numbering appended" \
 "r5k_tr_lex:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_lex -o run -- python3 bench.py --no-cpu --no-pcie --steps 5 --warmup 2"
