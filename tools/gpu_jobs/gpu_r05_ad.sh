tools/gpu_job.sh \
 "r5ad_sw:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,1376272,1441808" \
 "r5ad_tr:300:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/tr_ad -o run -- python3 tools/sweep.py --config C3 --rounds 1 --reps 3 --opt flags=16,1376272,1441808"
