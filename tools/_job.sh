tools/gpu_job.sh \
 "q0:120:python -u tools/bench_stats.py --metric graded --reps 20" \
 "q1:120:PMX_EXP_QUAL_ORDER=1 PMX_EXP_QUAL_BLOCKS=1536 python -u tools/bench_stats.py --metric graded --reps 20" \
 "q1b:120:PMX_EXP_QUAL_ORDER=1 PMX_EXP_QUAL_BLOCKS=3072 python -u tools/bench_stats.py --metric graded --reps 20" \
 "q2:120:PMX_EXP_QUAL_ORDER=2 PMX_EXP_QUAL_BLOCKS=1536 python -u tools/bench_stats.py --metric graded --reps 20" \
 "q2b:120:PMX_EXP_QUAL_ORDER=2 PMX_EXP_QUAL_BLOCKS=4096 python -u tools/bench_stats.py --metric graded --reps 20" \
 "numbering:600:python -u tools/numbering.py --config C3 --variants lex,vmorton,tmorton --rounds 3" \
 "sweep9:300:python -u tools/sweep.py --config C3 --rounds 3 --reps 5 --check --opt flags=0,589824" && \
tools/gpu_job.sh \
 "p1:120:PMX_EXP_PRILEN=1 python -u tools/bench_stats.py --metric graded --reps 10" \
 "p2:120:PMX_EXP_PRILEN=2 python -u tools/bench_stats.py --metric graded --reps 10" \
 "pp1:200:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && PMX_EXP_PRILEN=1 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_prilen -f csv -d gpurun_out/pp1 -o run -- python3 tools/bench_stats.py --metric graded --reps 2" \
 "pp2:200:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && PMX_EXP_PRILEN=2 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_prilen -f csv -d gpurun_out/pp2 -o run -- python3 tools/bench_stats.py --metric graded --reps 2"
