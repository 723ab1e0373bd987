set -e
mkdir -p gpurun_out
for sc in 0 4 2 8 0 4; do
PMX_PRILEN_SCHED=$sc timeout -k 10 200 python -u tools/bench_stats.py --metric graded --reps 10 >> gpurun_out/prilen_sched.jsonl 2>> gpurun_out/prilen_sched.err
done
