cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/len_ab
for r in 1 2; do
for x in 0 128; do
for m in iso graded; do
  PMX_PRILEN_EXP=$x timeout -k 10 200 python3 tools/bench_stats.py --reps 10 --metric $m > gpurun_out/len_ab/t_${m}_${x}_$r.json 2>/dev/null || { echo "fail $x $m"; exit 2; }
  echo "ok $x $m $r"
done; done; done
