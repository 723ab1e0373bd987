cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prilen_occ
for x in 0 32 33 0 32 33; do
  PMX_PRILEN_EXP=$x timeout -k 10 200 python3 tools/bench_stats.py --reps 5 > gpurun_out/prilen_occ/t_$x.$RANDOM.json 2>/dev/null || { echo "x$x failed"; exit 2; }
  echo "x$x ok"
done
