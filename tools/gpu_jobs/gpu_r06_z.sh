cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r6z
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r6z/trace -o run -- python3 bench.py --no-cpu --no-seq --steps 3 --warmup 1 > gpurun_out/prof_r6z/trace.log 2>&1
echo "trace rc=$?"
