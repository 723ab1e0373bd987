cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/qual_r6ah
tools/gpu_job.sh \
 "r6ah_stats:500:python -u -m pytest tests/test_gpu_stats.py tests/test_adapter.py tests/test_gpu_configs.py::test_c5_share_stats_counts -x -q --timeout 400 --timeout-method thread" \
 "r6ah_t1:200:python3 tools/bench_stats.py --reps 10 > gpurun_out/qual_r6ah/t1.json" \
 "r6ah_t3:200:python3 tools/bench_stats.py --reps 10 --metric graded > gpurun_out/qual_r6ah/t3.json" \
 "r6ah_t1b:200:python3 tools/bench_stats.py --reps 10 > gpurun_out/qual_r6ah/t1b.json"
