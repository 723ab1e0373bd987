set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_stats.py tests/test_adapter.py tests/test_gpu_parity.py > gpurun_out/t_stats2.log 2>&1
for i in 1 2; do
timeout -k 10 200 python -u tools/bench_stats.py --metric graded --reps 10 >> gpurun_out/stats_kq2.jsonl 2>> gpurun_out/stats_kq2.err
done
bash tools/gpu_r04_l.sh
