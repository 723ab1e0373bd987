set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_edge_cases.py tests/test_gpu_seq_surface.py "tests/test_gpu_stats.py::test_new_tets_shuffled_numbering" > gpurun_out/r6p_t.log 2>&1
B="timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3"
$B > gpurun_out/r6p_win_a.json 2> gpurun_out/r6p_win_a.err
PMX_MARK_WIN=0 $B > gpurun_out/r6p_old_a.json 2> gpurun_out/r6p_old_a.err
$B --run-exp 26 > gpurun_out/r6p_win26_a.json 2> gpurun_out/r6p_win26_a.err
$B > gpurun_out/r6p_win_b.json 2> gpurun_out/r6p_win_b.err
PMX_MARK_WIN=0 $B > gpurun_out/r6p_old_b.json 2> gpurun_out/r6p_old_b.err
$B --run-exp 26 > gpurun_out/r6p_win26_b.json 2> gpurun_out/r6p_win26_b.err
