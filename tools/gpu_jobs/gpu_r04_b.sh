set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stats.py tests/test_adapter.py tests/test_gpu_resident.py > gpurun_out/t2.log 2>&1
PMX_NT_STORES=0 timeout -k 10 400 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b_nt0.json 2> gpurun_out/b_nt0.err
timeout -k 10 400 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b_nt1.json 2> gpurun_out/b_nt1.err
