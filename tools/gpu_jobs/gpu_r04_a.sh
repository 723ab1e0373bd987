set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_stats.py tests/test_adapter.py > gpurun_out/t1.log 2>&1
timeout -k 10 500 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/b_c3.json 2> gpurun_out/b_c3.err
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3 --numbering shuffle > gpurun_out/b_shuf.json 2> gpurun_out/b_shuf.err
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3 --numbering appended > gpurun_out/b_app.json 2> gpurun_out/b_app.err
