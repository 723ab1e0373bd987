set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tre.json 2> gpurun_out/tre.err
timeout -k 10 600 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err
