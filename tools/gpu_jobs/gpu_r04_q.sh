set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all3.log 2>&1
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/trq.json 2> gpurun_out/trq.err
timeout -k 10 300 python -u tools/trace_binding.py C3 3 > gpurun_out/trbq.json 2> gpurun_out/trbq.err
