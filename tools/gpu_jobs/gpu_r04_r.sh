set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_tpk.log 2>&1
PMX_TPK=0 timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tr_tpk0.json 2> gpurun_out/tr_tpk0.err
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tr_tpk1.json 2> gpurun_out/tr_tpk1.err
PMX_TPK=0 timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tr_tpk0b.json 2> gpurun_out/tr_tpk0b.err
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tr_tpk1b.json 2> gpurun_out/tr_tpk1b.err
