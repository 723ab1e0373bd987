set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_resident.py C3 2 > gpurun_out/tr_def.json 2> gpurun_out/tr_def.err
PMX_HOST_THREADS=12 timeout -k 10 300 python -u tools/trace_resident.py C3 2 > gpurun_out/tr_12.json 2> gpurun_out/tr_12.err
PMX_HOST_THREADS=16 timeout -k 10 300 python -u tools/trace_resident.py C3 2 > gpurun_out/tr_16.json 2> gpurun_out/tr_16.err
nproc > gpurun_out/nproc.txt; python -c "import os; print(len(os.sched_getaffinity(0)))" >> gpurun_out/nproc.txt
