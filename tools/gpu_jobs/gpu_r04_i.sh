set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_binding.py C3 2 > gpurun_out/trb.json 2> gpurun_out/trb.err
