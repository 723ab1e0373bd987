set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/t_all5.log 2>&1
for i in 1 2; do
PMX_NT_STORES=0 timeout -k 10 300 python -u tools/trace_binding.py C3 3 > gpurun_out/tw_nt0_$i.json 2> gpurun_out/tw_nt0_$i.err
timeout -k 10 300 python -u tools/trace_binding.py C3 3 > gpurun_out/tw_nt1_$i.json 2> gpurun_out/tw_nt1_$i.err
done
