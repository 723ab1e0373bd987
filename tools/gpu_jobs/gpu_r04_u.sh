set -e
mkdir -p gpurun_out
for i in 1 2; do
PMX_NT_STORES=0 timeout -k 10 300 python -u tools/trace_binding.py C3 3 > gpurun_out/tb_nt0_$i.json 2> gpurun_out/tb_nt0_$i.err
timeout -k 10 300 python -u tools/trace_binding.py C3 3 > gpurun_out/tb_nt1_$i.json 2> gpurun_out/tb_nt1_$i.err
done
