set -e
mkdir -p gpurun_out
for i in 1 2; do
PMX_NT_STORES=0 timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/trv_nt0_$i.json 2> gpurun_out/trv_nt0_$i.err
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/trv_nt1_$i.json 2> gpurun_out/trv_nt1_$i.err
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_edge_cases.py tests/test_gpu_resident.py tests/test_adapter.py > gpurun_out/t_ntdl.log 2>&1
