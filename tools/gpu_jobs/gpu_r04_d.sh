set -e
mkdir -p gpurun_out
for i in 1 2; do
for th in 8 16 24; do
PMX_HOST_THREADS=$th timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/tra_${th}_$i.json 2> gpurun_out/tra_${th}_$i.err
done
done
cat /sys/fs/cgroup/cpu.max > gpurun_out/cg.txt 2>&1 || true
lscpu > gpurun_out/lscpu.txt 2>&1 || true
