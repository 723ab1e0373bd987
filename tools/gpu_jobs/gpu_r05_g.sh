cat /sys/fs/cgroup/memory.max /sys/fs/cgroup/cpu.max > gpurun_out/r5g_box.txt 2>&1; grep -E "MemTotal|MemAvailable" /proc/meminfo >> gpurun_out/r5g_box.txt; nproc >> gpurun_out/r5g_box.txt
tools/gpu_job.sh \
 "r5g_tests:1150:python -u -m pytest tests -m gpu -x -v --timeout 1000 --timeout-method thread" \
 "r5g_smoke:300:python -c 'import __graft_entry__ as g; g.smoke()'" \
 "r5g_bench:600:python bench.py > gpurun_out/r5g_bench.json"
