set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3"
$B > gpurun_out/r6o_base_a.json 2> gpurun_out/r6o_base_a.err
$B --run-exp 26 > gpurun_out/r6o_e26p0_a.json 2> gpurun_out/r6o_e26p0_a.err
PMX_MARK_PIPE=1 $B --run-exp 26 > gpurun_out/r6o_e26p1_a.json 2> gpurun_out/r6o_e26p1_a.err
$B > gpurun_out/r6o_base_b.json 2> gpurun_out/r6o_base_b.err
$B --run-exp 26 > gpurun_out/r6o_e26p0_b.json 2> gpurun_out/r6o_e26p0_b.err
PMX_MARK_PIPE=1 $B --run-exp 26 > gpurun_out/r6o_e26p1_b.json 2> gpurun_out/r6o_e26p1_b.err
