set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3"
PMX_MARK_PIPE=0 $B > gpurun_out/r6n_p0_8192.json 2> gpurun_out/r6n_p0_8192.err
PMX_MARK_BLOCKS=2048 $B > gpurun_out/r6n_p1_2048.json 2> gpurun_out/r6n_p1_2048.err
PMX_MARK_BLOCKS=1024 $B > gpurun_out/r6n_p1_1024.json 2> gpurun_out/r6n_p1_1024.err
PMX_MARK_BLOCKS=512 $B > gpurun_out/r6n_p1_512.json 2> gpurun_out/r6n_p1_512.err
PMX_MARK_PIPE=0 PMX_MARK_BLOCKS=2048 $B > gpurun_out/r6n_p0_2048.json 2> gpurun_out/r6n_p0_2048.err
PMX_MARK_PIPE=0 $B > gpurun_out/r6n_p0_8192b.json 2> gpurun_out/r6n_p0_8192b.err
PMX_MARK_BLOCKS=1024 $B > gpurun_out/r6n_p1_1024b.json 2> gpurun_out/r6n_p1_1024b.err
