set -e
mkdir -p gpurun_out
B="timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3"
PMX_MARK_H=8 $B > gpurun_out/r6q_h8_a.json 2> gpurun_out/r6q_h8_a.err
PMX_MARK_H=8 $B --run-exp 26 > gpurun_out/r6q_h8e26_a.json 2> gpurun_out/r6q_h8e26_a.err
$B --run-exp 26 > gpurun_out/r6q_h4e26_a.json 2> gpurun_out/r6q_h4e26_a.err
$B > gpurun_out/r6q_h4_a.json 2> gpurun_out/r6q_h4_a.err
PMX_MARK_H=8 $B > gpurun_out/r6q_h8_b.json 2> gpurun_out/r6q_h8_b.err
PMX_MARK_H=8 $B --run-exp 26 > gpurun_out/r6q_h8e26_b.json 2> gpurun_out/r6q_h8e26_b.err
$B --run-exp 26 > gpurun_out/r6q_h4e26_b.json 2> gpurun_out/r6q_h4e26_b.err
$B > gpurun_out/r6q_h4_b.json 2> gpurun_out/r6q_h4_b.err
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r6q -o run -- python3 bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 > gpurun_out/prof_r6q.log 2>&1
