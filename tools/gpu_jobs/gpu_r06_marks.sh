set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_edge_cases.py tests/test_gpu_seq_surface.py > gpurun_out/r6m_t.log 2>&1
PMX_MARK_PIPE=0 timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 > gpurun_out/r6m_b0a.json 2> gpurun_out/r6m_b0a.err
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 > gpurun_out/r6m_b1a.json 2> gpurun_out/r6m_b1a.err
PMX_MARK_PIPE=0 timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 > gpurun_out/r6m_b0b.json 2> gpurun_out/r6m_b0b.err
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-seq --steps 20 --warmup 3 > gpurun_out/r6m_b1b.json 2> gpurun_out/r6m_b1b.err
