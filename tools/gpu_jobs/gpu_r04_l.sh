set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py --config C2 --no-cpu --no-pcie --steps 20 --warmup 5 > gpurun_out/b_c2.json 2> gpurun_out/b_c2.err
timeout -k 10 400 python -u bench.py --config C4 --no-cpu --no-pcie --steps 10 --warmup 3 > gpurun_out/b_c4.json 2> gpurun_out/b_c4.err
timeout -k 10 1000 python -u -m pytest -x -s -q --timeout 1100 --timeout-method thread "tests/test_gpu_configs.py::test_full_size_parity" > gpurun_out/t_fullsize.log 2>&1
