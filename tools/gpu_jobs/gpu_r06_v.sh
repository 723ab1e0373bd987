tools/gpu_job.sh \
 "r6v_seq:600:python -u -m pytest tests/test_gpu_seq_surface.py tests/test_gpu_seq_seam.py tests/test_gpu_configs.py::test_full_size_parity -x -q -s --timeout 500 --timeout-method thread" \
 "r6v_b:300:python -u bench.py --no-cpu --no-pcie --steps 10" \
 "r6v_tr:300:bash tools/profile_trace.sh r6v --steps 3 --warmup 1"
