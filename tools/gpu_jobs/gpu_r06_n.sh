tools/gpu_job.sh \
 "r6n_seq:900:python -u -m pytest tests/test_gpu_seq_surface.py tests/test_gpu_seq_seam.py tests/test_gpu_configs.py -x -v -s --timeout 800 --timeout-method thread" \
 "r6n_b:300:python -u bench.py --no-cpu --no-pcie --steps 10"
