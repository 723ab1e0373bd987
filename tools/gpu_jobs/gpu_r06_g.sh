tools/gpu_job.sh \
 "r6g_stats:900:python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py tests/test_adapter.py tests/test_gpu_seq_surface.py tests/test_gpu_configs.py -x -v -s --timeout 800 --timeout-method thread" \
 "r6g_prilen:700:bash tools/prilen_breakdown.sh r6g" \
 "r6g_bapp:400:python -u bench.py --numbering appended --no-cpu --no-pcie"
