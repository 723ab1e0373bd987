tools/gpu_job.sh \
 "r6f_stats:900:python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_parity.py tests/test_adapter.py tests/test_gpu_seq_surface.py tests/test_gpu_configs.py -x -v -s --timeout 800 --timeout-method thread" \
 "r6f_prilen:700:bash tools/prilen_breakdown.sh r6f" \
 "r6f_bseq:400:python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3"
