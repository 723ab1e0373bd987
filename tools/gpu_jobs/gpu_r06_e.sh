tools/gpu_job.sh \
 "r6e_seq:900:python -u -m pytest tests/test_gpu_seq_surface.py tests/test_gpu_configs.py -x -v -s --timeout 800 --timeout-method thread -k 'seq or full_size'" \
 "r6e_prilen:700:bash tools/prilen_breakdown.sh r6e" \
 "r6e_bseq:400:python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3"
