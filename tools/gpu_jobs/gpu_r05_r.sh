tools/gpu_job.sh \
 "r5r_test:300:python -u -m pytest tests/test_gpu_wrec.py tests/test_gpu_parity.py -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5r_bench:500:python -u bench.py" \
 "r5r_app:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5 --numbering appended" \
 "r5r_shuf:300:python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3 --numbering shuffle" \
 "r5r_lex:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5r_prof:600:bash tools/profile.sh r5final3"
