tools/gpu_job.sh \
 "r5o_tests:600:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5o_smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r5o_bench:500:python -u bench.py" \
 "r5o_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5o_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5o_shuf:300:python -u bench.py --no-cpu --no-pcie --steps 10 --warmup 3 --numbering shuffle"
