tools/gpu_job.sh \
 "r6y_tests:600:python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread" \
 "r6y_smoke:150:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6y_bench:200:python -u bench.py --no-cpu --no-pcie --no-seq"
