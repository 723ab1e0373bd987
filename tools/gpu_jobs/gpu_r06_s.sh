tools/gpu_job.sh \
 "r6s_tests:900:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r6s_smoke:150:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6s_bench:420:python -u bench.py"
