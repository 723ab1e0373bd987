tools/gpu_job.sh \
 "r6aj_tests:900:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r6aj_smoke:150:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6aj_bench:480:python -u bench.py"
