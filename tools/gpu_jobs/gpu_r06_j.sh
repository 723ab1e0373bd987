tools/gpu_job.sh \
 "r6j_tests:1000:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r6j_smoke:150:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'"
