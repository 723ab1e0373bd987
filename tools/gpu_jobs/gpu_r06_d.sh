tools/gpu_job.sh \
 "r6d_tests:1100:python -u -m pytest tests -m gpu -x -v -s --timeout 1000 --timeout-method thread" \
 "r6d_smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6d_bench:600:python -u bench.py"
