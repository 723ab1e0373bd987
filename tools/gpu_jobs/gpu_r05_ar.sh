tools/gpu_job.sh \
 "r5ar_smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r5ar_bench:500:python -u bench.py"
