tools/gpu_job.sh \
 "r5z5_tests:600:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r5z5_smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r5z5_bench:500:python -u bench.py" \
 "r5z5_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5z5_c4:300:python -u bench.py --config C4 --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5z5_app:300:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5 --numbering appended" \
 "r5z5_prof:600:bash tools/profile.sh r5final8"
