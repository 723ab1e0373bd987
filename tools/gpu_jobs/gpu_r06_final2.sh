tools/gpu_job.sh \
 "r6z_tests:600:python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread" \
 "r6z_smoke:150:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
 "r6z_bench:420:python -u bench.py" \
 "r6z_c2:200:python -u bench.py --config C2 --no-cpu --no-pcie --no-seq" \
 "r6z_c4:200:python -u bench.py --config C4 --no-cpu --no-pcie --no-seq" \
 "r6z_prof:250:cd /tmp && export TMPDIR=/tmp && cd \$GRAFT_REPO_ROOT && rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r6z -o run -- python3 bench.py --no-cpu --no-pcie --no-seq"
