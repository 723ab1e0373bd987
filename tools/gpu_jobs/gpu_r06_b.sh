tools/gpu_job.sh \
 "r6b_diag:200:python -u tools/dbg/fresh_diff.py" \
 "r6b_seq:600:python -u -m pytest tests/test_gpu_seq_surface.py -x -v -s --timeout 280 --timeout-method thread"
