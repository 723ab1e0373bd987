export PRILEN_VARIANTS="0 4 8 16 24"
tools/gpu_job.sh \
 "r6i_seam:300:python -u -m pytest tests/test_gpu_seq_seam.py -x -v -s --timeout 280 --timeout-method thread" \
 "r6i_prilen:600:bash tools/prilen_breakdown.sh r6i" \
 "r6i_wpmc:900:bash tools/walk_pmc_env.sh r6i default= compact=PMX_WALK_RECORDS=compact owner=PMX_HINT_SAMPLE_ORDER=2"
