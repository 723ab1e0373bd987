tools/gpu_job.sh \
 "r6h_stats:600:python -u -m pytest tests/test_gpu_stats.py tests/test_gpu_configs.py::test_c5_share_stats_counts tests/test_adapter.py -x -q --timeout 500 --timeout-method thread" \
 "r6h_prilen:700:bash tools/prilen_breakdown.sh r6h"
