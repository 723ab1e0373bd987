tools/gpu_job.sh \
 "r5ai_8k:200:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5ai_64k:200:PMX_DERIVE_BLOCKS=65536 python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5ai_2k:200:PMX_DERIVE_BLOCKS=2048 python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5ai_8kb:200:python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5ai_64kb:200:PMX_DERIVE_BLOCKS=65536 python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5" \
 "r5ai_2kb:200:PMX_DERIVE_BLOCKS=2048 python -u bench.py --no-cpu --no-pcie --steps 20 --warmup 5"
