tools/gpu_job.sh \
 "r6af_eq:300:python -u tools/ab_exp_equal.py --exp 25 --config C2" \
 "r6af_0a:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6af_25a:200:python -u bench.py --no-cpu --no-pcie --no-seq --run-exp 25" \
 "r6af_0b:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6af_25b:200:python -u bench.py --no-cpu --no-pcie --no-seq --run-exp 25" \
 "r6af_c4_25:250:python -u bench.py --config C4 --no-cpu --no-pcie --no-seq --run-exp 25" \
 "r6af_c2_25:150:python -u bench.py --config C2 --no-cpu --no-pcie --no-seq --run-exp 25"
