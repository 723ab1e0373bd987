tools/gpu_job.sh \
 "r6aa_eq:300:python -u tools/ab_exp_equal.py --exp 24 --config C2" \
 "r6aa_0a:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6aa_24a:200:python -u bench.py --no-cpu --no-pcie --no-seq --run-exp 24" \
 "r6aa_0b:200:python -u bench.py --no-cpu --no-pcie --no-seq" \
 "r6aa_24b:200:python -u bench.py --no-cpu --no-pcie --no-seq --run-exp 24" \
 "r6aa_c2_0:150:python -u bench.py --config C2 --no-cpu --no-pcie --no-seq" \
 "r6aa_c2_24:150:python -u bench.py --config C2 --no-cpu --no-pcie --no-seq --run-exp 24"
