tools/gpu_job.sh \
 "r6w_bind:400:PMX_TRACE=1 python -u tools/bench_binding.py --iters 2"
