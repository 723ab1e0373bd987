tools/gpu_job.sh \
 "r5ac_n2:400:PMX_BENCH_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --config C2 --steps 5 --warmup 2" \
 "r5ac_sw15:400:python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,983056"
