set -e
mkdir -p gpurun_out
PMX_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo --no-cpu > gpurun_out/b_n2_gloo.json 2> gpurun_out/b_n2_gloo.err
