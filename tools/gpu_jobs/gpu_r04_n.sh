set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --opt flags=16,24,589840,851984,852000 > gpurun_out/sweep_streams.log 2>&1
