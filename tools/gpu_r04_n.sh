set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/sweep.py --config C3 --rounds 5 --reps 5 --check --opt flags=16,851984 > gpurun_out/sweep_hintd.log 2>&1
