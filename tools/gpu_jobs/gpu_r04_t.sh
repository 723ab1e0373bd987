set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/sweep.py --config C3 --rounds 7 --reps 5 --check --opt flags=16,983056 > gpurun_out/sweep_nthash.log 2>&1
