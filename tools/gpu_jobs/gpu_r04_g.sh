set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_resident.py C3 3 > gpurun_out/trg.json 2> gpurun_out/trg.err
bash tools/profile.sh r04c3
bash tools/profile_stats.sh r04c5 --metric graded
