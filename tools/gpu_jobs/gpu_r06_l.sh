tools/gpu_job.sh \
 "r6l_prof:700:bash tools/profile.sh r6l" \
 "r6l_c4:250:bash tools/profile_trace.sh r6l_c4 --config C4 --no-seq" \
 "r6l_c2:200:bash tools/profile_trace.sh r6l_c2 --config C2 --no-seq"
