tools/gpu_job.sh \
 "r5al_c2:500:bash tools/profile.sh r5c2final --config C2" \
 "r5al_c4:500:bash tools/profile.sh r5c4final --config C4"
