tools/gpu_job.sh \
 "r5p_prof:900:bash tools/profile.sh r5final"
