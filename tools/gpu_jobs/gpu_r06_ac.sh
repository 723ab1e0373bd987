tools/gpu_job.sh \
 "r6ac_prof:800:bash tools/profile.sh r6ac --no-seq"
