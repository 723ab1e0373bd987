tools/gpu_job.sh "r5e_dbg:300:python -u tools/dbg/prilen_dist_dbg.py"
