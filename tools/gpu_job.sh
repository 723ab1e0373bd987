#!/bin/bash
# Run GPU steps in order; stop at the first step that ends in a fault, abort,
# segfault or time limit (anything but 0 = ok / 1 = test failures).
# usage: tools/gpu_job.sh "<name>:<timeout_s>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"
  tmo="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($tmo s): $cmd" | tee -a gpurun_out/job.log
  timeout -k 10 "$tmo" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name exit $rc" | tee -a gpurun_out/job.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/job.log
    exit $rc
  fi
done
exit 0
