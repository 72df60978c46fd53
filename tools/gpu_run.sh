#!/bin/bash
# Run GPU steps in order; stop at the first step that crashes/aborts/times out
# (exit codes other than 0/1), per the pool's rules.  Usage: tools/gpu_run.sh "<label>:<secs>:<cmd>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  label="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $label ($secs s): $cmd" | tee -a gpurun_out/run.log
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$label.log" 2>&1
  rc=$?
  echo "=== $label rc=$rc" | tee -a gpurun_out/run.log
  tail -5 "gpurun_out/$label.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $label (rc=$rc)"; exit $rc
  fi
done
exit 0
