#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault,
# abort, segfault or timeout (exit codes other than 0/1).  Usage:
#   scripts/gpu_step.sh <seconds> <logname> <cmd...>
secs=$1; shift; log=$1; shift
mkdir -p gpurun_out
echo "=== $(date +%T) $log: $*" | tee -a gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "=== $(date +%T) $log rc=$rc" | tee -a gpurun_out/steps.log
tail -5 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "FATAL step $log rc=$rc: stopping" | tee -a gpurun_out/steps.log
  exit 99
fi
exit 0
