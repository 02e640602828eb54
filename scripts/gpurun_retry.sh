#!/bin/bash
# gpurun with retries on "transient" (box not prepared) / exit 3 (no box);
# a command that actually ran is never retried.
for i in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | grep '^\[gpurun\]'
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then sleep 45; continue; fi
  exit $rc
done
exit 1
