#!/bin/bash
# configs[3] Zstd decode with the batch cut into 1 / 2 / 3 / 4 pipelined input ranges (verified)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
rm -f gpurun_out/zp_sum.log
for k in 1 2 3 4 1 2 4; do
  JFS_ZSTD_PIPE=$k scripts/gpu_step.sh 200 zp_$k.log python -u scripts/prof_run.py 4096 5 T zstd || exit 1
  echo "pipe $k: $(grep -E 'ms/launch|ok' gpurun_out/zp_$k.log | tr '\n' ' ')" >> gpurun_out/zp_sum.log
done
cat gpurun_out/zp_sum.log
