#!/bin/bash
# 20-way Zstd encode at slot budgets 1024 / 2048 / 4096 (segments per block 1 / 2 / 4), interleaved
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -f gpurun_out/sl_sum.log
for sl in 1024 2048 4096 1024 2048 4096; do
  JFS_ZL1_SLOTS=$sl scripts/gpu_step.sh 200 sl_$sl.log python -u scripts/r6_z20.py || exit 1
  echo "slots $sl: $(grep 'burst [12]' gpurun_out/sl_$sl.log | tr '\n' ' ')" >> gpurun_out/sl_sum.log
done
cat gpurun_out/sl_sum.log
