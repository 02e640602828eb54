#!/bin/bash
# Round 6 LZ4 decode loop on the GPU box: parity tests of the device path,
# then wall time per launch (4096 text blocks) with the chain bitmap on/off,
# then a rocprofv3 kernel-time summary of the chain path.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 t.log python -u -m pytest tests/test_lz4_kernel_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/t.log && ! grep -q "failed" gpurun_out/t.log || { echo "TESTS FAILED"; cat gpurun_out/t.log | tail -30; exit 1; }
for r in 1 2; do
  for ch in 1 0; do
    JFS_LZ4_CHAIN=$ch scripts/gpu_step.sh 120 tv_$ch.log python scripts/prof_run.py 4096 5 T || exit 1
    echo "chain=$ch $(head -1 gpurun_out/tv_$ch.log)" | tee -a gpurun_out/tv.log
  done
done
scripts/gpu_step.sh 200 rp.log rocprofv3 --kernel-trace --stats -d gpurun_out/rp -o run -- python scripts/prof_run.py 4096 5 T || exit 1
find gpurun_out/rp -name "*kernel_stats.csv" -exec cp {} gpurun_out/r6_kstats.csv \;
cat gpurun_out/tv.log; cut -d, -f1-8 gpurun_out/r6_kstats.csv | head -8
