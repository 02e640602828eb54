#!/bin/bash
# lone one-call decode with its output D2H in 1 / 2 / 4 byte pieces (copy-out of a
# piece overlapping the D2H of the next), two runs each; one-call tests with 2 pieces
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_BYTE_PIECES=2 scripts/gpu_step.sh 400 bp_t.log python -u -m pytest tests/test_coalescer_gpu.py tests/test_lz4_gpu.py tests/test_zstd_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/bp_t.log && ! grep -q "failed" gpurun_out/bp_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/bp_t.log; exit 1; }
rm -f gpurun_out/bp_sum.log
for r in 1 2; do for n in 0 2 4; do
  JFS_BYTE_PIECES=$n JFS_LONE_ENC=0 scripts/gpu_step.sh 120 bp_$n.log python -u scripts/r6_lone.py 21 || exit 1
  echo "pieces=$n: $(grep 'lone decode' gpurun_out/bp_$n.log | tr '\n' ' ')" >> gpurun_out/bp_sum.log
done; done
grep passed gpurun_out/bp_t.log; cat gpurun_out/bp_sum.log
