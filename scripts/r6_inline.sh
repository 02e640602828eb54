#!/bin/bash
# inline lone decodes: one-call tests, lone latency and one-call legs with and without
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 il_t.log python -u -m pytest tests/test_lz4_gpu.py tests/test_batch_gpu.py tests/test_zstd_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/il_t.log && ! grep -q "failed" gpurun_out/il_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/il_t.log; exit 1; }
rm -f gpurun_out/il_sum.log
for r in 1 2; do for v in 1 0; do
  JFS_INLINE_LONE=$v JFS_LONE_ENC=0 scripts/gpu_step.sh 120 il_$v.log python -u scripts/r6_lone.py 21 || exit 1
  echo "inline=$v: $(grep 'lone decode' gpurun_out/il_$v.log | tr '\n' ' ')" >> gpurun_out/il_sum.log
done; done
for v in 1 0; do JFS_INLINE_LONE=$v scripts/gpu_step.sh 300 il_os_$v.log python -u scripts/oneshot.py || exit 1; done
grep passed gpurun_out/il_t.log; cat gpurun_out/il_sum.log
