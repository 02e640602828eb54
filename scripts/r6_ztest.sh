#!/bin/bash
# Round 6 Zstd/batch checks on the GPU box: parity tests, then configs[3] timing.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 500 zt.log python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_split_gpu.py tests/test_batch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/zt.log && ! grep -q "failed" gpurun_out/zt.log || { echo "TESTS FAILED"; tail -30 gpurun_out/zt.log; exit 1; }
scripts/gpu_step.sh 300 zc.log python scripts/prof_run.py 4096 3 T zstd || exit 1
grep -E "passed|ms/launch" gpurun_out/zt.log gpurun_out/zc.log
