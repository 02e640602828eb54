#!/bin/bash
# Zstd decode: parity tests (one-wave path + split path), then configs[3] timing of variants
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 zt.log python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/zt.log && ! grep -q "failed" gpurun_out/zt.log || { echo "TESTS FAILED"; tail -30 gpurun_out/zt.log; exit 1; }
scripts/gpu_step.sh 500 tz.log scripts/time_zvariants.sh "$@" "$@" || exit 1
grep -v amdgpu gpurun_out/tz.log
