#!/bin/bash
# LZ4 decode iteration loop on the GPU box: parity tests, then the timing of
# every library named (base = juicefs_amd/lib/libjfsgpu.so).
cd "$GRAFT_REPO_ROOT"
scripts/gpu_step.sh 300 qt.log python -u -m pytest tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/qt.log && ! grep -q "failed" gpurun_out/qt.log || { echo "TESTS FAILED"; exit 1; }
scripts/gpu_step.sh 300 qv.log scripts/time_variants.sh "$@"
