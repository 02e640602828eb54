#!/bin/bash
# LZ4 encode parity (segment + serial + golden) and the one-call legs
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 500 le_t.log python -u -m pytest tests/test_lz4_eseg_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/le_t.log && ! grep -q "failed" gpurun_out/le_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/le_t.log; exit 1; }
scripts/gpu_step.sh 300 le_os.log python -u scripts/oneshot.py || exit 1
grep passed gpurun_out/le_t.log
