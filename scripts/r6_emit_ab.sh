#!/bin/bash
# split-decoder parity + one-call legs at HEAD vs the round-5 library
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 em_t.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/em_t.log && ! grep -q "failed" gpurun_out/em_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/em_t.log; exit 1; }
scripts/gpu_step.sh 200 em_heada.log python -u scripts/oneshot.py || exit 1
JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_r5.so scripts/gpu_step.sh 200 em_r5.log python -u scripts/oneshot.py || exit 1
scripts/gpu_step.sh 200 em_headb.log python -u scripts/oneshot.py || exit 1
grep passed gpurun_out/em_t.log
