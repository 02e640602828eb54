#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 coal_t.log python -u -m pytest tests/test_coalescer_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
JFS_INLINE_LONE=0 scripts/gpu_step.sh 400 coal_t0.log python -u -m pytest tests/test_coalescer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "lone or 200" || exit 1
grep -E "PASS|FAIL|passed|failed" gpurun_out/coal_t.log | tail -12; tail -2 gpurun_out/coal_t0.log
