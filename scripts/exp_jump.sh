#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
scripts/gpu_step.sh 400 st.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_coalescer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/st.log && ! grep -q "failed" gpurun_out/st.log || { echo "TESTS FAILED"; exit 1; }
NLIST=1,8,32,128 scripts/gpu_step.sh 200 sp.log python scripts/split_timing.py || exit 1
for c in 8 16 32; do
  JFS_COALESCE_CHUNK=$c scripts/gpu_step.sh 300 one_$c.log python scripts/oneshot.py || exit 1
done
