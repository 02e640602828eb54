#!/bin/bash
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
scripts/gpu_step.sh 400 st.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_coalescer_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/st.log && ! grep -q "failed" gpurun_out/st.log || { echo "TESTS FAILED"; exit 1; }
NLIST=1,8,32,128 scripts/gpu_step.sh 200 sp.log python scripts/split_timing.py || exit 1
NLIST=8,32,128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks3 -o ks --output-format csv -- python scripts/split_timing.py > gpurun_out/ks3.log 2>&1 || exit 1
find gpurun_out/ks3 -name '*kernel_stats.csv' -exec cp {} gpurun_out/split_stats3.csv \;
scripts/gpu_step.sh 300 one.log python scripts/oneshot.py || exit 1
