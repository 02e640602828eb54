#!/bin/bash
# Zstd L1 encode: byte parity (GPU tests), lone frame latency and kernel split
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 500 ze_t.log python -u -m pytest tests/test_zstd_encode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/ze_t.log && ! grep -q "failed" gpurun_out/ze_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/ze_t.log; exit 1; }
scripts/gpu_step.sh 120 ze_lone.log python -u scripts/r6_lone.py 9 || exit 1
scripts/gpu_step.sh 200 ze_kt.log rocprofv3 --kernel-trace --stats -d gpurun_out/ze_kt -o run -- python -u scripts/r6_lone.py 3 0 || exit 1
f=$(find gpurun_out/ze_kt -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/ze_kstats.csv
grep -E "passed" gpurun_out/ze_t.log; grep -h "lone" gpurun_out/ze_lone.log
