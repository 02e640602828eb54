#!/bin/bash
# encode parity + the one-call legs alone (LZ4 and Zstd, lone and concurrent)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 500 e2_t.log python -u -m pytest tests/test_zstd_encode_gpu.py tests/test_batch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/e2_t.log && ! grep -q "failed" gpurun_out/e2_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/e2_t.log; exit 1; }
scripts/gpu_step.sh 300 e2_os.log python -u scripts/oneshot.py || exit 1
scripts/gpu_step.sh 200 e2_kt.log rocprofv3 --kernel-trace --stats -d gpurun_out/e2_kt -o run -- python -u scripts/r6_lone.py 3 0 || exit 1
f=$(find gpurun_out/e2_kt -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/e2_kstats.csv
grep -E "passed" gpurun_out/e2_t.log; tail -3 gpurun_out/e2_os.log
