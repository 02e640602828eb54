#!/bin/bash
# zsblk state-pass rewrite: Zstd parity (split + batch paths), lone latency, kernel stats
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 zs_t.log python -u -m pytest tests/test_zstd_split_gpu.py tests/test_zstd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/zs_t.log && ! grep -q "failed" gpurun_out/zs_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/zs_t.log; exit 1; }
scripts/gpu_step.sh 120 zs_lone.log python -u scripts/r6_lone.py 15 || exit 1
scripts/gpu_step.sh 200 zs_lp.log rocprofv3 --kernel-trace --stats -d gpurun_out/zs_lp -o run -- python -u scripts/r6_lone.py 15 0 || exit 1
f=$(find gpurun_out/zs_lp -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/zs_lone_kstats.csv
grep -E "passed|lone decode" gpurun_out/zs_t.log gpurun_out/zs_lone.log
