#!/bin/bash
# 17 pointer hops per jump round (five rounds for 4 MiB instead of eight), both
# split paths: parity (LZ4 + Zstd split and batch tests), lone latency, kernel stats
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 500 hp_t.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_lz4_gpu.py tests/test_zstd_split_gpu.py tests/test_zstd_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/hp_t.log && ! grep -q "failed" gpurun_out/hp_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/hp_t.log; exit 1; }
for k in 1 2; do JFS_LONE_ENC=0 scripts/gpu_step.sh 120 hp_lone$k.log python -u scripts/r6_lone.py 21 || exit 1; done
JFS_LONE_ENC=0 scripts/gpu_step.sh 200 hp_lp.log rocprofv3 --kernel-trace -d gpurun_out/hp_lp -o run -- python -u scripts/r6_lone.py 15 0 || exit 1
f=$(find gpurun_out/hp_lp -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/hp_kstats.csv
grep passed gpurun_out/hp_t.log; grep -h "lone decode" gpurun_out/hp_lone1.log gpurun_out/hp_lone2.log
grep -E "jump|zsjump|gather" gpurun_out/hp_kstats.csv | cut -c1-60,100-200
