#!/bin/bash
# zseqb state pass with the extra-bit counts in VALU arithmetic: Zstd GPU tests,
# configs[3] launch time (verified), kernel stats
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 zxb_t.log python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/zxb_t.log && ! grep -q "failed" gpurun_out/zxb_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/zxb_t.log; exit 1; }
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
for k in 1 2; do scripts/gpu_step.sh 200 zxb_r$k.log python -u scripts/prof_run.py 4096 5 T zstd || exit 1; done
scripts/gpu_step.sh 300 zxb_kt.log rocprofv3 --kernel-trace --stats -d gpurun_out/zxb_kt -o run -- python -u scripts/prof_run.py 4096 3 T zstd || exit 1
f=$(find gpurun_out/zxb_kt -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/zxb_kstats.csv
grep passed gpurun_out/zxb_t.log; grep -h -E "ms/launch|ok" gpurun_out/zxb_r1.log gpurun_out/zxb_r2.log
grep -E "zseqb|zexec" gpurun_out/zxb_kstats.csv | cut -c1-40,200-
