#!/bin/bash
# emit without the modulo for non-overlapping matches: split tests, lone timeline, lone latency
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 em2_t.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/em2_t.log && ! grep -q "failed" gpurun_out/em2_t.log || { echo "TESTS FAILED"; tail -30 gpurun_out/em2_t.log; exit 1; }
bash scripts/r6_lz4tl.sh || exit 1
JFS_LONE_CODECS=lz4 JFS_LONE_ENC=0 scripts/gpu_step.sh 120 em2_lone.log python -u scripts/r6_lone.py 21 || exit 1
grep passed gpurun_out/em2_t.log; grep -E "emit|lone" gpurun_out/lz4_tl.txt | tail -6; grep "lone decode" gpurun_out/em2_lone.log
