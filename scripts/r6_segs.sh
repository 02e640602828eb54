#!/bin/bash
# lone Zstd encode at 8 and 16 segments per block (and 4), interleaved
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for s in 8 16 4 16 8; do
  JFS_ZL1_SEGS=$s scripts/gpu_step.sh 120 sg_$s.log python -u scripts/r6_lone.py 12 || exit 1
  echo "segs $s: $(grep 'zstd lone encode' gpurun_out/sg_$s.log)" >> gpurun_out/sg_sum.log
done
JFS_ZL1_SEGS=16 scripts/gpu_step.sh 200 sg_kt.log rocprofv3 --kernel-trace --stats -d gpurun_out/sg_kt -o run -- python -u scripts/r6_lone.py 3 0 || exit 1
f=$(find gpurun_out/sg_kt -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/sg_kstats.csv
cat gpurun_out/sg_sum.log
