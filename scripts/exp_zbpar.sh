#!/bin/bash
# Block-parallel Zstd encoder: rate and ratio of warm-up variants vs one wave
# per frame, lone-frame latency, one-call legs; split-decoder kernel split.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in base w16 w128 w256; do
  if [ $v = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib scripts/gpu_step.sh 200 ze_$v.log python scripts/time_zenc.py 1024 || exit 1
done
JFS_ZSTD_BPAR=0 scripts/gpu_step.sh 200 ze0.log python scripts/time_zenc.py 1024 || exit 1
scripts/gpu_step.sh 200 ze1.log python scripts/time_zenc.py 1 || exit 1
JFS_ZSTD_BPAR=0 scripts/gpu_step.sh 200 ze1s.log python scripts/time_zenc.py 1 || exit 1
scripts/gpu_step.sh 200 ze8.log python scripts/time_zenc.py 8 || exit 1
scripts/gpu_step.sh 300 one.log python scripts/oneshot.py || exit 1
NLIST=8,32,128 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ks -o ks --output-format csv -- python scripts/split_timing.py > gpurun_out/ks.log 2>&1 || exit 1
find gpurun_out/ks -name '*kernel_stats.csv' -exec cp {} gpurun_out/split_stats.csv \;
cat gpurun_out/ze_*.log gpurun_out/ze0.log gpurun_out/ze1.log gpurun_out/ze1s.log gpurun_out/ze8.log | grep -v amdgpu
