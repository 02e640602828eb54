#!/bin/bash
# phase split of the Zstd L1 parse (prof build): 1 frame (segments) and 256 frames (frame-serial)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_prof.so scripts/gpu_step.sh 200 zpp1.log python -u scripts/zpprof.py 1 || exit 1
JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_prof.so scripts/gpu_step.sh 300 zpp256.log python -u scripts/zpprof.py 256 || exit 1
cat gpurun_out/zpp1.log gpurun_out/zpp256.log
