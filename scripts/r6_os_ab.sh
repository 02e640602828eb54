#!/bin/bash
# one-call legs A/B: the library before 6a572b8 (lone-latency commit) vs HEAD
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_r5.so scripts/gpu_step.sh 200 ab_r5a.log python -u scripts/oneshot.py || exit 1
scripts/gpu_step.sh 200 ab_heada.log python -u scripts/oneshot.py || exit 1
JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_r5.so scripts/gpu_step.sh 200 ab_r5b.log python -u scripts/oneshot.py || exit 1
scripts/gpu_step.sh 200 ab_headb.log python -u scripts/oneshot.py || exit 1
JFS_GATHER_PROBE_US=0 scripts/gpu_step.sh 200 ab_head_p0.log python -u scripts/oneshot.py || exit 1
