#!/bin/bash
# lone one-call decode latency, traced; default gather window and none
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_HOST_TRACE=1 scripts/gpu_step.sh 120 lone_a.log python -u scripts/r6_lone.py || exit 1
JFS_GATHER_US=0 JFS_HOST_TRACE=1 scripts/gpu_step.sh 120 lone_b.log python -u scripts/r6_lone.py || exit 1
grep "lone decode" gpurun_out/lone_a.log gpurun_out/lone_b.log
