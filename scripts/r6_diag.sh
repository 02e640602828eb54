#!/bin/bash
# 20-way Zstd encode timeline + lone LZ4 decode host trace and kernel timeline
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/r6_z20.sh || exit 1
JFS_LONE_ENC=0 JFS_HOST_TRACE=1 scripts/gpu_step.sh 120 lone_tr.log python -u scripts/r6_lone.py 9 || exit 1
JFS_LONE_ENC=0 bash scripts/r6_lone_prof.sh > gpurun_out/lone_tl.txt 2>&1 || exit 1
