#!/bin/bash
# zseq phase shares (prof build)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
scripts/gpu_step.sh 300 zsp.log python scripts/zsprof.py 2048 || exit 1
cat gpurun_out/zsp.log
