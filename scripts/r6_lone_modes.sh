#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for k in 1 2; do scripts/gpu_step.sh 200 lm_$k.log python -u scripts/r6_lone_modes.py || exit 1; done
cat gpurun_out/lm_1.log gpurun_out/lm_2.log
