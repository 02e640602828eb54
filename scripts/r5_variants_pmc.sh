#!/bin/bash
# time + one PMC pass (instruction mix) per LZ4-decode library variant
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 tv.log scripts/time_variants.sh "$@" || exit 1
scripts/gpu_step.sh 600 pmc.log scripts/pmc_insts.sh "$@" || exit 1
