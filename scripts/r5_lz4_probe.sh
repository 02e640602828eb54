#!/bin/bash
# Round 5 LZ4-decode probe on the GPU box: timing of the named library
# variants (4096 text blocks), the phase stamps of the prof build, and one PMC
# pass (instruction mix + waits) of the first variant.
# usage: scripts/r5_lz4_probe.sh name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 200 tv.log scripts/time_variants.sh "$@" || exit 1
if [ -f juicefs_amd/lib/libjfsgpu_prof.so ]; then
  scripts/gpu_step.sh 120 prof.log python scripts/prof_decode.py 4096 T || exit 1
fi
scripts/gpu_step.sh 200 pmc.log scripts/pmc_insts.sh "$1" || exit 1
cat gpurun_out/tv.log gpurun_out/prof.log gpurun_out/pmc.log
