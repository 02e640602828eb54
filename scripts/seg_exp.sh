#!/bin/bash
# Segment-walk parser experiment on the GPU box: parity of the main kernel,
# wall time per launch of variants, phase stamps of new vs old parser.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/seg
scripts/gpu_step.sh 300 seg/t.log python -u -m pytest tests/test_lz4_kernel_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/seg/t.log && ! grep -q "failed" gpurun_out/seg/t.log || { echo "TESTS FAILED"; exit 1; }
scripts/gpu_step.sh 400 seg/v.log scripts/time_variants.sh base old "$@" || exit 1
cat gpurun_out/seg/v.log
scripts/gpu_step.sh 120 seg/p_new.log python scripts/prof_decode.py 4096 T || exit 1
PROF_LIB=juicefs_amd/lib/libjfsgpu_oldprof.so scripts/gpu_step.sh 120 seg/p_old.log python scripts/prof_decode.py 4096 T || exit 1
cat gpurun_out/seg/p_new.log gpurun_out/seg/p_old.log
