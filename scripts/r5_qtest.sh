#!/bin/bash
# parity of LZ4-decode library variants (kernel corpus + API tests), then timing
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib scripts/gpu_step.sh 300 t_$v.log python -u -m pytest tests/test_lz4_kernel_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  grep -q " passed" gpurun_out/t_$v.log && ! grep -q "failed" gpurun_out/t_$v.log || { echo "TESTS FAILED $v"; exit 1; }
done
scripts/gpu_step.sh 400 tv.log scripts/time_variants.sh "$@" "$@" || exit 1
grep -v amdgpu gpurun_out/tv.log
