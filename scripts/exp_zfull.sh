#!/bin/bash
# Full GPU test suite, then configs[3] timing of zseq variants.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
scripts/gpu_step.sh 900 gt.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread || exit 1
grep -E "passed|failed" gpurun_out/gt.log | tail -2
grep -q " failed" gpurun_out/gt.log && { echo "TESTS FAILED"; exit 1; }
scripts/gpu_step.sh 300 zc.log python scripts/prof_run.py 4096 0 T zstd || exit 1
for v in base ${ZVARS}; do
  if [ $v = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for rep in 1 2; do
    r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py 4096 3 T zstd | grep -v amdgpu | head -1) || exit 1
    echo "$v $r" | tee -a gpurun_out/zx.log
  done
done
