#!/bin/bash
# zlit overlapped with the sequence kernels (JFS_ZSTD_OVERLAP) x ring size variants: parity and configs[3] time.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
JFS_ZSTD_OVERLAP=1 JFS_GPU_LIB=juicefs_amd/lib/libjfsgpu_r256.so scripts/gpu_step.sh 300 zo.log python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_encode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/zo.log && ! grep -q "failed" gpurun_out/zo.log || { echo "TESTS FAILED"; exit 1; }
scripts/gpu_step.sh 300 zc.log python scripts/prof_run.py 4096 0 T zstd || exit 1
for v in base r256; do
  if [ $v = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for ov in 0 1; do
    r=$(JFS_ZSTD_OVERLAP=$ov JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py 4096 3 T zstd | grep -v amdgpu | head -1) || exit 1
    echo "$v overlap=$ov $r" | tee -a gpurun_out/zx.log
  done
done
