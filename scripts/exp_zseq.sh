#!/bin/bash
# zseq two-wave LDS decoder: parity (Zstd decode tests), configs[3] time vs variants, phase profile.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
scripts/gpu_step.sh 300 zd.log python -u -m pytest tests/test_zstd_gpu.py tests/test_zstd_encode_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/zd.log && ! grep -q "failed" gpurun_out/zd.log || { echo "TESTS FAILED"; exit 1; }
scripts/gpu_step.sh 300 zc.log python scripts/prof_run.py 4096 0 T zstd || exit 1
for v in base ${ZVARS:-zs1}; do
  if [ $v = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for rep in 1 2; do
    r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py 4096 3 T zstd | grep -v amdgpu | head -1) || exit 1
    echo "$v $r" | tee -a gpurun_out/zx.log
  done
done
[ -n "$ZQUICK" ] && exit 0
scripts/gpu_step.sh 300 zsp.log python scripts/zsprof.py 2048 || exit 1
cat gpurun_out/zsp.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kz -o kz --output-format csv -- python scripts/prof_run.py 4096 3 T zstd > gpurun_out/kz.log 2>&1 || exit 1
find gpurun_out/kz -name '*kernel_stats.csv' -exec cp {} gpurun_out/zstd_stats_zseq2.csv \;
