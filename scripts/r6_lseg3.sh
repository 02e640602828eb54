#!/bin/bash
# LZ4 split segment size 256 (HEAD) / 128 / 64: split parity (stays on the split path), lone decode latency
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -f gpurun_out/sg3_sum.log
for v in seg128 seg64; do
  JFS_GPU_LIB=$PWD/juicefs_amd/lib/libjfsgpu_$v.so scripts/gpu_step.sh 300 sg3_t_$v.log python -u -m pytest tests/test_lz4_split_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
  echo "$v tests: $(tail -1 gpurun_out/sg3_t_$v.log)" >> gpurun_out/sg3_sum.log
done
for r in 1 2; do for v in base seg128 seg64; do
  L=$PWD/juicefs_amd/lib/libjfsgpu_$v.so; [ $v = base ] && L=$PWD/juicefs_amd/lib/libjfsgpu.so
  JFS_GPU_LIB=$L JFS_LONE_CODECS=lz4 JFS_LONE_ENC=0 scripts/gpu_step.sh 120 sg3_$v.log python -u scripts/r6_lone.py 15 || exit 1
  echo "$v: $(grep 'lone decode' gpurun_out/sg3_$v.log)" >> gpurun_out/sg3_sum.log
done; done
for v in base seg64; do
  L=$PWD/juicefs_amd/lib/libjfsgpu_$v.so; [ $v = base ] && L=$PWD/juicefs_amd/lib/libjfsgpu.so
  JFS_GPU_LIB=$L scripts/gpu_step.sh 300 sg3_os_$v.log python -u scripts/oneshot.py || exit 1
done
cat gpurun_out/sg3_sum.log
