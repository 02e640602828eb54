#!/bin/bash
# device-side time of the split LZ4 decoder at segment sizes 256 / 128 / 64, 1..64 blocks (interleaved twice)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -f gpurun_out/sg4_sum.log
for r in 1 2; do for v in base seg128 seg64; do
  L=$PWD/juicefs_amd/lib/libjfsgpu_$v.so; [ $v = base ] && L=$PWD/juicefs_amd/lib/libjfsgpu.so
  NMAX=64 NLIST=1,2,4,16,64 JFS_GPU_LIB=$L scripts/gpu_step.sh 200 sg4_$v.log python -u scripts/split_timing.py || exit 1
  echo "== $v" >> gpurun_out/sg4_sum.log; grep "small" gpurun_out/sg4_$v.log | awk '{print $1, $3, $4, $7}' >> gpurun_out/sg4_sum.log
done; done
cat gpurun_out/sg4_sum.log
