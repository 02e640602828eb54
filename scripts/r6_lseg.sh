#!/bin/bash
# encode parity, one-call legs, and the lone LZ4 encode at 64 / 32 / 16 KiB segments
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/r6_enc2.sh || exit 1
rm -f gpurun_out/ls_sum.log
for kb in 64 32 16 64 32; do
  JFS_LZ4E_SEG_MIN_KB=$kb scripts/gpu_step.sh 120 ls_$kb.log python -u scripts/r6_lone.py 9 || exit 1
  echo "seg $kb KiB: $(grep 'lz4 lone encode' gpurun_out/ls_$kb.log)" >> gpurun_out/ls_sum.log
done
cat gpurun_out/ls_sum.log
