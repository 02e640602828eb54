#!/bin/bash
# rounds to settle of the segment-parallel LZ4 encode at 16 / 32 KiB minimum segments
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for kb in 16 32 64; do
  JFS_LZ4E_SEG_MIN_KB=$kb CLS=T,Z,R NLIST=1,8,32 scripts/gpu_step.sh 300 l2_$kb.log python -u scripts/eseg_timing.py || exit 1
done
for kb in 16 32 64; do echo "== $kb KiB"; grep -E "KiB:" gpurun_out/l2_$kb.log; done
