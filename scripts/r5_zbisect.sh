#!/bin/bash
# one Zstd decode test file per library variant (bisecting a parity failure)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
t=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -k 10 200 python -u -m pytest $t -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/zb_$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/zb_$v.log)"
done
