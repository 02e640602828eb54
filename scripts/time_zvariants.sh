#!/bin/bash
# Wall time per configs[3] Zstd decode launch (4096 frames, 256 distinct) for library variants
# usage: scripts/time_zvariants.sh name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  r=$(JFS_GPU_LIB=$lib timeout -k 10 120 python scripts/prof_run.py 4096 5 T zstd | sed -n 1p) || exit 1
  echo "$v $r"
done
