#!/bin/bash
# Zstd level-3 decode launch time (N 4 MiB text frames) for library variants ("base" = libjfsgpu.so).
# usage: scripts/time_zstd_variants.sh N name...
cd "$GRAFT_REPO_ROOT"
n=$1; shift
timeout -k 10 300 python scripts/prof_run.py $n 0 T zstd > /dev/null 2>&1 || exit 1   # frame cache (host libzstd)
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py $n 3 T zstd 2>/dev/null | head -2 | tr '\n' ' ') || exit 1
  echo "$v $r"
done
