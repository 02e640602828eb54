#!/bin/bash
# Wall time per LZ4 decode launch (4096 text blocks) for library variants,
# without output verification (diagnostic variants skip phases).
# usage: scripts/time_variants.sh name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  r=$(JFS_GPU_LIB=$lib JFS_NOVERIFY=1 timeout -k 10 120 python scripts/prof_run.py 4096 5 T | sed -n 1p) || exit 1
  echo "$v $r"
done
