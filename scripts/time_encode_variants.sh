#!/bin/bash
# LZ4 encode launch time (4096 text blocks) for library variants ("base" = libjfsgpu.so).
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/time_encode.py 4096 T 2>/dev/null | head -1) || exit 1
  echo "$v $r"
done
