#!/bin/bash
# Zstd level-1 encode rate of library variants: scripts/zenc_variants.sh N name...  ("base" = libjfsgpu.so)
N=$1; shift
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/time_zenc.py $N 2>&1 | tail -1 || exit 1
done
