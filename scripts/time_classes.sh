#!/bin/bash
# LZ4 decode launch time per data class (N blocks) for library variants ("base" = libjfsgpu.so).
# usage: scripts/time_classes.sh N "T Z R" name...
cd "$GRAFT_REPO_ROOT"
n=$1; cls=$2; shift 2
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for c in $cls; do
    r=$(JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py $n 3 $c 2>/dev/null | head -2 | tr '\n' ' ') || exit 1
    echo "$v $c $r"
  done
done
