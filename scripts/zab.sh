#!/bin/bash
# configs[3] Zstd decode launch time of library variants: scripts/zab.sh name...  ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  echo -n "$v "; JFS_GPU_LIB=$lib timeout -k 10 200 python scripts/prof_run.py 4096 4 T zstd 2>&1 | grep "ms/launch" || exit 1
done
