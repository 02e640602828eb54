#!/bin/bash
# Zstd decode kernel times per library variant (rocprofv3 kernel stats).
# usage: scripts/zstd_kernel_variants.sh name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/prof_run.py 2048 0 T zstd > gpurun_out/zc.log 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib JFS_NOVERIFY=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/k_$v -o k --output-format csv -- python scripts/prof_run.py 2048 3 T zstd > gpurun_out/k_$v.log 2>&1 || exit 1
  echo "== $v"
  python3 -c "
import csv, glob, sys
f = glob.glob('gpurun_out/k_$v/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'zstdd::' in r['Name']:
        print(r['Name'].split('(')[0], round(float(r['AverageNs']) / 1e6, 2), 'ms')
"
done
