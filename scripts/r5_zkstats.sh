#!/bin/bash
# Per-kernel times (rocprofv3 kernel stats) of the configs[3] Zstd decode for library variants
# usage: scripts/r5_zkstats.sh name...   ("base" = libjfsgpu.so); JFS_NOVERIFY=1 for diagnostic variants
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/zks_$v -o zks --output-format csv -- python scripts/prof_run.py 4096 3 T zstd > gpurun_out/zks_$v.log 2>&1 || exit 1
  f=$(find /tmp/zks_$v -name '*kernel_stats.csv' | head -1)
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    n=r['Name']
    if 'zstdd' in n: print('  %-14s %8.2f ms' % (n.split('zstdd::')[1].split('(')[0], float(r['AverageNs'])/1e6))
" "$f"
done
