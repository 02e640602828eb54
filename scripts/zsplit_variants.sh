#!/bin/bash
# zsblk kernel time of library variants on a lone 4 MiB frame and on 32:
# scripts/zsplit_variants.sh name...  ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp JFS_NOVERIFY=1
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 && timeout -k 10 300 python scripts/prof_run.py 1 0 T zstd > /dev/null 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  for nb in 1 32; do
    JFS_GPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zv_${v}_$nb -o zv --output-format csv -- python scripts/prof_run.py $nb 5 T zstd > gpurun_out/zv_${v}_$nb.log 2>&1 || exit 1
    f=$(find gpurun_out/zv_${v}_$nb -name '*kernel_stats.csv' | head -1)
    python3 -c "import csv,sys; [print(sys.argv[2], sys.argv[3], round(float(r[\"AverageNs\"])/1e3,1), \"us\") for r in csv.DictReader(open(sys.argv[1])) if \"zsblk\" in r[\"Name\"]]" $f $v $nb
  done
done
