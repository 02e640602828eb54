#!/bin/bash
# zexec instruction mix + time per library variant (Zstd configs[3], one launch per PMC pass)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib JFS_ZSTD_DBG=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY -d /tmp/zv_$v -o p --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > gpurun_out/zv_$v.log 2>&1 || exit 1
  f=$(find /tmp/zv_$v -name '*counter_collection.csv' | head -1)
  python - "$f" "$v" <<'PY'
import csv, sys, collections
d = collections.defaultdict(float); t = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "zexec_kernel" in k:
        d[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[2], " ".join(f"{c}={v/1e9:.2f}G" for c, v in sorted(d.items())))
PY
done
