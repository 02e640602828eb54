#!/bin/bash
# Zstd decode kernel split (rocprofv3 kernel stats) + instruction mix per kernel, for one library
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/zp
lib=${1:-juicefs_amd/lib/libjfsgpu.so}
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 || exit 1
JFS_GPU_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/zkt -o kt --output-format csv -- python scripts/prof_run.py 4096 3 T zstd > gpurun_out/zp/kt.log 2>&1 || exit 1
f=$(find /tmp/zkt -name '*kernel_stats.csv' | head -1); cp $f gpurun_out/zp/kernel_stats.csv
grep zstdd $f | awk -F'","' '{print $1, $4}' | sed 's/(.*"/ /' | cut -c1-120
JFS_GPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY -d /tmp/zpmc -o p --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > gpurun_out/zp/pmc.log 2>&1 || exit 1
f=$(find /tmp/zpmc -name '*counter_collection.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
d = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Kernel_Name"]
    if "zstdd::" in k:
        d[(k.split("zstdd::")[1].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
for (k, c), v in sorted(d.items()):
    print(f"{k:16s} {c:16s} {v/1e9:9.3f} G")
PY
