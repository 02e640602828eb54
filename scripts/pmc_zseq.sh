#!/bin/bash
# Instruction mix / waits of the Zstd sequence kernels (one PMC pass).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python scripts/prof_run.py 4096 0 T zstd || exit 1
JFS_NOVERIFY=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM -d /tmp/pmcz -o p --output-format csv -- python scripts/prof_run.py 4096 1 T zstd > gpurun_out/pmcz.log 2>&1 || exit 1
f=$(find /tmp/pmcz -name '*counter_collection.csv' | head -1)
python - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'].split('(')[0]
    if 'zstdd' in k: agg[(k, r['Counter_Name'])] += float(r['Counter_Value'])
for (k, c), v in sorted(agg.items()): print(f"{k:30s} {c:22s} {v/1e9:10.3f} G")
PY
