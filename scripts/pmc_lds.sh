#!/bin/bash
# LDS bank-conflict counters of the LZ4 decode kernel per library variant.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d gpurun_out/lds_$v -o l --output-format csv -- python scripts/prof_run.py 4096 1 T > gpurun_out/lds_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/lds_$v -name '*counter_collection.csv' | head -1)
  echo "== $v"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lz4_decode' in r['Kernel_Name']: print(r['Counter_Name'], r['Counter_Value'])
"
done
