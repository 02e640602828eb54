#!/bin/bash
# Instruction mix of the LZ4 decode kernel for library variants (one PMC pass each).
# usage: scripts/pmc_insts.sh name...   ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib JFS_NOVERIFY=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM -d gpurun_out/pmc_$v -o p --output-format csv -- python scripts/prof_run.py 4096 1 T > gpurun_out/pmc_$v.log 2>&1 || exit 1
  f=$(find gpurun_out/pmc_$v -name '*counter_collection.csv' | head -1)
  echo "== $v"; grep lz4_decode_kernel "$f" | awk -F, '{print $(NF-3), $(NF-2)}'
done
