#!/bin/bash
# instruction mix of the lone-frame Zstd kernels (zsblk's serial state pass)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM -d gpurun_out/zpmc -o p --output-format csv -- python scripts/r6_lone.py 5 0 > gpurun_out/zpmc.log 2>&1 || exit 1
f=$(find gpurun_out/zpmc -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" --kernel zsblk
