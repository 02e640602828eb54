#!/bin/bash
# LZ4 decode diagnostics on the GPU box: phase stamps (prof build) + one PMC pass.
# usage: scripts/prof_lz4.sh [nblk]
set -e
N=${1:-2048}
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/prof_decode.py $N T > gpurun_out/phases.txt 2>&1
cat gpurun_out/phases.txt
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM -d gpurun_out/pmc1 -o pmc1 --output-format csv -- python scripts/prof_run.py $N 1 T > gpurun_out/pmc1.log 2>&1
f=$(find gpurun_out/pmc1 -name '*counter_collection.csv' | head -1)
grep lz4_decode_kernel "$f" | awk -F, '{print $(NF-3), $(NF-2)}'
