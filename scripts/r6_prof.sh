#!/bin/bash
# Round 6: phase stamps (prof build) of the LZ4 decoder with the chain bitmap
# on and off, and one PMC instruction-mix pass of every LZ4 kernel (chain on).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for ch in 1 0; do
  JFS_LZ4_CHAIN=$ch scripts/gpu_step.sh 120 prof_$ch.log python scripts/prof_decode.py 4096 T || exit 1
done
JFS_NOVERIFY=1 scripts/gpu_step.sh 120 pmc.log rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM -d gpurun_out/pmc_r6 -o p --output-format csv -- python scripts/prof_run.py 4096 1 T || exit 1
f=$(find gpurun_out/pmc_r6 -name '*counter_collection.csv' | head -1)
python scripts/pmc_summary.py "$f" --kernel lz4 > gpurun_out/pmc_sum.txt
cat gpurun_out/prof_1.log gpurun_out/prof_0.log gpurun_out/pmc_sum.txt
