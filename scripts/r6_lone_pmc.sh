#!/bin/bash
# instruction mix and wait share of the lone LZ4 split-path kernels (21 lone decodes)
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out/lpmc
T=/tmp/lpmc; mkdir -p $T
SQC="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM"
JFS_LONE_CODECS=lz4 JFS_LONE_ENC=0 timeout -s KILL 90 rocprofv3 --pmc $SQC -d $T/a -o a --output-format csv -- python scripts/r6_lone.py 21 > gpurun_out/lpmc/a.log 2>&1 || exit 1
python scripts/pmc_summary.py $(find $T/a -name '*counter_collection.csv' | head -1) --kernel lz4s > gpurun_out/lpmc/a.txt
JFS_LONE_CODECS=lz4 JFS_LONE_ENC=0 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM -d $T/b -o b --output-format csv -- python scripts/r6_lone.py 21 > gpurun_out/lpmc/b.log 2>&1 || exit 1
python scripts/pmc_summary.py $(find $T/b -name '*counter_collection.csv' | head -1) --kernel lz4s > gpurun_out/lpmc/b.txt
cat gpurun_out/lpmc/a.txt gpurun_out/lpmc/b.txt
