#!/bin/bash
# Zstd level-1 encoder evidence: kernel-trace stats and PMC passes (instruction
# mix, waits, HBM bytes) of one 1,024 x 4 MiB text encode (time_zenc.py).
# Run from the repo root under gpurun.  Output: gpurun_out/zenc/.
set -e
export TMPDIR=/tmp
O=gpurun_out/zenc
T=/tmp/zenc
mkdir -p $O $T
N=${1:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/kt -o kt --output-format csv -- python scripts/time_zenc.py $N > $O/kt.log 2>&1
find $T/kt -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats.csv \;
i=0
for pmc in "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $pmc -d $T/p$i -o p --output-format csv -- python scripts/time_zenc.py $N > $O/p$i.log 2>&1
done
python scripts/pmc_summary.py $(find $T/p1 $T/p2 $T/p3 -name '*counter_collection.csv') --kernel zl1_ > $O/pmc_summary.txt
cat $O/pmc_summary.txt
echo zenc-done
