#!/bin/bash
# Kernel split of a lone 4 MiB Zstd frame decode (device path), and of 32 frames.
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
timeout -k 10 300 python scripts/prof_run.py 4096 0 T zstd > /dev/null 2>&1 && timeout -k 10 300 python scripts/prof_run.py 1 0 T zstd > /dev/null 2>&1 || exit 1
for nb in 1 32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/zl$nb -o zl --output-format csv -- python scripts/prof_run.py $nb 5 T zstd > gpurun_out/zl$nb.log 2>&1 || exit 1
  find gpurun_out/zl$nb -name '*kernel_stats.csv' -exec cp {} gpurun_out/zlone_$nb.csv \;
done
