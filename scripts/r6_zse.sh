#!/bin/bash
# Zstd split parity + lone decode kernel times; then the GPU suite twice (flakiness) and smoke
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/r6_zsblk.sh || exit 1
python scripts/rocpd_stats.py $(find gpurun_out/zs_lp -name "*.db" | head -1) gpurun_out/zs_lone_kstats.csv
bash scripts/r6_flaky.sh || exit 1
