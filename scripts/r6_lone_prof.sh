#!/bin/bash
# kernel timeline of lone one-call decodes (LZ4 + Zstd), rocprofv3 kernel trace
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 200 lp.log rocprofv3 --kernel-trace --stats -d gpurun_out/lp -o run -- python -u scripts/r6_lone.py 15 0 || exit 1
f=$(find gpurun_out/lp -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/lone_kstats.csv
python - "$f" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
# the last LZ4 lone call: find the last 'lz4s' / split kernels sequence
t = [(r[0].split('(')[0][:40], r[1], r[2]) for r in rows]
last = t[-400:]
prev = None
for n, s, e in last[-60:]:
    gap = (s - prev) / 1e3 if prev else 0
    print(f"{n:42s} dur {((e - s) / 1e3):8.1f} us  gap {gap:7.1f} us")
    prev = e
PY
