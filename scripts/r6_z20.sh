#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_HOST_TRACE=1 scripts/gpu_step.sh 200 z20.log python -u scripts/r6_z20.py || exit 1
scripts/gpu_step.sh 200 z20_kt.log rocprofv3 --kernel-trace -d gpurun_out/z20_kt -o run -- python -u scripts/r6_z20.py || exit 1
f=$(find gpurun_out/z20_kt -name "*.db" | head -1)
python - "$f" > gpurun_out/z20_timeline.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
t0 = rows[0][1]
for n, s, e in rows:
    nm = n.split('(')[0][-34:]
    if 'zl1' in nm or 'copy' in nm.lower():
        print(f"{(s - t0) / 1e6:10.3f} ms  {nm:36s} {(e - s) / 1e6:8.3f} ms")
PY
grep burst gpurun_out/z20.log
