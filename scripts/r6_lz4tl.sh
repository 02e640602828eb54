#!/bin/bash
# lone LZ4 one-call decode: kernel + memory-copy timeline of the last calls
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
JFS_LONE_CODECS=lz4 JFS_LONE_ENC=0 scripts/gpu_step.sh 200 tl.log rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl -o run -- python -u scripts/r6_lone.py 9 0.005 || exit 1
f=$(find gpurun_out/tl -name "*.db" | head -1)
python - "$f" > gpurun_out/lz4_tl.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
tabs = [r[0] for r in c.execute("select name from sqlite_master where type in ('table','view')")]
print(tabs)
ev = [(r[1], r[2], r[0].split('(')[0][-36:]) for r in c.execute("select name, start, end from kernels")]
for t in tabs:
    if 'memory_copies' in t or t == 'memory_copies':
        cols = [r[1] for r in c.execute(f"pragma table_info({t})")]
        print(t, cols)
        try:
            for r in c.execute(f"select start, end, size, direction from {t}"):
                ev.append((r[0], r[1], f"COPY {r[3]} {r[2]}"))
        except Exception as e:
            print(e)
        break
ev.sort()
last = ev[-80:]
prev = None
for s, e, n in last:
    print(f"{n:44s} dur {(e - s) / 1e3:8.1f} us  gap {((s - prev) / 1e3 if prev else 0):8.1f} us")
    prev = e
PY
grep "lone decode" gpurun_out/tl.log
