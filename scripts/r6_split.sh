#!/bin/bash
# small-batch LZ4 decoder: parity tests, lone latency, lone kernel timeline
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 400 st.log python -u -m pytest tests/test_lz4_split_gpu.py tests/test_lz4_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/st.log && ! grep -q "failed" gpurun_out/st.log || { echo "TESTS FAILED"; tail -30 gpurun_out/st.log; exit 1; }
scripts/gpu_step.sh 120 lone3.log python -u scripts/r6_lone.py 15 0 || exit 1
scripts/gpu_step.sh 200 lp.log rocprofv3 --kernel-trace --stats -d gpurun_out/lp2 -o run -- python -u scripts/r6_lone.py 15 0 || exit 1
f=$(find gpurun_out/lp2 -name "*.db" | head -1)
python scripts/rocpd_stats.py "$f" gpurun_out/lone_kstats2.csv
grep passed gpurun_out/st.log; grep "lone decode" gpurun_out/lone3.log
python3 - <<'PY'
import csv
rows = list(csv.reader(open("gpurun_out/lone_kstats2.csv")))
tot = {"lz4": 0, "zstd": 0}
for r in rows[1:]:
    name = r[0]
    key = "lz4" if ("lz4s::" in name or "lz4_decode" in name) else "zstd" if "zstdd::" in name else None
    if key:
        tot[key] += int(r[2])
        print(f"{name.split('(')[0]:40s} calls {int(r[1]):4d} us/decode {int(r[2]) / 15 / 1e3:8.1f}")
print({k: round(v / 15 / 1e3, 1) for k, v in tot.items()}, "us per lone decode (kernels)")
PY
python3 - "$f" <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
rows = c.execute("select name, start, end from kernels order by start").fetchall()
seq = [(r[0].split('(')[0], (r[2] - r[1]) / 1e3) for r in rows if 'lz4s::' in r[0]]
last = seq[-25:]
print(" | ".join(f"{n.split('::')[-1].replace('_kernel','')} {d:.1f}" for n, d in last))
PY
