#!/bin/bash
# the full bench with and without lone-block byte pieces: the one-call lone legs inside the bench process
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
for n in 4 0; do
  JFS_BYTE_PIECES=$n timeout -k 10 900 python bench.py > gpurun_out/bp3_$n.json 2> gpurun_out/bp3_$n.err || exit 1
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/bp3_{n}.json") if l.startswith("{")][-1])["summary"]
print("pieces", n, "lz4 lone", d["oneshot_lz4"]["dec_lone_p50_ms"], "zstd lone", d["oneshot_zstd"]["dec_lone_p50_ms"], "py200", d["oneshot_lz4"]["dec200_GiBs"], "native200", d["oneshot_lz4"]["dec200_native_GiBs"])
PY
done
