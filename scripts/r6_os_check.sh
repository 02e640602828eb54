#!/bin/bash
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 300 osc.log python -u scripts/oneshot.py || exit 1
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/osc.log") if l.startswith("{")][-1])
print("lz4 lone", d["decompress_lone"]["calls"], round(d["decompress_lone"]["p50_ms"], 3), "zstd lone", d["zstd"]["decompress_lone"]["calls"], round(d["zstd"]["decompress_lone"]["p50_ms"], 3), "errors", d["decompress_lone"]["errors"] + d["zstd"]["decompress_lone"]["errors"])
PY
