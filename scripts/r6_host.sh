#!/bin/bash
# host-path checks: batch / coalescer / one-call tests, lone latency, the
# bench's one-call concurrency leg
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
scripts/gpu_step.sh 600 ht.log python -u -m pytest tests/test_host_pipeline_gpu.py tests/test_coalescer_gpu.py tests/test_batch_gpu.py tests/test_lz4_gpu.py tests/test_encrypt_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q "passed" gpurun_out/ht.log && ! grep -q "failed" gpurun_out/ht.log || { echo "TESTS FAILED"; tail -30 gpurun_out/ht.log; exit 1; }
JFS_HOST_TRACE=1 scripts/gpu_step.sh 120 lone.log python -u scripts/r6_lone.py 15 0 || exit 1
scripts/gpu_step.sh 120 lone2.log python -u scripts/r6_lone.py 15 0.02 || exit 1
scripts/gpu_step.sh 300 osc.log python -u scripts/oneshot.py || exit 1
grep -E "passed" gpurun_out/ht.log; grep "lone decode" gpurun_out/lone.log gpurun_out/lone2.log
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/osc.log") if l.startswith("{")][-1])
for k in ("decompress_lone", "compress_lone", "decompress_200_concurrent", "decompress_200_concurrent_native", "compress_20_concurrent"):
    v = d.get(k, {}); print(k, {x: round(v[x], 3) for x in ("value", "p50_ms", "p99_ms") if x in v})
z = d.get("zstd", {})
for k in ("decompress_lone", "compress_lone", "decompress_20_concurrent", "compress_20_concurrent"):
    v = z.get(k, {}); print("zstd", k, {x: round(v[x], 3) for x in ("value", "p50_ms", "p99_ms") if x in v})
PY
