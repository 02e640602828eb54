#!/bin/bash
# decode gather gap (JFS_GATHER_US decode part): the one-call legs at 300 (default) / 600 / 1000 us, twice
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -f gpurun_out/ga_sum.log
for r in 1 2; do for g in 300 600 1000; do
  JFS_GATHER_US=$g,2000 scripts/gpu_step.sh 300 ga_$g.log python -u scripts/oneshot.py || exit 1
  python - "$g" >> gpurun_out/ga_sum.log <<'PY'
import json, sys
g = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/ga_{g}.log") if l.startswith("{")][-1])
p = d["decompress_200_concurrent"]; n = d["decompress_200_concurrent_native"]; z = d["zstd"]["decompress_20_concurrent"]
print(f"gap {g}: py200 {p['value']:.2f} GiB/s p99 {p['p99_ms']:.1f} batches {p['device_batches']} | native200 {n['value']:.2f} p99 {n['p99_ms']:.1f} | lone {d['decompress_lone']['p50_ms']:.3f} | zstd20 {z['value']:.2f}")
PY
done; done
cat gpurun_out/ga_sum.log
