#!/bin/bash
# the bench's one-call leg alone (scripts/oneshot.py) with and without byte pieces, twice
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
rm -f gpurun_out/bp2_sum.log
for r in 1 2; do for n in 4 0; do
  JFS_BYTE_PIECES=$n scripts/gpu_step.sh 300 bp2_$n.log python -u scripts/oneshot.py || exit 1
  python - "$n" >> gpurun_out/bp2_sum.log <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/bp2_{n}.log") if l.startswith("{")][-1])
print(f"pieces {n}: lz4 lone {d['decompress_lone']['p50_ms']:.3f} (p99 {d['decompress_lone']['p99_ms']:.3f}) zstd lone {d['zstd']['decompress_lone']['p50_ms']:.3f} py200 {d['decompress_200_concurrent']['value']:.2f} native200 {d['decompress_200_concurrent_native']['value']:.2f}")
PY
done; done
cat gpurun_out/bp2_sum.log
