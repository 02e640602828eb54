#!/bin/bash
# 200 concurrent one-call LZ4 decodes under coalescer settings (2 runs each):
#   scripts/concur_sweep.sh "ENV=..." ...   ("" = defaults)
cd "$GRAFT_REPO_ROOT"
for cfg in "$@"; do
  for r in 1 2; do
    env $cfg timeout -k 10 200 python scripts/concur.py 200 2 > gpurun_out/cs.json || exit 1
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))['decompress_200_concurrent']
print(repr(sys.argv[2]), round(d['value'],2), 'GiB/s p50', round(d['p50_ms'],1), 'p99', round(d['p99_ms'],1), 'batches', d['device_batches'], flush=True)" gpurun_out/cs.json "$cfg"
  done
done
