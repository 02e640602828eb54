#!/bin/bash
# LZ4 encode rate (4,096 x 4 MiB text) of library variants: scripts/lenc_variants.sh name...  ("base" = libjfsgpu.so)
cd "$GRAFT_REPO_ROOT"
for v in "$@"; do
  if [ "$v" = base ]; then lib=juicefs_amd/lib/libjfsgpu.so; else lib=juicefs_amd/lib/libjfsgpu_$v.so; fi
  JFS_GPU_LIB=$lib timeout -k 10 200 python -c "
import torch
from juicefs_amd import device as D
b = D.Lz4Batch(4096, 4 << 20, 'T', seed_base=1)
c0 = b.comp.clone()
for i in range(3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); b.compress(); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print('$v', round(4096 * 4 / 1024 / (ms / 1e3), 2), 'GiB/s', round(ms, 1), 'ms', 'same' if torch.equal(b.comp, c0) else 'DIFF', flush=True)
" || exit 1
done
