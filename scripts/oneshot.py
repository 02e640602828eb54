"""Time bench.py's oneshot_concurrency leg alone (the one-call API under
pkg/chunk's concurrency) on 32 distinct 4 MiB text blocks."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from juicefs_amd import device as D  # noqa: E402

U = 4 << 20
dev = torch.device("cuda:0")
b = D.Lz4Batch(32, U, "T", seed_base=1, device=dev)
comp = [b.comp[i * b.slot:i * b.slot + int(b.csize[i])].cpu().numpy().tobytes() for i in range(32)]
raw = [b.raw[i * U:(i + 1) * U].cpu().numpy().tobytes() for i in range(32)]
del b
torch.cuda.synchronize()
print(json.dumps(bench.oneshot_concurrency(comp, raw, U)), flush=True)
