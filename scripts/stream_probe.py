"""How many kernels on distinct streams run side by side in one process?
Launches the LZ4 encode kernel (one 4 MiB block per launch, ~0.5 s) on k
streams at once and reports the wall time; concurrent streams finish in one
block's time, streams that share a hardware queue serialise."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from juicefs_amd import device as D  # noqa: E402

U = 4 << 20
dev = torch.device("cuda:0")
n = 8
raw = torch.empty(n * U, dtype=torch.uint8, device=dev)
D.gen_blocks(raw, n, U, "T", 5)
bound = U + U // 255 + 16
comp = torch.empty(n * bound, dtype=torch.uint8, device=dev)
descs = [D.make_desc(raw, [i * U], [U], comp, [i * bound], [bound]) for i in range(n)]
rets = [torch.zeros(1, dtype=torch.int32, device=dev) for _ in range(n)]
print("GPU_MAX_HW_QUEUES", os.environ.get("GPU_MAX_HW_QUEUES"), flush=True)
streams = [torch.cuda.Stream() for _ in range(n)]
D.lz4_compress(descs[0], rets[0])
torch.cuda.synchronize()
for k in (1, 2, 3, 4, 5, 6, 8):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(k):
        D.lz4_compress(descs[i], rets[i], streams[i])
    torch.cuda.synchronize()
    print(f"k={k} streams: {1e3 * (time.perf_counter() - t0):.0f} ms", flush=True)
