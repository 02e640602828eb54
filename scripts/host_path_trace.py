"""Diagnostic: one traced LZ4 host batch (JFS_HOST_TRACE=1 prints per-chunk
stage-in / wait / copy-out times)."""
import os, sys, time
os.environ.setdefault("JFS_HOST_TRACE", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import compress as C, device as D
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
U = 4 << 20
b = D.Lz4Batch(64, U, "T", seed_base=1)
comp = [b.comp[i * b.slot:i * b.slot + int(b.csize[i])].cpu().numpy().tobytes() for i in range(64)]
srcs = (comp * (nblk // 64 + 1))[:nblk]
pairs = [(bytearray(U), s) for s in srcs]
c = C.LZ4()
for rep in range(2):
    t0 = time.perf_counter()
    res = c.DecompressBatch(pairs)
    dt = time.perf_counter() - t0
    print(f"rep {rep}: {nblk} blocks {dt*1e3:.1f} ms  {nblk*U/dt/2**30:.2f} GiB/s", file=sys.stderr, flush=True)
