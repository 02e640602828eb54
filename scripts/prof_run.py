"""Minimal decode run for rocprofv3 (no CPU legs): N blocks, K launches."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import device as D
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cls = sys.argv[3] if len(sys.argv) > 3 else "T"
b = D.Lz4Batch(nblk, 4 << 20, cls, seed_base=1)
for _ in range(k):
    b.decompress()
torch.cuda.synchronize()
assert b.verify()
print("ok", nblk, b.comp_bytes)
