"""LZ4 encode launch time (device-resident, byte-identical to LZ4_compress_default)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import device as D
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cls = sys.argv[2] if len(sys.argv) > 2 else "T"
b = D.Lz4Batch(nblk, 4 << 20, cls, seed_base=1)
for _ in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); b.compress(); e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
print(f"encode {nblk} x 4 MiB {cls}: {ms:.1f} ms  {nblk * 4 / 1024 / (ms / 1e3):.2f} GiB/s  (first launch {b.enc_ms:.1f} ms)")
b.decompress()
assert b.verify()
print("round trip ok")
