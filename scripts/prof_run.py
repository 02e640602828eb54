"""Minimal decode run for rocprofv3 (no CPU legs): N blocks, K launches.
usage: prof_run.py [N] [K] [cls] [codec]   (codec: lz4 | zstd)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import device as D
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
k = int(sys.argv[2]) if len(sys.argv) > 2 else 2
cls = sys.argv[3] if len(sys.argv) > 3 else "T"
codec = sys.argv[4] if len(sys.argv) > 4 else "lz4"
if codec == "lz4":
    b = D.Lz4Batch(nblk, 4 << 20, cls, seed_base=1)
else:
    b = D.ZstdBatch(nblk, 4 << 20, cls, level=3, distinct=256, seed_base=1,
                    cache_dir=os.path.join(os.environ.get("TMPDIR", "/tmp"), "jfs_frames"))
if k == 0:  # generate the frame cache only (no GPU work)
    print("cached"); sys.exit(0)
import time
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(k):
    b.decompress()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / max(k, 1)
print(f"{dt*1e3:.2f} ms/launch  {nblk*4/1024/dt:.1f} GiB/s")
ok = b.verify()
if not (os.environ.get("JFS_ZSTD_DBG") or os.environ.get("JFS_NOVERIFY")): assert ok
print("ok", codec, nblk, b.comp_bytes)
