"""Diagnostic: LZ4 decode of 4096 blocks whose compressed inputs are only
`ndistinct` distinct blocks (input lines L2/MALL-resident) vs all distinct.
usage: r5_shared_src.py [ndistinct ...]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from juicefs_amd import device as D
nblk = 4096
full = D.Lz4Batch(nblk, 4 << 20, "T", seed_base=1)
def run(desc, ret, k=5):
    D.lz4_decompress(desc, ret); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k): D.lz4_decompress(desc, ret)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k
dt = run(full.dec_desc, full.dec_ret)
print(f"distinct={nblk}: {dt*1e3:.2f} ms  {nblk*4/1024/dt:.1f} GiB/s")
offs = np.arange(nblk, dtype=np.int64)
for nd in [int(a) for a in sys.argv[1:]] or [1, 16, 256]:
    src = (offs % nd) * full.slot
    desc = D.make_desc(full.comp, src, full.csize[offs % nd], full.out, offs * full.U, [full.U] * nblk)
    ret = torch.empty(nblk, dtype=torch.int32, device="cuda")
    dt = run(desc, ret)
    ok = bool((ret == full.U).all().item())
    print(f"distinct={nd}: {dt*1e3:.2f} ms  {nblk*4/1024/dt:.1f} GiB/s ok={ok}")
