"""Straggler check for the LZ4 headline: decode time of the mixed batch vs
batches whose 4096 entries all point at one compressed block (the smallest,
largest and a few sampled blocks by compressed size).
usage: r5_lz4_uniform.py [N]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch
from juicefs_amd import device as D

nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
b = D.Lz4Batch(nblk, 4 << 20, "T", seed_base=1)
U = 4 << 20


def timeit(desc, k=5):
    ret = torch.empty(nblk, dtype=torch.int32, device="cuda")
    D.lz4_decompress(desc, ret)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(k):
        D.lz4_decompress(desc, ret)
    e1.record()
    torch.cuda.synchronize()
    assert (ret.cpu().numpy() == U).all()
    return e0.elapsed_time(e1) / k


offs = np.arange(nblk, dtype=np.int64)
print(f"mixed: {timeit(b.dec_desc):.2f} ms  csize min/mean/max {b.csize.min()}/{b.csize.mean():.0f}/{b.csize.max()}")
order = np.argsort(b.csize)
for q in (0, 0.25, 0.5, 0.75, 1.0):
    i = int(order[min(nblk - 1, int(q * (nblk - 1)))])
    d = D.make_desc(b.comp, np.full(nblk, i * b.slot), [int(b.csize[i])] * nblk, b.out, offs * U, [U] * nblk)
    print(f"uniform q={q:.2f} block {i} csize {b.csize[i]}: {timeit(d):.2f} ms")
