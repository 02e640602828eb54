"""Segment-parallel LZ4 encode (jfs_lz4_compress_device_small) against the
serial kernel (jfs_lz4_compress_device): time per launch and byte equality.
NLIST = block counts, CLS = data classes, U = block bytes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from juicefs_amd import device as D  # noqa: E402

U = int(os.environ.get("U", 4 << 20))
for cls in os.environ.get("CLS", "T").split(","):
    for nblk in [int(x) for x in os.environ.get("NLIST", "1,8,64").split(",")]:
        b = D.Lz4Batch(nblk, U, cls, seed_base=1)
        comp2 = torch.zeros_like(b.comp)
        offs = np.arange(nblk, dtype=np.int64)
        desc = D.make_desc(b.raw, offs * U, [U] * nblk, comp2, offs * b.slot, [b.slot] * nblk)
        ret = torch.zeros(nblk, dtype=torch.int32, device=b.device)
        D.lz4_eseg_counts(reset=True)
        best = 1e30
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            D.lz4_compress_small(desc, ret, [U] * nblk)
            e1.record()
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        cnt = D.lz4_eseg_counts()
        r = ret.cpu().numpy().astype(np.int64)
        same = bool((r == b.csize).all())
        if same:
            for i in range(nblk):
                n = int(r[i])
                if not torch.equal(comp2[i * b.slot:i * b.slot + n], b.comp[i * b.slot:i * b.slot + n]):
                    same = False
                    print(f"  block {i}: bytes differ", flush=True)
                    break
        else:
            bad = np.nonzero(r != b.csize)[0][:4]
            print(f"  sizes differ at {bad.tolist()}: {r[bad].tolist()} vs {b.csize[bad].tolist()}", flush=True)
        print(f"{cls} {nblk:5d} x {U >> 10} KiB: segment {best:8.2f} ms ({nblk * U / 2**30 / (best / 1e3):6.2f} GiB/s)"
              f"  serial {b.enc_ms:8.2f} ms  identical={same}  settled-after-rounds={cnt}", flush=True)
        del b, comp2
        torch.cuda.empty_cache()
