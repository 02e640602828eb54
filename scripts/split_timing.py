"""Kernel time of the small-batch LZ4 decoder (jfs_lz4_decompress_device_small)
vs the one-workgroup-per-block kernel (jfs_lz4_decompress_device) for 1..128
device-resident 4 MiB text blocks; every output verified."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from juicefs_amd import device as D  # noqa: E402

U = 4 << 20
dev = torch.device("cuda:0")
NMAX = int(os.environ.get("NMAX", "128"))
b = D.Lz4Batch(NMAX, U, os.environ.get("CLS", "T"), seed_base=3, device=dev)
csize = [int(x) for x in b.csize]


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) / reps


D.lz4_split_counts(reset=True)
NLIST = [int(x) for x in os.environ.get("NLIST", "1,2,4,8,16,32,64,128").split(",")]
for nb in NLIST:
    if nb > NMAX:
        break
    offs = np.arange(nb, dtype=np.int64)
    out = torch.zeros(nb * U, dtype=torch.uint8, device=dev)
    desc = D.make_desc(b.comp, offs * b.slot, csize[:nb], out, offs * U, [U] * nb)
    ret = torch.zeros(nb, dtype=torch.int32, device=dev)
    t_small = timed(lambda: D.lz4_decompress_small(desc, ret, csize[:nb], [U] * nb))
    ok_small = bool((ret == U).all().item()) and torch.equal(out, b.raw[:nb * U])
    out.zero_()
    ret.zero_()
    t_big = timed(lambda: D.lz4_decompress(desc, ret))
    ok_big = bool((ret == U).all().item()) and torch.equal(out, b.raw[:nb * U])
    cnt = D.lz4_split_counts(reset=True)
    print(f"nb={nb:4d} counts {cnt}", flush=True)
    print(f"nb={nb:4d}  small {t_small:8.3f} ms ({nb * U / t_small / 1e6:7.1f} GB/s) ok={ok_small}   "
          f"one-WG {t_big:8.3f} ms ({nb * U / t_big / 1e6:7.1f} GB/s) ok={ok_big}", flush=True)
print("split counts (decoded, handed over):", D.lz4_split_counts(), flush=True)
