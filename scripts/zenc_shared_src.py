"""Zstd level-1 encode of N frames that all read the SAME 4 MiB source (L2 /
MALL-friendly) vs N distinct sources: how much of the parse is source-miss
latency.  usage: zenc_shared_src.py [N]"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from juicefs_amd import device as D

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
U = 4 << 20
dev = torch.device("cuda")
raw = torch.empty(n * U, dtype=torch.uint8, device=dev)
D.gen_blocks(raw, n, U, "T", 7)
slot = (D.zstd_bound(U) + 255) // 256 * 256
comp = torch.empty(n * slot, dtype=torch.uint8, device=dev)
offs = np.arange(n, dtype=np.int64)
for name, so in (("distinct", offs * U), ("shared", offs * 0), ("distinct", offs * U)):
    desc = D.make_desc(raw, so, [U] * n, comp, offs * slot, [slot] * n)
    ret = torch.empty(n, dtype=torch.int32, device=dev)
    D.zstd_compress(desc, ret)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(); D.zstd_compress(desc, ret); e1.record(); torch.cuda.synchronize()
    print(name, n, round(e0.elapsed_time(e1), 1), "ms", flush=True)
