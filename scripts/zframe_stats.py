"""Composition of GPU-encoded Zstd frames (diagnostics): bytes per block in
literal sections by type and in sequence sections; compare with libzstd-1."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
from juicefs_amd import device as D
from juicefs_amd.blockgen import gen_block


def stats(f):
    p = 4
    fhd = f[p]; p += 1
    single = (fhd >> 5) & 1
    if not single: p += 1
    fcs = {0: (1 if single else 0), 1: 2, 2: 4, 3: 8}[fhd >> 6]
    p += fcs
    st = {"raw_lit": 0, "rle_lit": 0, "huf_lit": 0, "treeless": 0, "lit_bytes_in": 0, "seq_bytes": 0, "nseq": 0,
          "raw_blocks": 0, "blocks": 0, "hdr": 0}
    while True:
        bh = f[p] | (f[p + 1] << 8) | (f[p + 2] << 16); p += 3
        last, bt, bs = bh & 1, (bh >> 1) & 3, bh >> 3
        st["blocks"] += 1
        if bt == 0:
            st["raw_blocks"] += 1; p += bs
        elif bt == 1:
            p += 1
        else:
            b = f[p:p + bs]
            lt, sf = b[0] & 3, (b[0] >> 2) & 3
            if lt <= 1:
                hs = 1 if sf in (0, 2) else (2 if sf == 1 else 3)
                rg = (b[0] >> 3) if hs == 1 else ((b[0] | b[1] << 8) >> 4 if hs == 2 else (b[0] | b[1] << 8 | b[2] << 16) >> 4)
                sec = hs + (rg if lt == 0 else 1)
                st["raw_lit" if lt == 0 else "rle_lit"] += sec
            else:
                hs = 3 if sf <= 1 else (4 if sf == 2 else 5)
                v = int.from_bytes(bytes(b[:hs]), "little")
                bits = 10 if sf <= 1 else (14 if sf == 2 else 18)
                rg = (v >> 4) & ((1 << bits) - 1); cs = (v >> (4 + bits)) & ((1 << bits) - 1)
                sec = hs + cs
                st["huf_lit" if lt == 2 else "treeless"] += sec
            st["lit_bytes_in"] += rg
            st["seq_bytes"] += bs - sec
            ns = b[sec]
            if ns >= 128:
                ns = ((ns - 128) << 8) + b[sec + 1] if ns < 255 else b[sec + 1] + (b[sec + 2] << 8) + 0x7F00
            st["nseq"] += ns
            p += bs
        if last: break
    return st


srcs = [gen_block("T", 900 + i, 4 << 20) for i in range(2)]
dev = torch.device("cuda:0")
src = torch.from_numpy(np.frombuffer(b"".join(srcs), dtype=np.uint8).copy()).to(dev)
cap = (4 << 20) + (4 << 12) + 64
dst = torch.zeros(2 * cap, dtype=torch.uint8, device=dev)
desc = D.make_desc(src, [0, 4 << 20], [4 << 20] * 2, dst, [0, cap], [cap] * 2)
ret = torch.zeros(2, dtype=torch.int32, device=dev)
D.zstd_compress(desc, ret)
torch.cuda.synchronize()
r = ret.cpu().tolist()
h = dst.cpu().numpy()
for i in range(2):
    print("GPU", r[i], stats(bytes(h[i * cap:i * cap + r[i]])))
z = D._libzstd()
for lvl in (1, 3):
    out = ctypes.create_string_buffer(cap)
    n = z.ZSTD_compress(out, cap, srcs[0], len(srcs[0]), lvl)
    print(f"libzstd-{lvl}", n, stats(out.raw[:n]))
