"""LZ4 encoder phase shares from libjfsgpu_prof.so (s_memtime ticks summed
over the encoder waves).  usage: eprof.py [N]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JFS_GPU_LIB"] = os.environ.get("PROF_LIB") or os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
import torch
from juicefs_amd import _lib, device as D
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
b = D.Lz4Batch(n, 4 << 20, "T", seed_base=1)
lib.jfs_eprof_reset()
b.compress(); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 12)()
lib.jfs_eprof_read(buf)
names = ["search", "cand check", "catch-up", "literals", "offset+ext", "token+flush", "rematch"]
tot = sum(buf[:7])
print(f"blocks={n} encode {b.enc_ms:.1f} ms (this launch)")
for i, nm in enumerate(names):
    print(f"{nm:12s} {buf[i] / tot * 100:6.2f}%  {buf[i] / n / 1e6:8.2f} Mcyc/block")
m = max(buf[8], 1)
print(f"per block: tokens {buf[8] / n:.0f}  search steps {buf[7] / n:.0f}  cand checks {buf[9] / n:.0f}  rematches {buf[10] / n:.0f}")
print(f"per token: {tot / m:.0f} cycles  search steps {buf[7] / m:.2f}")
