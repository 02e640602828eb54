"""Phase split of the Zstd level-1 parse kernel (prof build: JFS_GPU_LIB=juicefs_amd/lib/libjfsgpu_prof.so).
usage: zpprof.py [N]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from juicefs_amd import _lib as L, device as D
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1
lib = L.load()
lib.jfs_zpprof_reset()
r, ratio, ms = D.zstd_compress_rate(n, 4 << 20, "T", seed_base=7)  # warm-up + timed launch
buf = (ctypes.c_ulonglong * 12)()
lib.jfs_zpprof_read(buf)
v = list(buf)
names = ["positions+windows+hash", "after-match+rep loop", "table reads+tags", "candidates+decision",
         "table writes", "extension+emit", "block setup"]
tot = sum(v[:7])
print(f"{n} frames, {ms:.1f} ms (2 launches counted); seqs {v[8]}, search steps {v[9]}, ext round trips {v[10]}, blocks {v[11]}")
for i, nm in enumerate(names):
    print(f"  {nm:26s} {v[i] / max(tot, 1) * 100:5.1f} %  {v[i] / max(v[8], 1):8.1f} cyc/seq")
print(f"  total {tot / max(v[8], 1):.1f} cyc/seq (s_memtime units), steps/seq {v[9] / max(v[8], 1):.2f}")
