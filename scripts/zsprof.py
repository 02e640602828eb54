"""zseq phase shares from libjfsgpu_prof.so (s_memtime ticks summed over waves).
usage: zsprof.py [N]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JFS_GPU_LIB"] = os.environ.get("PROF_LIB") or os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
import torch
from juicefs_amd import _lib, device as D
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
b = D.ZstdBatch(n, 4 << 20, "T", level=3, distinct=16, seed_base=1,
                cache_dir=os.path.join(os.environ.get("TMPDIR", "/tmp"), "jfs_frames"))
b.decompress(); torch.cuda.synchronize()
lib.jfs_zsprof_reset()
b.decompress(); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
lib.jfs_zsprof_read(buf)
names = ["phaseA walk+tables", "table staging", "phaseB decode", "phaseC", "sub-groups", "groups"]
tot = sum(buf[:4])
for i, nm in enumerate(names[:4]):
    print(f"{nm:20s} {buf[i] / tot * 100:6.2f}%  {buf[i] / n / 1e6:8.3f} Mcyc/frame")
print(f"decoder barrier waits {buf[4] / n / 1e6:8.3f} Mcyc/frame ({buf[4] / max(buf[2], 1) * 100:.1f}% of phase B)  groups {buf[5]}  frames {n}")
print("ok" if b.verify() else "MISMATCH")
