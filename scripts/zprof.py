"""zexec phase counters from libjfsgpu_prof.so (s_memtime ticks)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JFS_GPU_LIB"] = os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
import torch
from juicefs_amd import _lib, device as D
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
b = D.ZstdBatch(n, 4 << 20, "T", level=3, distinct=16, seed_base=1,
                cache_dir=os.path.join(os.environ.get("TMPDIR", "/tmp"), "jfs_frames"))
b.decompress(); torch.cuda.synchronize()
lib.jfs_zprof_reset()
b.decompress(); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
lib.jfs_zprof_read(buf)
names = ["item_load+litwin", "flush+far_issue", "literals", "far_land", "matches", "batches", "long_items(V2)", "total"]
for i, nm in enumerate(names):
    print(f"{nm:12s} per frame {buf[i] / n:14.0f}")
print(f"per batch: flush+far {buf[1] / max(buf[5], 1):.0f} literals {buf[2] / max(buf[5], 1):.0f} far_land {buf[3] / max(buf[5], 1):.0f} matches {buf[4] / max(buf[5], 1):.0f} ticks; match rounds per batch {buf[6] / max(buf[5], 1):.2f}")
print("ok" if b.verify() else "MISMATCH")
