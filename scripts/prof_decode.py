"""Diagnostic: phase shares of the LZ4 decode kernel from in-kernel s_memtime
stamps (libjfsgpu_prof.so, built with -DJFS_PROF).  Read the shares, not the
time (stamps perturb the schedule)."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["JFS_GPU_LIB"] = os.environ.get("PROF_LIB") or os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import _lib, device as D
lib = _lib.load()
nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
cls = sys.argv[2] if len(sys.argv) > 2 else "T"
b = D.Lz4Batch(nblk, 4 << 20, cls, seed_base=1)
b.decompress(); torch.cuda.synchronize()
lib.jfs_prof_reset()
t0 = time.perf_counter(); b.decompress(); torch.cuda.synchronize(); dt = time.perf_counter() - t0
assert b.verify()
buf = (ctypes.c_uint64 * 20)()
lib.jfs_prof_read(buf)
names = ["stage", "walk+fixup", "table+tokparse", "batching", "lits+pref", "far", "near", "long+serial", "copier wait", "parser wait"]
tot = sum(buf[:10])
print(f"blocks={nblk} cls={cls} wall={dt*1e3:.1f} ms  GiB/s={nblk*4/1024/dt:.1f}")
for n, v in zip(names, buf[:10]):
    print(f"{n:14s} {v/tot*100:6.2f}%  {v/nblk/1e6:8.3f} Mcyc/block")
w = max(buf[10], 1)
print(f"windows/block {buf[10]/nblk:.1f}  per window: walk iters {buf[11]/w:.2f}  fix-up rounds {buf[12]/w:.2f}  "
      f"partial iters {buf[13]/w:.2f}  batches {buf[14]/w:.2f}  near copy iters {buf[15]/w:.2f}")
b = max(buf[14], 1)
print(f"per batch: literal iters {buf[16]/b:.2f}  far iters {buf[17]/b:.2f}  near rounds {buf[18]/b:.2f}  near copy iters {buf[15]/b:.2f}  serial near matches {buf[19]/b:.2f}")
