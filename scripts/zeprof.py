"""Diagnostic: phase shares of the Zstd encoder from in-kernel s_memtime stamps
(libjfsgpu_prof.so, built with -DJFS_PROF).  usage: zeprof.py [N]"""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["JFS_GPU_LIB"] = os.environ.get("PROF_LIB") or os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
sys.path.insert(0, ROOT)
from juicefs_amd import _lib, device as D
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
D.zstd_compress_rate(min(n, 64), 4 << 20, "T", seed_base=7)
lib.jfs_zeprof_reset()
r, ratio, ms = D.zstd_compress_rate(n, 4 << 20, "T", seed_base=7)
buf = (ctypes.c_ulonglong * 12)()
lib.jfs_zeprof_read(buf)
names = ["parse", "lit hist+huf build", "huf streams", "lit section", "seq tables", "seq bitstream", "blk hdr/raw"]
tot = sum(buf[:7])
nb = max(buf[8], 1)
print(f"{n} frames  {ms:.1f} ms  {r:.2f} GiB/s  ratio {ratio:.4f}  blocks {buf[8]}  seqs/block {buf[9]/nb:.0f}")
for k, nm in enumerate(names):
    print(f"{nm:20s} {buf[k]/tot*100:6.2f}%  {buf[k]/nb/1e6:8.3f} Mcyc/block")
