"""Sequence-wave phase counters from libjfsgpu_prof.so (s_memtime, 100 MHz)."""
import ctypes, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["JFS_GPU_LIB"] = os.path.join(ROOT, "juicefs_amd", "lib", "libjfsgpu_prof.so")
import torch
from juicefs_amd import _lib, device as D
lib = _lib.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
b = D.ZstdBatch(n, 4 << 20, "T", level=3, distinct=16, seed_base=1)
b.decompress(); torch.cuda.synchronize()
lib.jfs_zprof_reset()
b.decompress(); torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 8)()
lib.jfs_zprof_read(buf)
t_tab, t_loop, t_tot, nblk, nseq = buf[0], buf[1], buf[2], buf[3], buf[4]
print(f"frames {n} blocks {nblk} seqs {nseq} seq/frame {nseq / n:.0f}")
print(f"memtime ticks per frame: tables {t_tab / n:.0f} loop {t_loop / n:.0f} total {t_tot / n:.0f}")
print(f"ticks per sequence (loop) {t_loop / max(nseq, 1):.2f}; per block tables {t_tab / max(nblk, 1):.0f}")
print("ok" if b.verify() else "MISMATCH")
