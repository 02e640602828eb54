"""Zstd GPU encoder ratio on 4 MiB text blocks (for encoder variants); NB blocks (default 64)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from juicefs_amd import device as D
nb = int(os.environ.get("NB", "64"))
r, ratio, ms = D.zstd_compress_rate(nb, 4 << 20, "T", seed_base=900)
print(f"{os.environ.get('JFS_GPU_LIB', 'base')}: ratio {ratio:.3f}  {r:.2f} GiB/s ({ms:.1f} ms, {nb} blocks)")
