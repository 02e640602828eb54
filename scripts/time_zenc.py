"""Zstd GPU encode rate and ratio (N 4 MiB text blocks in HBM; frames verified by the GPU decoder)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from juicefs_amd import device as D
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
r, ratio, ms = D.zstd_compress_rate(n, 4 << 20, "T", seed_base=7)
print(f"{os.environ.get('JFS_GPU_LIB', 'base')}: zstd encode {n} blocks {ms:.1f} ms  {r:.2f} GiB/s  ratio {ratio:.4f}")
