import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from juicefs_amd import device as D
for n in (64, 256, 512, 768, 1024):
    r, ratio, ms = D.zstd_compress_rate(n, 4 << 20, 'T', seed_base=7)
    print(n, round(r, 3), 'GiB/s', round(ms, 1), 'ms', flush=True)
