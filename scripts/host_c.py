"""PCIe-inclusive LZ4 CompressBatch of N host blocks, three timed calls (the
first includes staging growth).  usage: host_c.py [N]"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from juicefs_amd import compress as C, device as D
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
U = 4 << 20
b = D.Lz4Batch(32, U, "T", seed_base=1)
raws = [b.raw[i * U:(i + 1) * U].cpu().numpy().tobytes() for i in range(32)]
c = C.LZ4()
bound = c.CompressBound(U)
pairs = [(bytearray(bound), raws[i % 32]) for i in range(n)]
for r in range(3):
    t0 = time.perf_counter()
    res = c.CompressBatch(pairs)
    dt = time.perf_counter() - t0
    assert all(m > 0 and e is None for m, e in res)
    print(f"chunk_mb_lz4c={os.environ.get('JFS_HOST_CHUNK_MB_LZ4C', '4096')} call {r}: {n * U / dt / 2**30:.2f} GiB/s ({dt * 1e3:.0f} ms)", flush=True)
