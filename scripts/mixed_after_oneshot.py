"""bench.py's order for the configs[4] leg: one-call concurrency first, then mixed_host_path."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
U = 4 << 20
raw = [gen_block("T", 1 + i, U) for i in range(32)]
lz = C.LZ4()
pairs = [(bytearray(lz.CompressBound(U)), r) for r in raw]
res = lz.CompressBatch(pairs)
comp = [bytes(d[:n]) for (d, _), (n, e) in zip(pairs, res)]
if len(sys.argv) > 1 and sys.argv[1] == "oneshot":
    bench.oneshot_concurrency(comp, raw, U)
for _ in range(2):
    r = bench.mixed_host_path(raw, 4096)
    print("mixed", round(r["decompress"]["value"], 2), round(r["compress"]["value"], 2), flush=True)
