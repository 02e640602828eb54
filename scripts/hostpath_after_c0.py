"""bench.py's order: configs[0] round trip, then the host_path leg (2,048 blocks)."""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
U = 4 << 20
raw = [gen_block("T", 1 + i, U) for i in range(32)]
lz = C.LZ4()
pairs = [(bytearray(lz.CompressBound(U)), r) for r in raw]
res = lz.CompressBatch(pairs)
comp = [bytes(d[:n]) for (d, _), (n, e) in zip(pairs, res)]
c0 = bench.configs0_roundtrip(torch.device("cuda"), 1024, U)
print("c0", round(c0["value"], 2), flush=True)
for _ in range(2):
    hp = bench.host_path_rate(comp, raw, U, 2048)
    print("hp", round(hp["lz4_decompress"]["value"], 2), round(hp["lz4_compress"]["value"], 2), flush=True)
