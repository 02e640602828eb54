"""bench.py's host-buffer legs in the bench's order (configs[0], host path,
one-call, then configs[4]) to find what slows configs[4] down in the bench.
usage: r5_mixed_seq.py [skip...]  (skip: c0 hp os)"""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
skip = set(sys.argv[1:])
U = 4 << 20
raw = [gen_block("T", 1 + i, U) for i in range(32)]
lz = C.LZ4()
pairs = [(bytearray(lz.CompressBound(U)), r) for r in raw]
comp = [bytes(d[:n]) for (d, _), (n, e) in zip(pairs, lz.CompressBatch(pairs))]
dev = torch.device("cuda", 0)
t = time.perf_counter()
if "c0" not in skip:
    r = bench.configs0_roundtrip(dev, 1024, U); print("c0", round(r["value"], 2), round(time.perf_counter() - t, 1), flush=True)
if "hp" not in skip:
    r = bench.host_path_rate(comp, raw, U, 2048); print("hp", round(r["lz4_decompress"]["value"], 2), round(time.perf_counter() - t, 1), flush=True)
if "os" not in skip:
    r = bench.oneshot_concurrency(comp, raw, U); print("os", round(r["decompress_200_concurrent"]["value"], 2), round(time.perf_counter() - t, 1), flush=True)
for _ in range(2):
    r = bench.mixed_host_path(raw, 4096)
    print("mixed", round(r["decompress"]["value"], 2), round(r["compress"]["value"], 2), round(time.perf_counter() - t, 1), flush=True)
