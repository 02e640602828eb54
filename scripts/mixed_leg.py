"""bench.py's mixed_host_path leg alone (configs[4] shape): python scripts/mixed_leg.py [nblk]"""
import json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench
from juicefs_amd.blockgen import gen_block
U = 4 << 20
raw = [gen_block("T", 1 + i, U) for i in range(32)]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
for rep in range(int(sys.argv[2]) if len(sys.argv) > 2 else 1):
    r = bench.mixed_host_path(raw, n)
    print(round(r["decompress"]["value"], 2), round(r["compress"]["value"], 2), flush=True)
