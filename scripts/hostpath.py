"""bench.py's host_path leg alone: python scripts/hostpath.py [nblk] (JFS_HOST_TRACE=1 for the stage trace)."""
import json, os, sys
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
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
print(json.dumps(bench.host_path_rate(comp, raw, U, nb), indent=1))
