"""bench.py's oneshot_concurrency leg alone (one-call API from many host threads).
usage: python scripts/concur.py [n_dec] [n_enc]"""
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
nd = int(sys.argv[1]) if len(sys.argv) > 1 else 200
ne = int(sys.argv[2]) if len(sys.argv) > 2 else 20
print(json.dumps(bench.oneshot_concurrency(comp, raw, U, n_dec=nd, n_enc=ne), indent=1))
