"""Debug: decode individual cases on the GPU and compare with the oracle."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
from tests.oracle_ctypes import Oracle
orc = Oracle(os.path.join(ROOT, "oracle", "_build", "liboracle.so"))
c = C.LZ4()
cases = [(cls, n) for n in (100, 4096, 65535, 131072, 1 << 20, 4 << 20) for cls in "TZR"]
for i, (cls, n) in enumerate(cases):
    src = gen_block(cls, 900 + i, n)
    _, comp = orc.lz4_compress(src)
    for cap in (n, n + 77, n - 1):
        r_exp, ref = orc.lz4_decompress(comp, cap)
        dst = bytearray(cap)
        (r, err), = c.DecompressBatch([(dst, comp)])
        ok = r == r_exp and (r < 0 or bytes(dst[:r]) == ref)
        first = None
        if r >= 0 and r_exp >= 0 and not ok:
            m = min(r, r_exp)
            first = next((k for k in range(m) if dst[k] != ref[k]), None)
        print(f"{cls} n={n} cap={cap} ret={r} exp={r_exp} ok={ok} first_diff={first}", flush=True)
