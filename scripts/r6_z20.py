"""20 concurrent one-call Zstd compresses of distinct 4 MiB text blocks (the
bench's compress_20_concurrent shape), one burst after a warm-up burst; prints
the wall time per burst.  For a kernel timeline under rocprofv3."""
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from juicefs_amd import compress as C  # noqa: E402
from juicefs_amd.blockgen import gen_block  # noqa: E402

U = 4 << 20
n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
raws = [gen_block("T", 900 + i, U) for i in range(n)]
c = C.ZStandard()
dst = [bytearray(c.CompressBound(U)) for _ in range(n)]
for burst in range(3):
    bar = threading.Barrier(n)
    lat = [0.0] * n

    def one(i):
        bar.wait()
        t0 = time.perf_counter()
        m, e = c.Compress(dst[i], raws[i])
        lat[i] = (time.perf_counter() - t0) * 1e3
        assert e is None and m > 0
    th = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    t0 = time.perf_counter()
    [x.start() for x in th]
    [x.join() for x in th]
    wall = (time.perf_counter() - t0) * 1e3
    print(f"burst {burst}: wall {wall:.1f} ms, call p50 {sorted(lat)[n // 2]:.1f} ms, "
          f"{n * U / wall / 1e3 / 1.073741824:.3f} GiB/s", flush=True)
