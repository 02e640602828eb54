"""Lone one-call LZ4 / Zstd decode latency by calling pattern: with or
without a 20 ms gap between calls, into one reused output buffer or a
distinct (touched long before) buffer per call -- the bench's lone leg is
back to back into distinct buffers.  p50 / min of 21 calls per mode."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from juicefs_amd import compress as C  # noqa: E402
from juicefs_amd.blockgen import gen_block  # noqa: E402

U = 4 << 20
reps = 21
raw = gen_block("T", 5, U)
for name, codec in (("lz4", C.LZ4()), ("zstd", C.ZStandard())):
    comp = bytearray(codec.CompressBound(U))
    n, e = codec.Compress(comp, raw)
    assert e is None, e
    comp = bytes(comp[:n])
    outs = [bytearray(b"\x01") * U for _ in range(reps)]
    ballast = [bytearray(b"\x02") * (64 << 20) for _ in range(2)]  # evict the outputs from the host caches
    for gap in (0.02, 0.0):
        for distinct in (False, True):
            lat = []
            for r in range(reps):
                if gap:
                    time.sleep(gap)
                out = outs[r] if distinct else outs[0]
                t0 = time.perf_counter()
                m, e = codec.Decompress(out, comp)
                lat.append((time.perf_counter() - t0) * 1e3)
                assert m == U and e is None
            assert all(bytes(outs[r if distinct else 0]) == raw for r in range(reps if distinct else 1))
            print(f"{name} gap={gap * 1e3:.0f}ms distinct={int(distinct)}: p50 {np.median(lat):.3f} ms "
                  f"min {min(lat):.3f} max {max(lat):.3f}", flush=True)
            for b in ballast:
                b[::4096] = b"\x03" * len(b[::4096])
            outs = [bytearray(b"\x01") * U for _ in range(reps)]
