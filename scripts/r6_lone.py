"""Lone one-call latency (cachedStore.load's cache miss: one Decompress of a
4 MiB block, pkg/chunk/cached_store.go:814) for LZ4 and Zstd, p50 of 9 calls,
with the library's host trace on stderr (JFS_HOST_TRACE=1) for the breakdown.
usage: r6_lone.py [reps] [gap]; also times Compress (JFS_LONE_ENC=0: not)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from juicefs_amd import compress as C  # noqa: E402
from juicefs_amd.blockgen import gen_block  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 0.02  # seconds between calls
U = 4 << 20
raw = gen_block("T", 5, U)
codecs = os.environ.get("JFS_LONE_CODECS", "lz4,zstd").split(",")
for name, codec in [(n, c) for n, c in (("lz4", C.LZ4()), ("zstd", C.ZStandard())) if n in codecs]:
    comp = bytearray(codec.CompressBound(U))
    n, e = codec.Compress(comp, raw)
    assert e is None, e
    comp = bytes(comp[:n])
    out = bytearray(U)
    lat = []
    for _ in range(reps):
        time.sleep(gap)
        t0 = time.perf_counter()
        m, e = codec.Decompress(out, comp)
        lat.append((time.perf_counter() - t0) * 1e3)
        assert m == U and bytes(out) == raw
    print(f"{name} lone decode: p50 {np.median(lat):.3f} ms min {min(lat):.3f} ms  ({n} B compressed)", flush=True)
    print(f"[lone] {name} {' '.join(f'{x:.3f}' for x in lat)}", file=sys.stderr, flush=True)
    if os.environ.get("JFS_LONE_ENC", "1") != "0":
        elat = []
        for _ in range(max(3, reps // 3)):
            time.sleep(gap)
            t0 = time.perf_counter()
            m2, e = codec.Compress(comp2 := bytearray(codec.CompressBound(U)), raw)
            elat.append((time.perf_counter() - t0) * 1e3)
            assert e is None and bytes(comp2[:m2]) == comp
        print(f"{name} lone encode: p50 {np.median(elat):.3f} ms min {min(elat):.3f} ms", flush=True)
