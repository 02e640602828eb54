"""CPU: the Zstd level-1 encode oracle (oracle/zstd_l1_oracle.c, a restatement
of libzstd 1.4.9's ZSTD_compress(.., 1) -- pkg/compress/compress.go:82-91) is
byte-identical to libzstd's level-1 frames: the committed fixtures
(tests/golden/zstd_golden.json level-1 frames, tests/golden/zstd_l1_golden.json,
tests/golden/zstd_golden.json KATs) and, where /opt/conda/lib/libzstd.so.1
loads, ZSTD_compress itself on seeded inputs and ZSTD_getCParams on every
size tier."""
import ctypes
import hashlib
import json
import os
import random

import pytest

from juicefs_amd.blockgen import gen_block
from tests.zstd_l1_cases import make_case

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBZSTD = "/opt/conda/lib/libzstd.so.1"


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def zl1(oracle):
    lib = oracle.lib
    lib.oracle_zstd_compress_l1_ex.restype = ctypes.c_int64
    lib.oracle_zstd_compress_l1_ex.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64,
                                               ctypes.c_void_p]
    lib.oracle_zstd_l1_params.argtypes = [ctypes.c_int64, ctypes.c_void_p]

    def comp(src: bytes):
        n = len(src)
        cap = n + (n >> 8) + ((128 << 10) - n >> 11 if n < (128 << 10) else 0) + 64
        dst = ctypes.create_string_buffer(cap)
        r = lib.oracle_zstd_compress_l1_ex(src, n, dst, cap, None)
        assert r > 0
        return dst.raw[:r]

    def params(n: int):
        out = (ctypes.c_int32 * 3)()
        lib.oracle_zstd_l1_params(n, out)
        return tuple(out)

    comp.params = params
    return comp


@pytest.fixture(scope="module")
def libzstd():
    try:
        z = ctypes.CDLL(LIBZSTD)
    except OSError:
        pytest.skip("libzstd 1.4.9 not loadable here (the committed fixtures still pin the oracle)")
    z.ZSTD_compress.restype = ctypes.c_size_t
    z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    z.ZSTD_compressBound.restype = ctypes.c_size_t
    z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
    return z


def test_l1_kats(zl1, golden):
    for k in golden["zstd"]["kat"]:
        assert zl1(bytes.fromhex(k["src"])).hex() == k["comp_l1"]


def test_l1_golden_frames(zl1, golden):
    """Every level-1 frame of zstd_golden.json (1 B .. 1 MiB, classes T/Z/R)."""
    fr = [f for f in golden["zstd"]["frames"] if f["level"] == 1]
    assert len(fr) >= 19
    for f in fr:
        src = gen_block(f["cls"], f["seed"], f["size"])
        assert sha(src) == f["src_sha"]
        c = zl1(src)
        assert len(c) == f["csize"] and sha(c) == f["comp_sha"], (f["cls"], f["size"])


def test_l1_golden_cases(zl1):
    """zstd_l1_golden.json: 4 MiB T/Z/R/mixed/skewed frames (the bench shape),
    size-tier edges and multi-block mixes."""
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "zstd_l1_golden.json")))
    assert g["level"] == 1 and len(g["cases"]) >= 20
    for c in g["cases"]:
        src = make_case(c["kind"], c["seed"], c["size"])
        assert sha(src) == c["src_sha"]
        out = zl1(src)
        assert len(out) == c["csize"] and sha(out) == c["comp_sha"], (c["kind"], c["size"])


def test_l1_params_match_libzstd(zl1, libzstd):
    class CP(ctypes.Structure):
        _fields_ = [(n, ctypes.c_uint) for n in ("w", "c", "h", "s", "m", "t", "strat")]
    libzstd.ZSTD_getCParams.restype = CP
    libzstd.ZSTD_getCParams.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_size_t]
    sizes = sorted({*range(1, 70), *[1 << k for k in range(6, 27)], *[(1 << k) + d for k in range(6, 27) for d in (-1, 1)],
                    16384, 16385, 131072, 131073, 262144, 262145, 4 << 20})
    for n in sizes:
        c = libzstd.ZSTD_getCParams(1, n, 0)
        assert (c.strat, c.t) == (1, 0)
        assert zl1.params(n) == (c.w, c.h, c.m), n


def test_l1_matches_libzstd_seeded(zl1, libzstd):
    rng = random.Random(20261017)
    kinds = "TZRSM"
    for it in range(60):
        n = rng.choice([rng.randrange(0, 300), rng.randrange(0, 20000), rng.randrange(0, 300000),
                        rng.choice([131072, 262145, 1 << 20])])
        src = make_case(kinds[it % 5], 9000 + it, n)
        cap = libzstd.ZSTD_compressBound(n)
        d = ctypes.create_string_buffer(cap)
        m = libzstd.ZSTD_compress(d, cap, src, n, 1)
        assert zl1(src) == d.raw[:m], (kinds[it % 5], n)
