"""Generate tests/golden/zstd_l1_golden.json: libzstd 1.4.9 ZSTD_compress(level 1)
frames (sha256 + size) of the cases in tests/zstd_l1_cases.py.

libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1) is the C library this image
holds of the encoder pkg/compress reaches through github.com/DataDog/zstd
(pkg/compress/compress.go:82-91 -> zstd.CompressLevel(dst, src, 1)); the
reference pins v1.5.6, which is not available offline.
Data only: the inputs are described by (kind, seed, size), the outputs by
their sha256.  Run from the repo root: python tests/golden/make_zstd_l1_golden.py
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tests.zstd_l1_cases import CASES, make_case  # noqa: E402

ZS = ctypes.CDLL("/opt/conda/lib/libzstd.so.1")
ZS.ZSTD_compress.restype = ctypes.c_size_t
ZS.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
ZS.ZSTD_compressBound.restype = ctypes.c_size_t
ZS.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
ZS.ZSTD_isError.restype = ctypes.c_uint
ZS.ZSTD_isError.argtypes = [ctypes.c_size_t]


def main():
    out = {"version": ZS.ZSTD_versionNumber(), "level": 1, "cases": []}
    for kind, seed, n in CASES:
        src = make_case(kind, seed, n)
        cap = ZS.ZSTD_compressBound(n)
        dst = ctypes.create_string_buffer(cap)
        c = ZS.ZSTD_compress(dst, cap, src, n, 1)
        assert not ZS.ZSTD_isError(c)
        out["cases"].append({"kind": kind, "seed": seed, "size": n, "csize": c,
                             "src_sha": hashlib.sha256(src).hexdigest(),
                             "comp_sha": hashlib.sha256(dst.raw[:c]).hexdigest()})
    with open(os.path.join(HERE, "zstd_l1_golden.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
