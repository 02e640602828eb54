#!/usr/bin/env python3
"""Generate tests/golden/*.json from the C libraries JuiceFS's codecs wrap.

Run in the build container (not on the GPU box):
    python tests/golden/make_golden.py

Sources of truth (third-party libraries in this image, NOT the reference repo):
  * liblz4 1.9.3  (/opt/conda/lib/liblz4.so.1)  -- LZ4_compress_default /
    LZ4_decompress_safe, the C entry points pkg/compress reaches through
    github.com/hungys/go-lz4 (pkg/compress/compress.go:112-125).
  * libzstd 1.4.9 (/opt/conda/lib/libzstd.so.1) -- ZSTD_compress /
    ZSTD_decompress, reached through github.com/DataDog/zstd
    (pkg/compress/compress.go:79-103).
The pinned upstream versions (go-lz4 @2017-08-05, zstd 1.5.6) are not available
offline; see DESIGN.md "Parity pinning".

Outputs are data only (inputs described by generator seed, expected outputs as
hex or sha256), so the GPU box never needs these libraries.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from juicefs_amd.blockgen import gen_block  # noqa: E402

LZ = ctypes.CDLL("/opt/conda/lib/liblz4.so.1")
ZS = ctypes.CDLL("/opt/conda/lib/libzstd.so.1")
ZS.ZSTD_compress.restype = ctypes.c_size_t
ZS.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
ZS.ZSTD_decompress.restype = ctypes.c_size_t
ZS.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
ZS.ZSTD_isError.restype = ctypes.c_uint
ZS.ZSTD_isError.argtypes = [ctypes.c_size_t]
ZS.ZSTD_getErrorName.restype = ctypes.c_char_p
ZS.ZSTD_getErrorName.argtypes = [ctypes.c_size_t]
ZS.ZSTD_compressBound.restype = ctypes.c_size_t
ZS.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
ZS.ZSTD_createCCtx.restype = ctypes.c_void_p
ZS.ZSTD_CCtx_setParameter.restype = ctypes.c_size_t
ZS.ZSTD_CCtx_setParameter.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
ZS.ZSTD_compress2.restype = ctypes.c_size_t
ZS.ZSTD_compress2.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]


def sha(b: bytes) -> str:
    return hashlib.sha256(b).hexdigest()


def lz4_compress(src: bytes, cap: int | None = None):
    if cap is None:
        cap = LZ.LZ4_compressBound(len(src))
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = LZ.LZ4_compress_default(src, dst, len(src), cap)
    return n, dst.raw[: max(n, 0)]


def lz4_decompress(src: bytes, cap: int):
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = LZ.LZ4_decompress_safe(src, dst, len(src), cap)
    return n, dst.raw[: max(n, 0)]


def zstd_compress(src: bytes, level: int) -> bytes:
    cap = ZS.ZSTD_compressBound(len(src))
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = ZS.ZSTD_compress(dst, cap, src, len(src), level)
    assert not ZS.ZSTD_isError(n)
    return dst.raw[:n]


def zstd_decompress(src: bytes, cap: int):
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = ZS.ZSTD_decompress(dst, cap, src, len(src))
    if ZS.ZSTD_isError(n):
        return -1, ZS.ZSTD_getErrorName(n).decode()
    return n, dst.raw[:n]


def lz4_section():
    out = {"version": LZ.LZ4_versionNumber(), "kat": [], "blocks": [], "limited": [], "decode_corpus": []}
    # Known-answer vectors, plus the reference test inputs
    # (compress_test.go:26 uses c.Name(): "LZ4").
    for s in [b"", b"LZ4", b"Zstd", b"Noop", b"hello world" * 8, b"a" * 13, b"abcdefghijklm" * 3]:
        n, c = lz4_compress(s)
        out["kat"].append({"src": s.hex(), "bound": LZ.LZ4_compressBound(len(s)), "comp": c.hex(),
                           "dst1": LZ.LZ4_compress_default(s, ctypes.create_string_buffer(1), len(s), 1)})
    # Generated blocks: every class, sizes around the byU16/byU32 switch (65547)
    # and the JuiceFS block-size range ends (64 KiB ... 4 MiB).
    sizes = [1, 12, 13, 100, 4096, 65535, 65546, 65547, 65548, 131072, 1 << 20, 4 << 20]
    for cls in "TZR":
        for sz in sizes:
            if cls == "T" and sz == 4 << 20:
                seeds = [1000, 1001]
            else:
                seeds = [sz * 7 + ord(cls)]
            for seed in seeds:
                src = gen_block(cls, seed, sz)
                n, c = lz4_compress(src)
                ent = {"cls": cls, "seed": seed, "size": sz, "csize": n, "comp_sha": sha(c), "src_sha": sha(src)}
                if n <= 2048:
                    ent["comp"] = c.hex()
                out["blocks"].append(ent)
                # limited-output behaviour (compress_test.go:89 compresses into c[:4<<20])
                for cap in (n, n - 1, max(1, n // 2)):
                    m, c2 = lz4_compress(src, cap)
                    out["limited"].append({"cls": cls, "seed": seed, "size": sz, "cap": cap, "ret": m})
    # Decode acceptance corpus: mutations of valid small streams, with the exact
    # return value of LZ4_decompress_safe and sha256 of dst[:ret].
    rng = random.Random(20250815)
    streams = []
    for cls in "TZR":
        for sz in (16, 40, 100, 300, 1000, 3000):
            src = gen_block(cls, 77 + sz, sz)
            streams.append((lz4_compress(src)[1], sz))
    streams.append((lz4_compress(b"hello world" * 8)[1], 88))
    # handcrafted KATs from SURVEY.md section 8a (decoder acceptance table)
    lits12 = bytes(range(97, 109))
    hand = [
        (bytes.fromhex("30616263"), 3), (bytes.fromhex("30616263"), 2), (bytes.fromhex("3061626358"), 3),
        (bytes.fromhex("306162"), 3), (bytes.fromhex("00"), 0), (bytes.fromhex("00"), 5),
        (bytes.fromhex("40616263640400505a5a5a5a5a"), 13), (bytes.fromhex("40616263640400505a5a5a5a5a"), 20),
    ]
    for off in (0, 1, 2, 3, 13):
        for tail in (3, 4, 5, 6, 12):
            s = bytes([0xCF]) + lits12 + bytes([off & 255, off >> 8, 12]) + bytes([tail << 4]) + b"Z" * tail
            for cap in (12 + 31 + tail, 12 + 31 + tail + 1, 12 + 31 + tail + 100, 12 + 31 + tail - 1):
                hand.append((s, cap))
    for c, cap in hand:
        r, o = lz4_decompress(c, cap)
        out["decode_corpus"].append({"src": c.hex(), "cap": cap, "ret": r, "out_sha": sha(o) if r >= 0 else None})
    for _ in range(3000):
        c, U = streams[rng.randrange(len(streams))]
        c = bytearray(c)
        k = rng.randrange(6)
        if k == 0 and c:
            c[rng.randrange(len(c))] = rng.randrange(256)
        elif k == 1:
            c = c[: rng.randrange(len(c) + 1)]
        elif k == 2:
            c += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 4)))
        elif k == 3 and c:
            for _ in range(rng.randrange(1, 5)):
                c[rng.randrange(len(c))] = rng.randrange(256)
        elif k == 4:
            c = bytearray(rng.randrange(256) for _ in range(rng.randrange(1, 120)))
        cap = rng.choice([U, U + rng.randrange(1, 100), max(U - rng.randrange(1, 20), 0), rng.randrange(0, 300)])
        c = bytes(c)
        if not c:
            continue
        r, o = lz4_decompress(c, cap)
        out["decode_corpus"].append({"src": c.hex(), "cap": cap, "ret": r, "out_sha": sha(o) if r >= 0 else None})
    return out


def zstd_err(name: str) -> int:
    """libzstd error name -> oracle category (oracle/zstd_oracle.c ZO_ERR_*)."""
    if "too small" in name:
        return -2
    if "Src size is incorrect" in name:
        return -3
    return -1


def zstd_decompress_cat(src: bytes, cap: int):
    dst = ctypes.create_string_buffer(max(cap, 1))
    n = ZS.ZSTD_decompress(dst, cap, src, len(src))
    if ZS.ZSTD_isError(n):
        name = ZS.ZSTD_getErrorName(n).decode()
        return zstd_err(name), name, b""
    return n, None, dst.raw[:n]


def zstd_compress_params(src: bytes, params: dict) -> bytes:
    """ZSTD_compress2 with explicit parameters (ZSTD_cParameter numbers)."""
    cctx = ZS.ZSTD_createCCtx()
    for k, v in params.items():
        r = ZS.ZSTD_CCtx_setParameter(ctypes.c_void_p(cctx), k, v)
        assert not ZS.ZSTD_isError(r), (k, v)
    cap = ZS.ZSTD_compressBound(len(src)) + 64
    dst = ctypes.create_string_buffer(cap)
    n = ZS.ZSTD_compress2(ctypes.c_void_p(cctx), dst, cap, src, len(src))
    assert not ZS.ZSTD_isError(n)
    ZS.ZSTD_freeCCtx(ctypes.c_void_p(cctx))
    return dst.raw[:n]


ZSTD_C_LEVEL, ZSTD_C_WINDOWLOG, ZSTD_C_CONTENTSIZE, ZSTD_C_CHECKSUM = 100, 101, 200, 201


def zstd_section(bin_path: str):
    out = {"version": ZS.ZSTD_versionNumber(), "kat": [], "frames": [], "accept": [], "special": [],
           "corpus": [], "bin": os.path.basename(bin_path)}
    blob = bytearray()

    def put(c: bytes) -> int:
        off = len(blob)
        blob.extend(c)
        return off

    for s in [b"", b"LZ4", b"Zstd", b"Noop", b"hello world" * 8]:
        c = zstd_compress(s, 1)
        out["kat"].append({"src": s.hex(), "bound": ZS.ZSTD_compressBound(len(s)), "comp_l1": c.hex()})
    # Frames for decoder parity: level 1 (what pkg/compress writes, ZSTD_LEVEL=1,
    # compress.go:28) and level 3 (BASELINE config 4), plus higher levels to
    # exercise more block/literal/sequence modes.  Bytes go to the .bin file.
    for cls in "TZR":
        for sz in (1, 100, 4096, 65536, 131072, 300000, 1 << 20):
            for lvl in (1, 3, 9, 19):
                if sz >= 1 << 20 and lvl > 3 or cls == "R" and sz > 131072:
                    continue
                src = gen_block(cls, 31 * sz + lvl, sz)
                c = zstd_compress(src, lvl)
                out["frames"].append({"cls": cls, "seed": 31 * sz + lvl, "size": sz, "level": lvl, "csize": len(c),
                                      "comp_sha": sha(c), "src_sha": sha(src), "off": put(c)})
    # One BASELINE-sized block (configs[3]: level 3, 4 MiB).
    src = gen_block("T", 4242, 4 << 20)
    c = zstd_compress(src, 3)
    out["frames"].append({"cls": "T", "seed": 4242, "size": 4 << 20, "level": 3, "csize": len(c),
                          "comp_sha": sha(c), "src_sha": sha(src), "off": put(c)})
    # Header variants: checksum, no content size (window descriptor), small
    # windows (many blocks, offsets bounded by the window), long-distance levels.
    variants = [
        ("checksum", {ZSTD_C_LEVEL: 1, ZSTD_C_CHECKSUM: 1}),
        ("checksum_l3", {ZSTD_C_LEVEL: 3, ZSTD_C_CHECKSUM: 1}),
        ("no_fcs", {ZSTD_C_LEVEL: 1, ZSTD_C_CONTENTSIZE: 0}),
        ("no_fcs_l9", {ZSTD_C_LEVEL: 9, ZSTD_C_CONTENTSIZE: 0, ZSTD_C_CHECKSUM: 1}),
        ("wlog10", {ZSTD_C_LEVEL: 3, ZSTD_C_WINDOWLOG: 10, ZSTD_C_CONTENTSIZE: 0}),
        ("wlog12", {ZSTD_C_LEVEL: 19, ZSTD_C_WINDOWLOG: 12, ZSTD_C_CONTENTSIZE: 0}),
    ]
    for name, prm in variants:
        for cls, sz in (("T", 200000), ("T", 777), ("Z", 300000), ("R", 5000)):
            src = gen_block(cls, 99 + sz, sz)
            c = zstd_compress_params(src, prm)
            r, e, o = zstd_decompress_cat(c, sz)
            assert r == sz and o == src
            out["special"].append({"name": name, "cls": cls, "seed": 99 + sz, "size": sz, "csize": len(c),
                                   "src_sha": sha(src), "off": put(c)})
    z = zstd_compress(b"hello world" * 8, 1)
    z2 = zstd_compress(b"Zstd", 1)
    skip = bytes.fromhex("502a4d18") + (4).to_bytes(4, "little") + b"\x00\x01\x02\x03"
    flip = bytearray(z)
    flip[-3] ^= 0x40
    for frame, cap in [(z, 88), (z, 87), (z + b"\x00", 88), (z + z2, 92), (skip + z, 88), (bytes(flip), 88),
                       (z[:-1], 88), (z, 200), (skip, 10), (z + skip, 88)]:
        r, e, o = zstd_decompress_cat(frame, cap)
        out["accept"].append({"src": frame.hex(), "cap": cap, "ret": r, "err": e,
                              "out_sha": sha(o) if r >= 0 else None})
    # Acceptance corpus: mutations of small valid frames (all levels / classes),
    # libzstd's verdict per case (size + sha, or error category).
    rng = random.Random(20251015)
    base = []
    for cls in "TZR":
        for sz in (10, 100, 700, 2000):
            for lvl in (1, 3, 19):
                src = gen_block(cls, 5 * sz + lvl, sz)
                base.append((zstd_compress(src, lvl), sz))
    base.append((zstd_compress_params(gen_block("T", 3, 3000), {ZSTD_C_LEVEL: 3, ZSTD_C_CHECKSUM: 1}), 3000))
    for _ in range(2000):
        c, U = base[rng.randrange(len(base))]
        c = bytearray(c)
        k = rng.randrange(5)
        if k == 0:
            c[rng.randrange(len(c))] = rng.randrange(256)
        elif k == 1:
            c = c[: rng.randrange(1, len(c) + 1)]
        elif k == 2:
            c += bytes(rng.randrange(256) for _ in range(rng.randrange(1, 6)))
        elif k == 3:
            for _ in range(rng.randrange(1, 4)):
                i = rng.randrange(len(c))
                c[i] ^= 1 << rng.randrange(8)
        cap = rng.choice([U, U + rng.randrange(1, 100), max(U - rng.randrange(1, 20), 0)])
        r, e, o = zstd_decompress_cat(bytes(c), cap)
        out["corpus"].append({"src": bytes(c).hex(), "cap": cap, "ret": r, "err": e,
                              "out_sha": sha(o) if r >= 0 else None})
    with open(bin_path, "wb") as f:
        f.write(bytes(blob))
    return out


def main():
    only = sys.argv[1:] or ["lz4", "zstd"]
    data = {}
    if "lz4" in only:
        data["lz4"] = lz4_section()
    if "zstd" in only:
        data["zstd"] = zstd_section(os.path.join(HERE, "zstd_frames.bin"))
    for name, sec in data.items():
        path = os.path.join(HERE, f"{name}_golden.json")
        with open(path, "w") as f:
            json.dump(sec, f, indent=0, sort_keys=True)
        print(path, os.path.getsize(path))


if __name__ == "__main__":
    main()
