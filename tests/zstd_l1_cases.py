"""Deterministic inputs of the Zstd level-1 encode fixtures (test data only).

A case is (kind, seed, size):
  "T" / "Z" / "R"  juicefs_amd.blockgen classes (text-like, zeros, random);
  "S"              skewed bytes (an "R" block with each byte ANDed with two
                   shifted copies of itself: few distinct values, long
                   Huffman codes);
  "M"              a mix of T, R, Z and S runs of 1 B - 40 KiB (raw, RLE and
                   compressed blocks side by side in one frame; repeat-offset
                   and Huffman-table reuse across blocks).
tests/golden/make_zstd_l1_golden.py records libzstd 1.4.9's level-1 frame of
each case (sha256); tests compare the oracle and the GPU encoder with them.
"""
from __future__ import annotations

import numpy as np

from juicefs_amd.blockgen import gen_block


def _splitmix(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = x
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def _skewed(seed: int, n: int) -> bytes:
    r = np.frombuffer(gen_block("R", seed, n), dtype=np.uint8)
    return (r & (r >> 1) & (r >> 3)).astype(np.uint8).tobytes()


def make_case(kind: str, seed: int, n: int) -> bytes:
    if kind in ("T", "Z", "R"):
        return gen_block(kind, seed, n)
    if kind == "S":
        return _skewed(seed, n)
    if kind == "M":
        out = bytearray()
        st = seed * 2654435761 + 12345
        k = 0
        while len(out) < n:
            st = _splitmix(st)
            sel = st % 10
            ln = 1 + (st >> 8) % (40 << 10)
            if (st >> 40) % 4 == 0:
                ln = 1 + ln % 64  # short runs too
            sub = seed * 1000 + k
            if sel < 5:
                piece = gen_block("T", sub, ln)
            elif sel < 7:
                piece = gen_block("R", sub, ln)
            elif sel < 8:
                piece = bytes([(st >> 16) & 255]) * ln
            else:
                piece = _skewed(sub, ln)
            out += piece
            k += 1
        return bytes(out[:n])
    raise ValueError(kind)


# fixture cases (tests/golden/zstd_l1_golden.json): the bench shape (4 MiB),
# the size-tier edges of ZSTD_getCParams, and multi-block mixes
CASES = [("T", 4100, 4 << 20), ("Z", 4101, 4 << 20), ("R", 4102, 4 << 20), ("M", 4103, 4 << 20),
         ("M", 4104, 4 << 20), ("S", 4105, 4 << 20), ("T", 4106, 16384), ("T", 4107, 16385),
         ("T", 4108, 131073), ("T", 4109, 262144), ("T", 4110, 262145), ("T", 4111, (2 << 20) + 5),
         ("M", 4112, 1 << 20), ("M", 4113, 300000), ("M", 4114, 70000), ("S", 4115, 100000),
         ("S", 4116, 5000), ("M", 4117, 999), ("T", 4118, 7), ("T", 4119, 8), ("T", 4120, 24),
         ("Z", 4121, 131072 + 7), ("M", 4122, (3 << 20) + 77)]
