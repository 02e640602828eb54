"""Deterministic synthetic block generator (pure Python restatement).

Byte-identical to ``juicefs_amd/csrc/blockgen.h`` (the HIP/C++ generator used by
bench.py).  Spec: SURVEY.md section 8(d).  Used by tests to cross-check the
native generator and to build golden fixtures; slow (~0.5 s per 4 MiB 'T'
block), so tests keep sizes small.
"""
from __future__ import annotations

_M64 = (1 << 64) - 1
VOCAB_SEED = 0x4A7566734C5A3421


class _SplitMix64:
    __slots__ = ("s",)

    def __init__(self, seed: int):
        self.s = seed & _M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & _M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
        return z ^ (z >> 31)


def _vocab():
    r = _SplitMix64(VOCAB_SEED)
    out = []
    for _ in range(4096):
        n = 2 + r.next() % 10
        out.append(bytes(97 + r.next() % 26 for _ in range(n)))
    return out


_VOCAB = None


def gen_block(cls: str, seed: int, n: int) -> bytes:
    """Return ``n`` bytes of class 'T' (text-like), 'Z' (zeros) or 'R' (random)."""
    global _VOCAB
    if cls == "Z":
        return bytes(n)
    r = _SplitMix64(seed)
    if cls == "R":
        b = bytearray()
        while len(b) < n:
            b += r.next().to_bytes(8, "little")
        return bytes(b[:n])
    if cls != "T":
        raise ValueError(cls)
    if _VOCAB is None:
        _VOCAB = _vocab()
    buf = bytearray()
    wl = 0
    newline = True
    while len(buf) < n:
        if newline:
            newline = False
            if r.next() % 50 == 0:
                ln = 64 + r.next() % 960
                rb = bytearray()
                while len(rb) < ln:
                    rb += r.next().to_bytes(8, "little")
                buf += rb[:ln]
                continue
        x = r.next()
        k = x % 12
        idx = (1 << k) - 1 + ((x >> 8) % (1 << k))
        buf += _VOCAB[idx]
        wl += 1
        if wl == 512:
            buf += b"\n"
            wl = 0
            newline = True
        else:
            buf += b" "
    return bytes(buf[:n])
