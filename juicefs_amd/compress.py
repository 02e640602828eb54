"""Python mirror of JuiceFS pkg/compress over libjfsgpu.so.

Same names, argument meaning and error behaviour as
/root/reference/pkg/compress/compress.go so the parity tests read like the
reference's own compress_test.go:

    ZSTD_LEVEL = 1                                   compress.go:28
    class Compressor (Name / CompressBound / Compress / Decompress)   :31-36
    NewCompressor(algr) -> Compressor | None        :39-49
    noOp / ZStandard / LZ4                           :51-125

Go's ``(int, error)`` results become ``(n, err)`` tuples with ``err`` either
``None`` or a :class:`CompressError`.  ``dst`` must be a writable buffer
(bytearray / memoryview / numpy array); ``src`` any bytes-like object.  For
Zstd the capacity is ``len(dst)`` (Go passes ``cap(dst)``).

Every LZ4 byte is produced by the HIP kernels in libjfsgpu.so; there is no CPU
fallback (the library returns ``JFS_ERR_NO_DEVICE`` without a gfx950 GPU).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib as L

ZSTD_LEVEL = 1


class CompressError(Exception):
    def __init__(self, msg: str, code: int):
        super().__init__(msg)
        self.code = code


def _addr(buf, writable: bool):
    """Return (c_void_p, length, keepalive) for a buffer."""
    if buf is None:
        return None, 0, None
    # fast paths for the common types (a batch of 4,096 blocks spends
    # milliseconds here): the bytearray's own buffer / the bytes' own buffer
    t = type(buf)
    if t is bytearray and len(buf):
        c = ctypes.c_char.from_buffer(buf)
        return ctypes.c_void_p(ctypes.addressof(c)), len(buf), c
    if t is bytes and len(buf) and not writable:
        c = ctypes.c_char_p(buf)
        return ctypes.cast(c, ctypes.c_void_p), len(buf), (c, buf)
    mv = memoryview(buf)
    if not mv.contiguous:
        raise ValueError("buffer must be contiguous")
    mv = mv.cast("B")
    n = mv.nbytes
    if n == 0:
        return None, 0, mv
    if writable and mv.readonly:
        raise ValueError("dst must be writable")
    # address the buffer in place (no copy); numpy's view is much cheaper than
    # a per-call ctypes array type, which matters with 200 concurrent callers
    a = np.frombuffer(mv, dtype=np.uint8)
    return ctypes.c_void_p(a.ctypes.data), n, (mv, a)


def _err(code: int, dst_len: int, src_len: int, op: str) -> CompressError:
    if code == L.JFS_ERR_SHORT_BUFFER:
        return CompressError(f"buffer too short: {dst_len} < {src_len}", code)
    if code == L.JFS_ERR_EMPTY_INPUT:
        return CompressError("decompress an empty input", code)
    if code == L.JFS_ERR_COMPRESS_FAIL:
        return CompressError("lz4: compression failed (destination too small)", code)
    if code == L.JFS_ERR_CORRUPT:
        return CompressError("zstd: corrupted frame", code)
    if code == L.JFS_ERR_UNSUPPORTED:
        return CompressError(f"{op}: not supported by the GPU engine", code)
    if code == L.JFS_ERR_NO_DEVICE:
        return CompressError("no usable gfx950 device", code)
    if code <= L.JFS_ERR_BASE:
        return CompressError(f"{op}: error {code}", code)
    return CompressError(f"lz4: decompress failed ({code})", code)


class Compressor:
    """compress.go:31-36"""

    algo: int = -1

    def Name(self) -> str:
        return L.load().jfs_codec_name(self.algo).decode()

    def CompressBound(self, n: int) -> int:
        return int(L.load().jfs_compress_bound(self.algo, n))

    def Compress(self, dst, src):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        r = int(L.load().jfs_compress(self.algo, d, dn, s, sn))
        if r < 0:
            return 0, _err(r, dn, sn, "compress")
        return r, None

    def Decompress(self, dst, src):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        r = int(L.load().jfs_decompress(self.algo, d, dn, s, sn))
        if r < 0:
            # LZ4 passes LZ4_decompress_safe's negative value through (compress.go:124);
            # the other adapters return 0 with the error (compress.go:57-100).
            n = r if (self.algo == L.ALGO_LZ4 and r > L.JFS_ERR_BASE) else 0
            return n, _err(r, dn, sn, "decompress")
        return r, None

    # batch helpers (host buffers) -------------------------------------------
    def CompressBatch(self, pairs, device_mask: int = 0):
        return _batch(self.algo, pairs, device_mask, compress=True)

    def DecompressBatch(self, pairs, device_mask: int = 0):
        return _batch(self.algo, pairs, device_mask, compress=False)

    def DecompressBatchChecksum(self, pairs, device_mask: int = 0):
        """DecompressBatch plus each decoded block's disk-cache checksum
        (checksum() of pkg/chunk/disk_cache_file.go:139-152, written beside the
        block by disk_cache.go:536-537), computed on the GPU: [(n, err, csum)]"""
        return _batch(self.algo, pairs, device_mask, compress=False, with_csum=True)

    def CompressBatchChecksum(self, pairs, device_mask: int = 0):
        """CompressBatch plus each payload's CRC-32C (generateChecksum,
        pkg/object/checksum.go:30-45): [(n, err, crc)]"""
        return _batch(self.algo, pairs, device_mask, compress=True, with_crc=True)


class noOp(Compressor):  # noqa: N801  (reference name, compress.go:51)
    algo = L.ALGO_NONE


class ZStandard(Compressor):
    """compress.go:70-103; level is fixed at ZSTD_LEVEL (1)."""

    algo = L.ALGO_ZSTD

    def __init__(self, level: int = ZSTD_LEVEL):
        self.level = level


class LZ4(Compressor):
    """compress.go:105-125"""

    algo = L.ALGO_LZ4


def NewCompressor(algr: str):
    """compress.go:39-49: case-insensitive "zstd" / "lz4" / "none" / ""; else None."""
    a = L.load().jfs_codec_from_name(algr.encode())
    if a == L.ALGO_ZSTD:
        return ZStandard(ZSTD_LEVEL)
    if a == L.ALGO_LZ4:
        return LZ4()
    if a == L.ALGO_NONE:
        return noOp()
    return None


CSUM_BLOCK = 32 << 10  # disk_cache_file.go csBlock


def csum_bytes(n: int) -> int:
    """Length of checksum() for n data bytes: ((n-1)/32768+1)*4 (Go integer division)."""
    return (int((n - 1) / CSUM_BLOCK) + 1) * 4


def CompressBatchMixed(entries, device_mask: int = 0):
    """entries: list of (Compressor, dst, src) with any mix of codecs; the
    codecs' batches run at once on the GPU(s) (jfs_compress_batch_mixed).
    Returns [(n, err)] with each Compressor's own result semantics."""
    return _batch_mixed(entries, device_mask, compress=True)


def DecompressBatchMixed(entries, device_mask: int = 0):
    """DecompressBatch over blocks of several codecs (jfs_decompress_batch_mixed)."""
    return _batch_mixed(entries, device_mask, compress=False)


def _batch_mixed(entries, device_mask: int, compress: bool):
    lib = L.load()
    nb = len(entries)
    iov = (L.JfsIov * max(nb, 1))()
    algos = (ctypes.c_int32 * max(nb, 1))()
    keep = []
    for i, (cd, dst, src) in enumerate(entries):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        keep.append((kd, ks))
        iov[i].src, iov[i].src_len, iov[i].dst, iov[i].dst_cap = s, sn, d, dn
        algos[i] = cd.algo
    out = (ctypes.c_int64 * max(nb, 1))()
    fn = lib.jfs_compress_batch_mixed if compress else lib.jfs_decompress_batch_mixed
    rc = fn(algos, nb, iov, out, device_mask)
    if rc != 0:
        raise _err(rc, 0, 0, "batch")
    res = []
    for i in range(nb):
        r, algo = int(out[i]), int(algos[i])
        if r < 0:
            n = r if (algo == L.ALGO_LZ4 and not compress and r > L.JFS_ERR_BASE) else 0
            res.append((n, _err(r, iov[i].dst_cap, iov[i].src_len, "compress" if compress else "decompress")))
        else:
            res.append((r, None))
    return res


def _batch(algo: int, pairs, device_mask: int, compress: bool, with_crc: bool = False, with_csum: bool = False):
    """pairs: list of (dst, src).  Returns list of (n, err)."""
    lib = L.load()
    nb = len(pairs)
    iov = (L.JfsIov * max(nb, 1))()
    keep = []
    for i, (dst, src) in enumerate(pairs):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        keep.append((kd, ks))
        iov[i].src, iov[i].src_len, iov[i].dst, iov[i].dst_cap = s, sn, d, dn
    out = (ctypes.c_int64 * max(nb, 1))()
    crc = (ctypes.c_uint32 * max(nb, 1))()
    cs_bufs = []
    if with_csum:
        cs_bufs = [ctypes.create_string_buffer(csum_bytes(max(iov[i].dst_cap, 0))) for i in range(nb)]
        cs_ptrs = (ctypes.c_void_p * max(nb, 1))(*[ctypes.cast(b, ctypes.c_void_p) for b in cs_bufs])
    if with_crc:
        rc = lib.jfs_compress_batch_crc(algo, nb, iov, out, crc, device_mask)
    elif with_csum:
        rc = lib.jfs_decompress_batch_csum(algo, nb, iov, out, cs_ptrs, device_mask)
    else:
        fn = lib.jfs_compress_batch if compress else lib.jfs_decompress_batch
        rc = fn(algo, nb, iov, out, device_mask)
    if rc != 0:
        raise _err(rc, 0, 0, "batch")
    res = []
    for i in range(nb):
        r = int(out[i])
        if r < 0:
            n = r if (algo == L.ALGO_LZ4 and not compress and r > L.JFS_ERR_BASE) else 0
            res.append((n, _err(r, iov[i].dst_cap, iov[i].src_len, "compress" if compress else "decompress")))
        else:
            res.append((r, None))
    if with_crc:
        return [(n, e, int(crc[i])) for i, (n, e) in enumerate(res)]
    if with_csum:
        return [(n, e, cs_bufs[i].raw[:csum_bytes(n)] if e is None else None) for i, (n, e) in enumerate(res)]
    return res
