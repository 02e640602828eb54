"""ctypes binding of the CPU oracle (oracle/_build/liboracle.so) -- test infra only."""
from __future__ import annotations

import ctypes


class Oracle:
    def __init__(self, path: str):
        self.lib = lib = ctypes.CDLL(path)
        vp, i32, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
        lib.oracle_lz4_bound.argtypes = [i64]
        lib.oracle_lz4_bound.restype = i64
        lib.oracle_lz4_compress_default.argtypes = [vp, vp, i32, i32]
        lib.oracle_lz4_compress_default.restype = i32
        lib.oracle_lz4_decompress_safe.argtypes = [vp, vp, i32, i32]
        lib.oracle_lz4_decompress_safe.restype = i32
        lib.oracle_crc32c_update.argtypes = [ctypes.c_uint32, vp, ctypes.c_size_t]
        lib.oracle_crc32c_update.restype = ctypes.c_uint32
        lib.oracle_crc32c_segments.argtypes = [vp, i64, i64, vp]
        lib.oracle_crc32c_segments.restype = i64
        for f in (lib.oracle_aes256gcm_seal, lib.oracle_aes256gcm_open):
            f.argtypes = [vp, vp, vp, i64, vp]
            f.restype = i64
        self.has_zstd = hasattr(lib, "oracle_zstd_decompress")
        if self.has_zstd:
            lib.oracle_zstd_decompress.argtypes = [vp, i64, vp, i64]
            lib.oracle_zstd_decompress.restype = i64
            lib.oracle_zstd_set_strict_reserved.argtypes = [i32]
            lib.oracle_zstd_frame_content_size.argtypes = [vp, i64]
            lib.oracle_zstd_frame_content_size.restype = i64
            lib.oracle_xxh64.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64]
            lib.oracle_xxh64.restype = ctypes.c_uint64

    def lz4_bound(self, n: int) -> int:
        return self.lib.oracle_lz4_bound(n)

    def lz4_compress(self, src: bytes, cap: int | None = None):
        if cap is None:
            cap = self.lz4_bound(len(src))
        dst = ctypes.create_string_buffer(max(cap, 1))
        n = self.lib.oracle_lz4_compress_default(src, dst, len(src), cap)
        return n, dst.raw[: max(n, 0)]

    def lz4_decompress(self, src: bytes, cap: int):
        dst = ctypes.create_string_buffer(max(cap, 1))
        n = self.lib.oracle_lz4_decompress_safe(src, dst, len(src), cap)
        return n, dst.raw[: max(n, 0)]

    def zstd_decompress(self, src: bytes, cap: int):
        dst = ctypes.create_string_buffer(max(cap, 1))
        n = self.lib.oracle_zstd_decompress(src, len(src), dst, cap)
        return n, dst.raw[: max(n, 0)]

    def crc32c(self, data: bytes, crc: int = 0) -> int:
        """crc32.Update(crc, crc32c, data) (pkg/object/checksum.go:30-45)"""
        return self.lib.oracle_crc32c_update(crc, data, len(data))

    def crc32c_segments(self, data: bytes, seg: int = 32 << 10) -> bytes:
        """disk_cache_file.go checksum(): big-endian CRC-32C per seg bytes"""
        words = (len(data) - 1) // seg + 1 if len(data) else 1
        out = ctypes.create_string_buffer(4 * words)
        n = self.lib.oracle_crc32c_segments(data, len(data), seg, out)
        return out.raw[:n]

    def aes256gcm_seal(self, key: bytes, nonce: bytes, pt: bytes) -> bytes:
        """aead.Seal(nil, nonce, pt, nil) (pkg/object/encrypt.go:255)"""
        out = ctypes.create_string_buffer(len(pt) + 16)
        n = self.lib.oracle_aes256gcm_seal(key, nonce, pt, len(pt), out)
        return out.raw[:n]

    def aes256gcm_open(self, key: bytes, nonce: bytes, ct: bytes):
        """aead.Open; None when the tag does not verify"""
        out = ctypes.create_string_buffer(max(len(ct) - 16, 1))
        n = self.lib.oracle_aes256gcm_open(key, nonce, ct, len(ct), out)
        return None if n < 0 else out.raw[:n]

    def zstd_strict_reserved(self, on: bool):
        self.lib.oracle_zstd_set_strict_reserved(1 if on else 0)

    def xxh64(self, b: bytes, seed: int = 0) -> int:
        return self.lib.oracle_xxh64(b, len(b), seed)
