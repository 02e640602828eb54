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
        lib.oracle_sm4_encrypt_block.argtypes = [vp, vp, vp]
        for f in (lib.oracle_sm4gcm_seal, lib.oracle_sm4gcm_open):
            f.argtypes = [vp, vp, vp, i64, vp]
            f.restype = i64
        for f in (lib.oracle_chacha20poly1305_seal, lib.oracle_chacha20poly1305_open):
            f.argtypes = [vp, vp, vp, i64, vp, i64, vp]
            f.restype = i64
        lib.oracle_chacha20_block.argtypes = [vp, ctypes.c_uint32, vp, vp]
        lib.oracle_poly1305.argtypes = [vp, vp, i64, vp]
        lib.oracle_envelope_write.argtypes = [vp, i64, vp, i64, vp, i64, vp]
        lib.oracle_envelope_write.restype = i64
        lib.oracle_envelope_parse.argtypes = [vp, i64, ctypes.POINTER(i64), ctypes.POINTER(i64)]
        lib.oracle_envelope_parse.restype = i64
        if hasattr(lib, "oracle_zstd_compress_l1_ex"):
            lib.oracle_zstd_compress_l1_ex.argtypes = [vp, i64, vp, i64, vp]
            lib.oracle_zstd_compress_l1_ex.restype = i64
            lib.oracle_zstd_l1_params.argtypes = [i64, vp]
        self.has_zstd = hasattr(lib, "oracle_zstd_decompress")
        if self.has_zstd:
            lib.oracle_zstd_decompress.argtypes = [vp, i64, vp, i64]
            lib.oracle_zstd_decompress.restype = i64
            lib.oracle_zstd_set_strict_reserved.argtypes = [i32]
            lib.oracle_zstd_frame_content_size.argtypes = [vp, i64]
            lib.oracle_zstd_frame_content_size.restype = i64
            lib.oracle_xxh64.argtypes = [vp, ctypes.c_size_t, ctypes.c_uint64]
            lib.oracle_xxh64.restype = ctypes.c_uint64

    def zstd_compress_l1(self, src: bytes) -> bytes:
        """libzstd 1.4.9 ZSTD_compress(level 1), restated (oracle/zstd_l1_oracle.c)."""
        n = len(src)
        cap = n + (n >> 8) + (((128 << 10) - n) >> 11 if n < (128 << 10) else 0) + 64
        dst = ctypes.create_string_buffer(cap)
        r = self.lib.oracle_zstd_compress_l1_ex(src, n, dst, cap, None)
        assert r > 0
        return dst.raw[:r]

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

    # ---- SM4-GCM / ChaCha20-Poly1305 / the object envelope (aead_oracle.c) ----
    def sm4_block(self, key: bytes, block: bytes) -> bytes:
        out = ctypes.create_string_buffer(16)
        self.lib.oracle_sm4_encrypt_block(key, block, out)
        return out.raw

    def seal(self, cipher: str, key: bytes, nonce: bytes, pt: bytes, aad: bytes = b"") -> bytes:
        """aead.Seal(nil, nonce, pt, aad) for cipher in aes256gcm / chacha20 / sm4gcm"""
        out = ctypes.create_string_buffer(len(pt) + 16)
        if cipher == "aes256gcm":
            assert not aad
            n = self.lib.oracle_aes256gcm_seal(key, nonce, pt, len(pt), out)
        elif cipher == "sm4gcm":
            assert not aad
            n = self.lib.oracle_sm4gcm_seal(key, nonce, pt, len(pt), out)
        else:
            n = self.lib.oracle_chacha20poly1305_seal(key, nonce, aad, len(aad), pt, len(pt), out)
        return out.raw[:n]

    def open(self, cipher: str, key: bytes, nonce: bytes, ct: bytes, aad: bytes = b""):
        """aead.Open; None when the tag does not verify"""
        out = ctypes.create_string_buffer(max(len(ct) - 16, 1))
        if cipher == "aes256gcm":
            n = self.lib.oracle_aes256gcm_open(key, nonce, ct, len(ct), out)
        elif cipher == "sm4gcm":
            n = self.lib.oracle_sm4gcm_open(key, nonce, ct, len(ct), out)
        else:
            n = self.lib.oracle_chacha20poly1305_open(key, nonce, aad, len(aad), ct, len(ct), out)
        return None if n < 0 else out.raw[:n]

    def chacha20_block(self, key: bytes, counter: int, nonce: bytes) -> bytes:
        out = ctypes.create_string_buffer(64)
        self.lib.oracle_chacha20_block(key, counter, nonce, out)
        return out.raw

    def poly1305(self, key: bytes, msg: bytes) -> bytes:
        out = ctypes.create_string_buffer(16)
        self.lib.oracle_poly1305(key, msg, len(msg), out)
        return out.raw

    def envelope(self, wrapped: bytes, nonce: bytes, sealed: bytes) -> bytes:
        """dataEncryptor.Encrypt's output for a given wrapped key, nonce and sealed payload"""
        out = ctypes.create_string_buffer(3 + len(wrapped) + len(nonce) + len(sealed))
        n = self.lib.oracle_envelope_write(wrapped, len(wrapped), nonce, len(nonce), sealed, len(sealed), out)
        return out.raw[:n]

    def envelope_parse(self, env: bytes):
        """(payload offset or -1/-2, wrapped-key length, nonce length)"""
        w, nl = ctypes.c_int64(), ctypes.c_int64()
        r = self.lib.oracle_envelope_parse(env, len(env), ctypes.byref(w), ctypes.byref(nl))
        return r, w.value, nl.value
