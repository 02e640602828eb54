"""Loader for libjfsgpu.so (the HIP kernels + C ABI in include/jfs_gpucodec.h).

The library is built in-tree (``juicefs_amd/lib/libjfsgpu.so``) by
``__graft_entry__.build()`` / ``make -C juicefs_amd/csrc``.  There is no
fallback: if the library is missing, importing the codec raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("JFS_GPU_LIB") or os.path.join(_HERE, "lib", "libjfsgpu.so")

ALGO_NONE, ALGO_LZ4, ALGO_ZSTD = 0, 1, 2
JFS_OK = 0
JFS_ERR_BASE = -(1 << 40)  # library codes are <= this; LZ4 decode errors are int32
JFS_ERR_SHORT_BUFFER = JFS_ERR_BASE - 1
JFS_ERR_EMPTY_INPUT = JFS_ERR_BASE - 2
JFS_ERR_CORRUPT = JFS_ERR_BASE - 3
JFS_ERR_COMPRESS_FAIL = JFS_ERR_BASE - 4
JFS_ERR_UNSUPPORTED = JFS_ERR_BASE - 5
JFS_ERR_NO_DEVICE = JFS_ERR_BASE - 6
JFS_ERR_INVALID = JFS_ERR_BASE - 7
JFS_ERR_HIP = JFS_ERR_BASE - 8
JFS_ERR_NO_MEMORY = JFS_ERR_BASE - 9
JFS_ERR_AUTH = JFS_ERR_BASE - 10

# every symbol include/jfs_gpucodec.h declares
EXPORTS = [
    "jfs_codec_from_name", "jfs_codec_name", "jfs_compress_bound", "jfs_compress", "jfs_decompress",
    "jfs_compress_batch", "jfs_decompress_batch", "jfs_lz4_decompress_device", "jfs_lz4_compress_device",
    "jfs_zstd_decompress_device", "jfs_zstd_compress_device", "jfs_device_count", "jfs_version", "jfs_gen_blocks_device",
    "jfs_gen_block_host", "jfs_release_staging", "jfs_crc32c_device", "jfs_aes256gcm_seal_device",
    "jfs_aes256gcm_open_device", "jfs_lz4_compress_seal_device", "jfs_open_lz4_decompress_device",
    "jfs_gpu_mode", "jfs_stats", "jfs_stats_reset", "jfs_device_stats", "jfs_lz4_decompress_device_small",
    "jfs_lz4_split_counts", "jfs_zstd_split_counts", "jfs_lz4_compress_device_small", "jfs_lz4_eseg_counts", "jfs_cipher_from_name", "jfs_cipher_key_size", "jfs_aead_seal_device",
    "jfs_aead_open_device", "jfs_envelope_bound", "jfs_envelope_parse", "jfs_compress_seal_batch",
    "jfs_open_decompress_batch", "jfs_compress_batch_crc", "jfs_decompress_batch_csum", "jfs_deal_plan",
    "jfs_test_spread_locking", "jfs_compress_batch_mixed", "jfs_decompress_batch_mixed",
]

MODE_OFF, MODE_AUTO, MODE_FORCE = 0, 1, 2
CIPHER_AES256GCM, CIPHER_CHACHA20POLY1305, CIPHER_SM4GCM = 0, 1, 2
STATS_N = 6  # index algo * 2 + dir (0 compress, 1 decompress)


class JfsIov(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("src_len", ctypes.c_int64),
                ("dst", ctypes.c_void_p), ("dst_cap", ctypes.c_int64)]


class JfsOpStats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in ("calls", "blocks", "bytes_in", "bytes_out", "errors", "nanos",
                                               "batches")]


class JfsDeviceStat(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("pad_", ctypes.c_int32), ("batches", ctypes.c_uint64),
                ("blocks", ctypes.c_uint64)]


class JfsSealParam(ctypes.Structure):
    _fields_ = [("key", ctypes.c_void_p), ("nonce", ctypes.c_void_p), ("wrapped", ctypes.c_void_p),
                ("wrapped_len", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class JfsDevBlock(ctypes.Structure):
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p),
                ("src_len", ctypes.c_int32), ("dst_cap", ctypes.c_int32)]


_lib = None


def load() -> ctypes.CDLL:
    """Load libjfsgpu.so; raises if it has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make -C juicefs_amd/csrc` (or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    i64, i32, vp, u32 = ctypes.c_int64, ctypes.c_int32, ctypes.c_void_p, ctypes.c_uint32
    lib.jfs_codec_from_name.argtypes = [ctypes.c_char_p]
    lib.jfs_codec_from_name.restype = ctypes.c_int
    lib.jfs_codec_name.argtypes = [ctypes.c_int]
    lib.jfs_codec_name.restype = ctypes.c_char_p
    lib.jfs_compress_bound.argtypes = [ctypes.c_int, i64]
    lib.jfs_compress_bound.restype = i64
    for f in (lib.jfs_compress, lib.jfs_decompress):
        f.argtypes = [ctypes.c_int, vp, i64, vp, i64]
        f.restype = i64
    for f in (lib.jfs_compress_batch, lib.jfs_decompress_batch):
        f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(JfsIov), ctypes.POINTER(i64), u32]
        f.restype = i64
    for f in (lib.jfs_lz4_decompress_device, lib.jfs_lz4_compress_device, lib.jfs_zstd_decompress_device,
              lib.jfs_zstd_compress_device):
        f.argtypes = [vp, ctypes.c_int, vp, vp]
        f.restype = i64
    lib.jfs_lz4_decompress_device_small.argtypes = [vp, vp, vp, ctypes.c_int, vp, vp]
    lib.jfs_lz4_decompress_device_small.restype = i64
    lib.jfs_lz4_split_counts.argtypes = [vp, ctypes.c_int]
    lib.jfs_lz4_split_counts.restype = ctypes.c_int
    lib.jfs_zstd_split_counts.argtypes = [vp, ctypes.c_int]
    lib.jfs_zstd_split_counts.restype = ctypes.c_int
    lib.jfs_lz4_compress_device_small.argtypes = [vp, vp, ctypes.c_int, vp, vp]
    lib.jfs_lz4_compress_device_small.restype = ctypes.c_int64
    lib.jfs_lz4_eseg_counts.argtypes = [vp, ctypes.c_int]
    lib.jfs_lz4_eseg_counts.restype = ctypes.c_int
    lib.jfs_cipher_from_name.argtypes = [ctypes.c_char_p]
    lib.jfs_cipher_from_name.restype = ctypes.c_int
    lib.jfs_cipher_key_size.argtypes = [ctypes.c_int]
    lib.jfs_cipher_key_size.restype = ctypes.c_int
    for f in (lib.jfs_aead_seal_device, lib.jfs_aead_open_device):
        f.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, vp]
        f.restype = i64
    lib.jfs_envelope_bound.argtypes = [ctypes.c_int, i64, i32]
    lib.jfs_envelope_bound.restype = i64
    lib.jfs_envelope_parse.argtypes = [vp, i64] + [ctypes.POINTER(i64)] * 4
    lib.jfs_envelope_parse.restype = i64
    lib.jfs_compress_seal_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(JfsIov),
                                            ctypes.POINTER(JfsSealParam), ctypes.POINTER(i64), vp, u32]
    lib.jfs_compress_batch_crc.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(JfsIov), ctypes.POINTER(i64),
                                           vp, u32]
    lib.jfs_compress_batch_crc.restype = i64
    lib.jfs_decompress_batch_csum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(JfsIov), ctypes.POINTER(i64),
                                              ctypes.POINTER(ctypes.c_void_p), u32]
    lib.jfs_decompress_batch_csum.restype = i64
    lib.jfs_deal_plan.argtypes = [ctypes.POINTER(i64), ctypes.c_int, ctypes.c_int, ctypes.POINTER(i32)]
    lib.jfs_deal_plan.restype = None
    for f in (lib.jfs_compress_batch_mixed, lib.jfs_decompress_batch_mixed):
        f.argtypes = [ctypes.POINTER(i32), ctypes.c_int, ctypes.POINTER(JfsIov), ctypes.POINTER(i64), u32]
        f.restype = i64
    lib.jfs_test_spread_locking.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.jfs_test_spread_locking.restype = i64
    lib.jfs_compress_seal_batch.restype = i64
    lib.jfs_open_decompress_batch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.POINTER(JfsIov),
                                              ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(i64), u32]
    lib.jfs_open_decompress_batch.restype = i64
    lib.jfs_crc32c_device.argtypes = [vp, ctypes.c_int, ctypes.c_int32, vp, vp, vp]
    lib.jfs_crc32c_device.restype = i64
    for f in (lib.jfs_aes256gcm_seal_device, lib.jfs_aes256gcm_open_device):
        f.argtypes = [vp, ctypes.c_int, vp, vp]
        f.restype = i64
    for f in (lib.jfs_lz4_compress_seal_device, lib.jfs_open_lz4_decompress_device):
        f.argtypes = [vp, vp, ctypes.c_int, vp, vp, vp]
        f.restype = i64
    lib.jfs_release_staging.argtypes = []
    lib.jfs_release_staging.restype = None
    lib.jfs_device_count.argtypes = []
    lib.jfs_device_count.restype = ctypes.c_int
    lib.jfs_gpu_mode.argtypes = []
    lib.jfs_gpu_mode.restype = ctypes.c_int
    lib.jfs_stats.argtypes = [ctypes.POINTER(JfsOpStats), ctypes.c_int]
    lib.jfs_stats.restype = ctypes.c_int
    lib.jfs_device_stats.argtypes = [ctypes.POINTER(JfsDeviceStat), ctypes.c_int]
    lib.jfs_device_stats.restype = ctypes.c_int
    lib.jfs_stats_reset.argtypes = []
    lib.jfs_stats_reset.restype = None
    lib.jfs_version.argtypes = []
    lib.jfs_version.restype = ctypes.c_char_p
    lib.jfs_gen_blocks_device.argtypes = [vp, ctypes.c_int, i64, ctypes.c_char, ctypes.c_uint64, vp]
    lib.jfs_gen_blocks_device.restype = i64
    lib.jfs_gen_block_host.argtypes = [vp, i64, ctypes.c_char, ctypes.c_uint64]
    lib.jfs_gen_block_host.restype = None
    lib.jfs_selftest_wave.argtypes = [vp, vp]
    lib.jfs_selftest_wave.restype = ctypes.c_int
    _lib = lib
    return lib
