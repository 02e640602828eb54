"""CPU: libjfsgpu.so loads, exports every symbol include/jfs_gpucodec.h
declares, and its host-only surface behaves like pkg/compress.  No GPU compute
is called here."""
import ctypes
import os
import re

from juicefs_amd import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "jfs_gpucodec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(jfs_[a-z0-9_]+)\s*\(", src)))


def test_exports_every_header_symbol(lib):
    names = header_functions()
    assert len(names) >= 14
    assert sorted(L.EXPORTS) == names
    for n in names:
        assert hasattr(lib, n), n


def test_new_compressor_names(lib):
    # compress.go:39-49 (case-insensitive), Name() strings :53,76,109
    for s, a in [(b"zstd", 2), (b"ZSTD", 2), (b"Zstd", 2), (b"lz4", 1), (b"LZ4", 1), (b"none", 0), (b"", 0),
                 (b"NONE", 0), (b"gzip", -1), (b"lz4hc", -1)]:
        assert lib.jfs_codec_from_name(s) == a
    assert lib.jfs_codec_name(0) == b"Noop" and lib.jfs_codec_name(1) == b"LZ4" and lib.jfs_codec_name(2) == b"Zstd"
    assert lib.jfs_codec_name(7) is None


def test_compress_bound(lib):
    # LZ4_compressBound / ZSTD_COMPRESSBOUND
    assert lib.jfs_compress_bound(1, 4 << 20) == 4210768
    assert lib.jfs_compress_bound(1, 64 << 10) == 65809  # liblz4 1.9.3 (SURVEY a4 says 65,808: off by one)
    assert lib.jfs_compress_bound(1, 0) == 16
    assert lib.jfs_compress_bound(1, 0x7E000001) == 0
    assert lib.jfs_compress_bound(2, 4 << 20) == 4210688
    assert lib.jfs_compress_bound(2, 0) == 64
    assert lib.jfs_compress_bound(2, 3) == 66 and lib.jfs_compress_bound(2, 4) == 67
    assert lib.jfs_compress_bound(0, 12345) == 12345


def test_noop_is_copy_with_short_buffer_error(lib):
    # compress.go:55-68
    src = b"Noop"
    dst = ctypes.create_string_buffer(4)
    assert lib.jfs_compress(0, dst, 4, src, 4) == 4 and dst.raw == src
    assert lib.jfs_compress(0, dst, 1, src, 4) == L.JFS_ERR_SHORT_BUFFER
    assert lib.jfs_decompress(0, dst, 1, src, 4) == L.JFS_ERR_SHORT_BUFFER


def test_empty_input_errors_before_device(lib):
    dst = ctypes.create_string_buffer(100)
    # LZ4.Decompress empty -> "decompress an empty input" (compress.go:121-123)
    assert lib.jfs_decompress(1, dst, 100, None, 0) == L.JFS_ERR_EMPTY_INPUT
    # zstd.Decompress empty -> ErrEmptySlice
    assert lib.jfs_decompress(2, dst, 100, None, 0) == L.JFS_ERR_EMPTY_INPUT


def test_version(lib):
    assert b"gfx950" in lib.jfs_version()
