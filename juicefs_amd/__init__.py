"""juicefs_amd -- MI355X-native block compression engine for JuiceFS's pkg/compress.

``juicefs_amd.compress`` mirrors the reference Go package
(/root/reference/pkg/compress/compress.go): ``NewCompressor``, ``Compressor``,
``LZ4``, ``ZStandard``, ``ZSTD_LEVEL``.  The byte work runs in HIP kernels for
gfx950 inside ``lib/libjfsgpu.so`` (C ABI: include/jfs_gpucodec.h).
"""
from . import _lib  # noqa: F401

__all__ = ["compress", "device"]
