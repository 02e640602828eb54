"""Device-resident batch helpers (torch tensors in HBM -> libjfsgpu device API).

PyTorch is only plumbing here: it owns the HBM allocations and the stream; the
byte work is the HIP kernels behind ``jfs_lz4_decompress_device`` /
``jfs_lz4_compress_device`` / ``jfs_zstd_decompress_device``.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib as L

DESC_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("src_len", "<i4"), ("dst_cap", "<i4")])
assert DESC_DTYPE.itemsize == ctypes.sizeof(L.JfsDevBlock)


def make_desc(src: torch.Tensor, src_offs, src_lens, dst: torch.Tensor, dst_offs, dst_caps) -> torch.Tensor:
    """Build a device tensor of jfs_dev_block descriptors (24 bytes each)."""
    n = len(src_offs)
    a = np.zeros(n, dtype=DESC_DTYPE)
    a["src"] = src.data_ptr() + np.asarray(src_offs, dtype=np.uint64)
    a["dst"] = dst.data_ptr() + np.asarray(dst_offs, dtype=np.uint64)
    a["src_len"] = np.asarray(src_lens, dtype=np.int32)
    a["dst_cap"] = np.asarray(dst_caps, dtype=np.int32)
    t = torch.from_numpy(a.view(np.uint8).copy())
    return t.to(src.device)


def _stream_ptr(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {rc}")


def lz4_decompress(desc: torch.Tensor, ret: torch.Tensor, stream=None):
    n = desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_lz4_decompress_device(desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_lz4_decompress_device")


def lz4_compress(desc: torch.Tensor, ret: torch.Tensor, stream=None):
    n = desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_lz4_compress_device(desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_lz4_compress_device")


def lz4_decompress_small(desc: torch.Tensor, ret: torch.Tensor, src_lens, dst_caps, stream=None):
    """jfs_lz4_decompress_device_small: few blocks, each spread over the GPU;
    src_lens / dst_caps are host copies of the descriptors' sizes."""
    n = desc.numel() // DESC_DTYPE.itemsize
    sl = (ctypes.c_int32 * max(n, 1))(*[int(x) for x in src_lens])
    dc = (ctypes.c_int32 * max(n, 1))(*[int(x) for x in dst_caps])
    _check(L.load().jfs_lz4_decompress_device_small(desc.data_ptr(), sl, dc, n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_lz4_decompress_device_small")


def lz4_split_counts(reset: bool = False):
    """(blocks the small-batch path decoded itself, blocks it handed to the
    one-workgroup kernel, ... the reasons: fix-up, jumping, token, no last run)
    on the current device."""
    out = (ctypes.c_uint64 * 6)()
    _check(L.load().jfs_lz4_split_counts(out, 1 if reset else 0), "jfs_lz4_split_counts")
    return tuple(int(x) for x in out)


def zstd_split_counts(reset: bool = False):
    """(inputs the Zstd small-batch path replayed itself, inputs it handed to
    the exact one-wave replay) on the current device."""
    out = (ctypes.c_uint64 * 2)()
    _check(L.load().jfs_zstd_split_counts(out, 1 if reset else 0), "jfs_zstd_split_counts")
    return tuple(int(x) for x in out)


def lz4_compress_small(desc: torch.Tensor, ret: torch.Tensor, src_lens, stream=None):
    """jfs_lz4_compress_device_small: few blocks, each parsed as segments
    across the GPU (same bytes as lz4_compress); src_lens = host copies."""
    n = desc.numel() // DESC_DTYPE.itemsize
    sl = (ctypes.c_int32 * max(n, 1))(*[int(x) for x in src_lens])
    _check(L.load().jfs_lz4_compress_device_small(desc.data_ptr(), sl, n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_lz4_compress_device_small")


def lz4_eseg_counts(reset: bool = False):
    """Segment encoder: {rounds: blocks settled after that many rounds}, with
    0 = blocks handed to the serial kernel."""
    out = (ctypes.c_uint64 * 17)()
    _check(L.load().jfs_lz4_eseg_counts(out, 1 if reset else 0), "jfs_lz4_eseg_counts")
    return {i: int(x) for i, x in enumerate(out) if x}


def zstd_decompress(desc: torch.Tensor, ret: torch.Tensor, stream=None):
    n = desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_zstd_decompress_device(desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_zstd_decompress_device")


def zstd_decompress_sync(desc: torch.Tensor, ret: torch.Tensor, stream=None):
    """zstd_decompress, waited for.  The library sizes its scratch inside the
    call (include/jfs_gpucodec.h), so there is never anything to resubmit."""
    zstd_decompress(desc, ret, stream)
    torch.cuda.synchronize()


def zstd_compress(desc: torch.Tensor, ret: torch.Tensor, stream=None):
    n = desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_zstd_compress_device(desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)),
           "jfs_zstd_compress_device")


def crc32c(desc: torch.Tensor, crc: torch.Tensor | None = None, ret: torch.Tensor | None = None,
           seg_bytes: int = 0, stream=None):
    """CRC-32C per descriptor (jfs_crc32c_device): whole-block values into
    `crc` (uint32 as int32 tensor), per-segment big-endian sums into each dst."""
    n = desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_crc32c_device(desc.data_ptr(), n, seg_bytes, crc.data_ptr() if crc is not None else None,
                                      ret.data_ptr() if ret is not None else None, _stream_ptr(stream)),
           "jfs_crc32c_device")


AEAD_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("src_len", "<i4"), ("dst_cap", "<i4"),
                       ("key", "<u8"), ("nonce", "<u8")])


def make_aead_desc(src: torch.Tensor, src_offs, src_lens, dst: torch.Tensor, dst_offs, dst_caps,
                   kn: torch.Tensor, key_offs, nonce_offs) -> torch.Tensor:
    """jfs_aead_block descriptors (40 bytes each); keys and nonces live in `kn`."""
    a = np.zeros(len(src_offs), dtype=AEAD_DTYPE)
    a["src"] = src.data_ptr() + np.asarray(src_offs, dtype=np.uint64)
    a["dst"] = dst.data_ptr() + np.asarray(dst_offs, dtype=np.uint64)
    a["src_len"] = np.asarray(src_lens, dtype=np.int32)
    a["dst_cap"] = np.asarray(dst_caps, dtype=np.int32)
    a["key"] = kn.data_ptr() + np.asarray(key_offs, dtype=np.uint64)
    a["nonce"] = kn.data_ptr() + np.asarray(nonce_offs, dtype=np.uint64)
    return torch.from_numpy(a.view(np.uint8).copy()).to(src.device)


def aes256gcm(desc: torch.Tensor, ret: torch.Tensor, seal: bool, stream=None):
    """AES-256-GCM seal (True) or open (False) per jfs_aead_block descriptor."""
    n = desc.numel() // AEAD_DTYPE.itemsize
    lib = L.load()
    fn = lib.jfs_aes256gcm_seal_device if seal else lib.jfs_aes256gcm_open_device
    _check(fn(desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)), "jfs_aes256gcm")


CIPHERS = {"aes256gcm": L.CIPHER_AES256GCM, "chacha20": L.CIPHER_CHACHA20POLY1305, "sm4gcm": L.CIPHER_SM4GCM}


def aead(cipher: str, desc: torch.Tensor, ret: torch.Tensor, seal: bool, stream=None):
    """Seal (True) or open (False) with aes256gcm / chacha20 / sm4gcm per descriptor
    (jfs_aead_{seal,open}_device)."""
    n = desc.numel() // AEAD_DTYPE.itemsize
    lib = L.load()
    fn = lib.jfs_aead_seal_device if seal else lib.jfs_aead_open_device
    _check(fn(CIPHERS[cipher], desc.data_ptr(), n, ret.data_ptr(), _stream_ptr(stream)), "jfs_aead")


JFS_CHAIN_FAILED = -(1 << 31)  # the first step of a fused chain failed for this block


def lz4_compress_seal(comp_desc: torch.Tensor, aead_desc: torch.Tensor, ret_comp: torch.Tensor, ret: torch.Tensor,
                      stream=None):
    """Fused LZ4 compress -> AES-256-GCM seal (jfs_lz4_compress_seal_device)."""
    n = comp_desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_lz4_compress_seal_device(comp_desc.data_ptr(), aead_desc.data_ptr(), n, ret_comp.data_ptr(),
                                                 ret.data_ptr(), _stream_ptr(stream)), "jfs_lz4_compress_seal_device")


def open_lz4_decompress(aead_desc: torch.Tensor, dec_desc: torch.Tensor, ret_open: torch.Tensor, ret: torch.Tensor,
                        stream=None):
    """Fused AES-256-GCM open -> LZ4 decompress (jfs_open_lz4_decompress_device)."""
    n = dec_desc.numel() // DESC_DTYPE.itemsize
    _check(L.load().jfs_open_lz4_decompress_device(aead_desc.data_ptr(), dec_desc.data_ptr(), n, ret_open.data_ptr(),
                                                   ret.data_ptr(), _stream_ptr(stream)), "jfs_open_lz4_decompress_device")


def gen_blocks(out: torch.Tensor, nblk: int, block_bytes: int, cls: str, seed_base: int, stream=None):
    """Fill out[0 : nblk*block_bytes] with synthetic blocks."""
    assert out.numel() >= nblk * block_bytes
    _check(L.load().jfs_gen_blocks_device(out.data_ptr(), nblk, block_bytes, cls.encode(), seed_base,
                                          _stream_ptr(stream)), "jfs_gen_blocks_device")


def lz4_bound(n: int) -> int:
    return n + n // 255 + 16


class Lz4Batch:
    """A batch of equal-size blocks resident in HBM: raw, compressed, decoded.

    Compressed block i lives at comp[i*slot : i*slot + csize[i]] with
    slot = bound rounded up to 256 bytes (16-byte aligned slots).
    """

    def __init__(self, nblk: int, block_bytes: int, cls: str = "T", seed_base: int = 1, device="cuda"):
        self.nblk, self.U = nblk, block_bytes
        self.slot = (lz4_bound(block_bytes) + 255) // 256 * 256
        self.device = torch.device(device)
        self.raw = torch.empty(nblk * block_bytes, dtype=torch.uint8, device=self.device)
        gen_blocks(self.raw, nblk, block_bytes, cls, seed_base)
        self.comp = torch.empty(nblk * self.slot, dtype=torch.uint8, device=self.device)
        self.ret = torch.empty(nblk, dtype=torch.int32, device=self.device)
        offs = np.arange(nblk, dtype=np.int64)
        self.enc_desc = make_desc(self.raw, offs * block_bytes, [block_bytes] * nblk, self.comp, offs * self.slot,
                                  [self.slot] * nblk)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lz4_compress(self.enc_desc, self.ret)
        e1.record()
        torch.cuda.synchronize()
        self.enc_ms = e0.elapsed_time(e1)  # one GPU LZ4 encode launch over the whole batch
        self.csize = self.ret.cpu().numpy().astype(np.int64)
        if (self.csize <= 0).any():
            raise RuntimeError("device LZ4 compression failed")
        self.out = torch.empty(nblk * block_bytes, dtype=torch.uint8, device=self.device)
        self.dec_desc = make_desc(self.comp, offs * self.slot, self.csize, self.out, offs * block_bytes,
                                  [block_bytes] * nblk)
        self.dec_ret = torch.empty(nblk, dtype=torch.int32, device=self.device)

    def decompress(self, stream=None):
        lz4_decompress(self.dec_desc, self.dec_ret, stream)

    def compress(self, stream=None):
        """Re-encode raw -> comp (same bytes and sizes as the first encode)."""
        lz4_compress(self.enc_desc, self.ret, stream)

    @property
    def comp_bytes(self) -> int:
        return int(self.csize.sum())

    def verify(self) -> bool:
        torch.cuda.synchronize()
        ok = bool((self.dec_ret == self.U).all().item())
        ok = ok and bool((self.ret.cpu().numpy().astype(np.int64) == self.csize).all())
        return ok and bool(torch.equal(self.out, self.raw))


def zstd_bound(n: int) -> int:
    return n + (n >> 8) + (((128 << 10) - n) >> 11 if n < (128 << 10) else 0)


def zstd_compress_rate(nblk: int, block_bytes: int, cls: str = "T", seed_base: int = 1, device="cuda"):
    """Time one GPU Zstd encode launch over nblk synthetic blocks in HBM and
    check every frame with the GPU decoder.  Returns (GiB/s, ratio, ms)."""
    dev = torch.device(device)
    raw = torch.empty(nblk * block_bytes, dtype=torch.uint8, device=dev)
    gen_blocks(raw, nblk, block_bytes, cls, seed_base)
    slot = (zstd_bound(block_bytes) + 255) // 256 * 256
    comp = torch.empty(nblk * slot, dtype=torch.uint8, device=dev)
    offs = np.arange(nblk, dtype=np.int64)
    desc = make_desc(raw, offs * block_bytes, [block_bytes] * nblk, comp, offs * slot, [slot] * nblk)
    ret = torch.empty(nblk, dtype=torch.int32, device=dev)
    zstd_compress(desc, ret)  # warm-up (scratch allocation)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    zstd_compress(desc, ret)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    csize = ret.cpu().numpy().astype(np.int64)
    if (csize <= 0).any():
        raise RuntimeError("device Zstd compression failed")
    out = torch.empty(nblk * block_bytes, dtype=torch.uint8, device=dev)
    ddesc = make_desc(comp, offs * slot, csize, out, offs * block_bytes, [block_bytes] * nblk)
    dret = torch.empty(nblk, dtype=torch.int32, device=dev)
    zstd_decompress_sync(ddesc, dret)
    if not (bool((dret == block_bytes).all().item()) and torch.equal(out, raw)):
        raise RuntimeError("Zstd round trip mismatch")
    return nblk * block_bytes / (ms / 1e3) / 2**30, nblk * block_bytes / float(csize.sum()), ms


def _libzstd():
    """The system libzstd (data generator for benchmarks only: it produces the
    level-3 frames the GPU decodes; nothing on the product path uses it)."""
    for path in ("/opt/conda/lib/libzstd.so.1", "/usr/lib/x86_64-linux-gnu/libzstd.so.1"):
        try:
            z = ctypes.CDLL(path)
        except OSError:
            continue
        z.ZSTD_compress.restype = ctypes.c_size_t
        z.ZSTD_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        z.ZSTD_compressBound.restype = ctypes.c_size_t
        z.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
        z.ZSTD_isError.restype = ctypes.c_uint
        z.ZSTD_isError.argtypes = [ctypes.c_size_t]
        z.ZSTD_decompress.restype = ctypes.c_size_t
        z.ZSTD_decompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t]
        z.path = path
        return z
    return None


class ZstdBatch:
    """nblk Zstd frames (level `level`, block_bytes each) resident in HBM.

    `distinct` different blocks are generated (GPU generator) and compressed
    with the system libzstd on the host, then replicated over the nblk slots
    (the GPU sees nblk independent frames; the bench uses 256 distinct frames,
    ~300 MB of compressed input, beyond the 256 MB MALL).  Slot = max frame size rounded up to 256 B.
    """

    def __init__(self, nblk: int, block_bytes: int, cls: str = "T", level: int = 3, distinct: int = 16,
                 seed_base: int = 1, device="cuda", cache_dir: str | None = None):
        from .blockgen import gen_block
        self.nblk, self.U, self.level = nblk, block_bytes, level
        self.device = torch.device(device)
        distinct = min(distinct, nblk)
        raws, frames = [], []
        cache = None
        if cache_dir:
            cache = os.path.join(cache_dir, f"zstd_{cls}_{block_bytes}_{level}_{distinct}_{seed_base}.npz")
        # the raw blocks come from the GPU generator (the host one takes ~0.5 s
        # per 4 MiB text block); frames from host libzstd on a thread pool
        # (ctypes drops the GIL inside ZSTD_compress)
        raw_t = torch.empty(distinct * block_bytes, dtype=torch.uint8, device=self.device)
        gen_blocks(raw_t, distinct, block_bytes, cls, seed_base)
        raw_np = raw_t.cpu().numpy()
        raws = [raw_np[i * block_bytes:(i + 1) * block_bytes].tobytes() for i in range(distinct)]
        del raw_t
        if cache and os.path.exists(cache):
            with np.load(cache) as f:  # our own file (allow_pickle stays False)
                blob, lens = f["blob"], f["lens"]
            o = 0
            for n in lens:
                frames.append(blob[o:o + n].tobytes())
                o += n
        else:
            z = _libzstd()
            if z is None:
                raise RuntimeError("no libzstd on this host to generate frames")

            def one(src):
                cap = z.ZSTD_compressBound(len(src))
                dst = ctypes.create_string_buffer(cap)
                n = z.ZSTD_compress(dst, cap, src, len(src), level)
                if z.ZSTD_isError(n):
                    raise RuntimeError("ZSTD_compress failed")
                return dst.raw[:n]
            from concurrent.futures import ThreadPoolExecutor
            with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:
                frames = list(ex.map(one, raws))
            if cache:
                os.makedirs(cache_dir, exist_ok=True)
                np.savez(cache, blob=np.frombuffer(b"".join(frames), dtype=np.uint8),
                         lens=np.array([len(f) for f in frames], dtype=np.int64))
        self.frames = frames
        self.slot = (max(len(f) for f in frames) + 255) // 256 * 256
        host = np.zeros(nblk * self.slot, dtype=np.uint8)
        self.csize = np.zeros(nblk, dtype=np.int64)
        for i in range(nblk):
            f = frames[i % distinct]
            host[i * self.slot:i * self.slot + len(f)] = np.frombuffer(f, dtype=np.uint8)
            self.csize[i] = len(f)
        self.comp = torch.from_numpy(host).to(self.device)
        self.raw = torch.from_numpy(np.frombuffer(b"".join(raws), dtype=np.uint8).copy()).to(self.device)
        self.distinct = distinct
        self.out = torch.empty(nblk * block_bytes, dtype=torch.uint8, device=self.device)
        offs = np.arange(nblk, dtype=np.int64)
        self.dec_desc = make_desc(self.comp, offs * self.slot, self.csize, self.out, offs * block_bytes,
                                  [block_bytes] * nblk)
        self.dec_ret = torch.empty(nblk, dtype=torch.int32, device=self.device)
        zstd_decompress_sync(self.dec_desc, self.dec_ret)  # sizes the device scratch for this batch

    def decompress(self, stream=None):
        zstd_decompress(self.dec_desc, self.dec_ret, stream)

    @property
    def comp_bytes(self) -> int:
        return int(self.csize.sum())

    def verify(self) -> bool:
        torch.cuda.synchronize()
        if not bool((self.dec_ret == self.U).all().item()):
            return False
        U, d = self.U, self.distinct
        for i in range(self.nblk):
            j = i % d
            if not torch.equal(self.out[i * U:(i + 1) * U], self.raw[j * U:(j + 1) * U]):
                return False
        return True
