"""GPU: the batch C ABI at the BASELINE shapes and its error contract.

* configs[0]: 1024 x 4 MiB text blocks through jfs_compress_batch then
  jfs_decompress_batch (pkg/compress round trip); compressed bytes checked
  against the CPU oracle on a sample, every decoded block byte for byte.
* JuiceFS block sizes above 4 MiB (--block-size up to 16 MiB,
  cmd/format.go:218-234).
* Per-block error isolation: good blocks decode next to
  corrupt, short-capacity and over-sized ones in one coalesced batch.
* The caller's current HIP device is unchanged by the library.
"""
import hashlib
import os
import subprocess
import sys
import threading

import numpy as np
import pytest

from juicefs_amd import _lib as L
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _device_blocks(gpu, nblk, U, seed):
    import torch
    from juicefs_amd import device as D
    raw = np.empty(nblk * U, dtype=np.uint8)
    per = 256
    buf = torch.empty(per * U, dtype=torch.uint8, device=gpu)
    for s in range(0, nblk, per):
        k = min(per, nblk - s)
        D.gen_blocks(buf, k, U, "T", seed + s)
        raw[s * U:(s + k) * U] = buf[:k * U].cpu().numpy()
    return raw


def test_configs0_roundtrip_1024x4MiB(gpu, oracle):
    """BASELINE configs[0] through the C ABI (compress_test.go:25-64 semantics
    per block: bound-sized dst, round trip equal)."""
    nblk, U = 1024, 4 << 20
    raw = _device_blocks(gpu, nblk, U, 31000)
    c = C.LZ4()
    bound = c.CompressBound(U)
    comp = np.zeros(nblk * bound, dtype=np.uint8)
    res = c.CompressBatch([(comp[i * bound:(i + 1) * bound], raw[i * U:(i + 1) * U]) for i in range(nblk)])
    assert all(e is None and n > 0 for n, e in res)
    sizes = [n for n, _ in res]
    for i in (0, 1, 511, 1023):  # compressed bytes == LZ4_compress_default (oracle)
        m, ref = oracle.lz4_compress(raw[i * U:(i + 1) * U].tobytes())
        assert m == sizes[i]
        assert hashlib.sha256(comp[i * bound:i * bound + m].tobytes()).digest() == hashlib.sha256(ref).digest()
    out = np.zeros(nblk * U, dtype=np.uint8)
    res = c.DecompressBatch([(out[i * U:(i + 1) * U], comp[i * bound:i * bound + sizes[i]]) for i in range(nblk)])
    assert all(e is None and n == U for n, e in res)
    for i in range(nblk):
        assert np.array_equal(out[i * U:(i + 1) * U], raw[i * U:(i + 1) * U]), i


@pytest.mark.parametrize("U", [8 << 20, 16 << 20])
def test_large_blocks_lz4_and_zstd(gpu, oracle, U):
    """JuiceFS blocks above 4 MiB (up to 16 MiB): LZ4 byte-exact vs the oracle,
    Zstd round trip, both through the batch ABI; ragged last blocks too."""
    raw = _device_blocks(gpu, 2, U, 77 + U)
    srcs = [raw[:U].tobytes(), raw[U:U + U - 12345].tobytes()]
    lz, zs = C.LZ4(), C.ZStandard()
    pairs = [(bytearray(lz.CompressBound(len(s))), s) for s in srcs]
    res = lz.CompressBatch(pairs)
    for (d, s), (n, e) in zip(pairs, res):
        m, ref = oracle.lz4_compress(s)
        assert e is None and n == m and bytes(d[:n]) == ref
    back = lz.DecompressBatch([(bytearray(len(s)), bytes(d[:n])) for (d, s), (n, _) in zip(pairs, res)])
    assert all(e is None and n == len(s) for s, (n, e) in zip(srcs, back))
    zp = [(bytearray(zs.CompressBound(len(s))), s) for s in srcs]
    zr = zs.CompressBatch(zp)
    assert all(e is None and n > 0 for n, e in zr)
    outs = [bytearray(len(s)) for s in srcs]
    zb = zs.DecompressBatch([(o, bytes(d[:n])) for o, (d, _), (n, _) in zip(outs, zp, zr)])
    for s, o, (n, e) in zip(srcs, outs, zb):
        assert e is None and n == len(s) and bytes(o) == s


def test_error_isolation_in_one_batch(gpu, oracle):
    """Corrupt, short-capacity and huge-hint Zstd blocks next to good ones:
    each reports its own error, the good ones decode."""
    lz, zs = C.LZ4(), C.ZStandard()
    good = [gen_block("T", 600 + i, 70000 + 999 * i) for i in range(6)]
    comps = [oracle.lz4_compress(s)[1] for s in good]
    bad = bytearray(comps[0])
    bad[len(bad) // 2] ^= 0xFF
    bad = bytes(bad[:len(bad) // 2])  # truncated: an LZ4 error
    pairs = [(bytearray(len(s)), c) for s, c in zip(good, comps)]
    pairs.insert(2, (bytearray(len(good[0])), bad))
    pairs.insert(4, (bytearray(10), comps[1]))  # dst too short
    res = lz.DecompressBatch(pairs)
    assert res[2][1] is not None and res[2][0] < 0
    assert res[4][1] is not None and res[4][0] < 0
    gi = [i for i in range(len(pairs)) if i not in (2, 4)]
    for k, i in enumerate(gi):
        n, e = res[i]
        assert e is None and n == len(good[k]) and bytes(pairs[i][0]) == good[k]
    # Zstd: a frame without a content size (huge hint) next to good frames
    z_frames = []
    zp = [(bytearray(zs.CompressBound(len(s))), s) for s in good]
    for (d, _), (n, e) in zip(zp, zs.CompressBatch(zp)):
        assert e is None
        z_frames.append(bytes(d[:n]))
    no_fcs = bytes.fromhex("28b52ffd0000") + b"\x00" * 8  # FCS absent -> hint = 1e6
    zpairs = [(bytearray(len(s)), f) for s, f in zip(good, z_frames)]
    zpairs.insert(1, (bytearray(1000), no_fcs))
    zres = zs.DecompressBatch(zpairs)
    assert zres[1][1] is not None
    for k, i in enumerate([0] + list(range(2, len(zpairs)))):
        n, e = zres[i]
        assert e is None and bytes(zpairs[i][0][:n]) == good[k]


CHILD_NOMEM = r'''
import sys
sys.path.insert(0, sys.argv[1])
from juicefs_amd import compress as C, _lib as L
from juicefs_amd.blockgen import gen_block
lz = C.LZ4()
srcs = [gen_block("T", 40 + i, 1 << 20) for i in range(4)]
comps = []
for s in srcs:
    d = bytearray(lz.CompressBound(len(s)))
    n, e = lz.Compress(d, s)
    assert e is None
    comps.append(bytes(d[:n]))
# one request whose staging (96 MiB of capacity) exceeds JFS_STAGING_MAX_MB=64
pairs = [(bytearray(len(s)), c) for s, c in zip(srcs, comps)]
pairs.insert(1, (bytearray(96 << 20), comps[0]))
res = lz.DecompressBatch(pairs)
assert res[1][1] is not None and res[1][1].code == L.JFS_ERR_NO_MEMORY, res[1]
for i, (n, e) in enumerate(res):
    if i != 1:
        assert e is None and n == 1 << 20
# the same through the one-call API from concurrent threads (the coalescer)
import threading
errs = []
def work(i):
    cap = (96 << 20) if i == 3 else (1 << 20)
    out = bytearray(cap)
    n, e = lz.Decompress(out, comps[i % 4])
    if i == 3:
        if e is None or e.code != L.JFS_ERR_NO_MEMORY: errs.append(("big", n, e))
    elif e is not None or bytes(out[:n]) != srcs[i % 4]:
        errs.append((i, n, e))
th = [threading.Thread(target=work, args=(i,)) for i in range(12)]
[t.start() for t in th]; [t.join() for t in th]
assert not errs, errs
L.load().jfs_release_staging()
print("OK")
'''


def test_staging_failure_is_per_block(gpu):
    env = dict(os.environ, JFS_STAGING_MAX_MB="64")
    r = subprocess.run([sys.executable, "-c", CHILD_NOMEM, ROOT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def test_caller_device_unchanged(gpu):
    """capi.hip never leaves the calling thread on another device (PyTorch's
    current device / stream read it)."""
    import torch
    ndev = torch.cuda.device_count()
    torch.cuda.set_device(0)
    lib = L.load()
    assert lib.jfs_device_count() >= 1
    lz = C.LZ4()
    s = gen_block("T", 5, 100000)
    d = bytearray(lz.CompressBound(len(s)))
    res = lz.CompressBatch([(d, s)] * max(2, ndev))
    assert all(e is None for _, e in res)
    assert torch.cuda.current_device() == 0
    if ndev >= 2:
        torch.cuda.set_device(1)
        res = lz.CompressBatch([(bytearray(len(d)), s)] * 8, device_mask=0b01)
        assert all(e is None for _, e in res)
        assert torch.cuda.current_device() == 1
        torch.cuda.set_device(0)


def test_device_mask_round_robin(gpu):
    """The batch ABI's device deal (capi.hip batch_common) with an explicit
    mask of every visible device: results identical to the default deal."""
    import torch
    ndev = torch.cuda.device_count()
    lz = C.LZ4()
    srcs = [gen_block("T", 300 + i, 50000 + 777 * i) for i in range(16)]
    mask = (1 << ndev) - 1
    a = [(bytearray(lz.CompressBound(len(s))), s) for s in srcs]
    b = [(bytearray(lz.CompressBound(len(s))), s) for s in srcs]
    ra, rb = lz.CompressBatch(a), lz.CompressBatch(b, device_mask=mask)
    assert ra == rb
    assert all(bytes(x[0][:n]) == bytes(y[0][:n]) for x, y, (n, _) in zip(a, b, ra))
    # a mask naming no visible device
    with pytest.raises(C.CompressError):
        lz.CompressBatch(a, device_mask=1 << 31)


def test_blocks_dealt_to_distinct_devices(gpu, oracle):
    """with two or more GPUs a batch's blocks are dealt
    round-robin over the devices in device_mask -- every selected device runs
    some of them (jfs_device_stats) and every output is the oracle's.  With
    one GPU the deal degenerates to that device, which is checked instead."""
    import torch
    ndev = torch.cuda.device_count()
    lib = L.load()
    lz = C.LZ4()
    srcs = [gen_block("TZR"[i % 3], 700 + i, 30000 + 4099 * i) for i in range(24)]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    lib.jfs_stats_reset()
    cp = [(bytearray(lz.CompressBound(len(s))), s) for s in srcs]
    res = lz.CompressBatch(cp)
    assert all(e is None and bytes(d[:n]) == c for (d, _), (n, e), c in zip(cp, res, comps))
    dp = [(bytearray(len(s)), c) for s, c in zip(srcs, comps)]
    res = lz.DecompressBatch(dp)
    assert all(e is None and bytes(d) == s for (d, _), (n, e), s in zip(dp, res, srcs))
    ds = (L.JfsDeviceStat * 64)()
    nd = lib.jfs_device_stats(ds, 64)
    used = {int(ds[i].device): int(ds[i].blocks) for i in range(nd) if ds[i].blocks}
    assert sum(used.values()) == 2 * len(srcs)
    if ndev >= 2 and nd >= 2:
        assert len(used) == min(nd, len(srcs)), used  # every device got blocks
        assert max(used.values()) - min(used.values()) <= 2 * 1 + 2, used  # round-robin: balanced
    else:
        assert len(used) == 1, used


def test_decompress_batch_disk_cache_checksums(gpu, oracle):
    """jfs_decompress_batch_csum: the disk-cache checksum of each decoded block
    (pkg/chunk/disk_cache.go:536-537 / disk_cache_file.go:139-152: big-endian
    CRC-32C per 32 KiB), computed on the GPU, equals the oracle's layout; LZ4
    and Zstd, ragged sizes, a corrupt block (no checksum, error), "none"."""
    from juicefs_amd import compress as C
    sizes = [1, 100, 32767, 32768, 32769, 65536 + 5, 1 << 20, 4 << 20]
    raws = [gen_block("TZR"[i % 3], 6100 + i, n) for i, n in enumerate(sizes)]
    for name in ("lz4", "zstd", "none"):
        c = C.NewCompressor(name)
        comps = []
        for r in raws:
            d = bytearray(c.CompressBound(len(r)))
            n, e = c.Compress(d, r)
            assert e is None
            comps.append(bytes(d[:n]))
        if name != "none":
            comps.append(comps[3][: len(comps[3]) // 2])  # truncated: fails, no checksum
        outs = [bytearray(len(r)) for r in raws] + ([bytearray(32769)] if name != "none" else [])
        res = c.DecompressBatchChecksum(list(zip(outs, comps)))
        for i, r in enumerate(raws):
            n, e, cs = res[i]
            assert e is None and n == len(r) and bytes(outs[i][:n]) == r, (name, len(r))
            assert cs == oracle.crc32c_segments(r), (name, len(r))
        if name != "none":
            n, e, cs = res[-1]
            assert e is not None and cs is None


def test_mixed_codec_batches(gpu, oracle):
    """jfs_{de,}compress_batch_mixed (SURVEY.md 8(d) config 4 shape): LZ4, Zstd
    and "none" blocks of 64 KiB - 4 MiB in one call; every compressed block is
    byte-identical to the oracle of its codec (liblz4 1.9.3 / libzstd 1.4.9
    level 1), every block round-trips, an unknown codec fails alone."""
    rng = np.random.default_rng(5)
    sizes = np.exp(rng.uniform(np.log(64 << 10), np.log(4 << 20), 24)).astype(np.int64)
    raws = [gen_block("TZR"[i % 3] if i % 4 else "T", 7100 + i, int(n)) for i, n in enumerate(sizes)]
    cds = [(C.LZ4(), C.ZStandard(), C.noOp())[i % 3] for i in range(len(raws))]
    ents = [(cd, bytearray(cd.CompressBound(len(r))), r) for cd, r in zip(cds, raws)]
    res = C.CompressBatchMixed(ents)
    comp = []
    for (cd, buf, r), (n, e) in zip(ents, res):
        assert e is None and n > 0, e
        got = bytes(buf[:n])
        if isinstance(cd, C.LZ4):
            assert got == oracle.lz4_compress(r)[1]
        elif isinstance(cd, C.ZStandard):
            assert got == oracle.zstd_compress_l1(r)
        else:
            assert got == r
        comp.append(got)
    outs = [(cd, bytearray(len(r)), c) for cd, r, c in zip(cds, raws, comp)]
    back = C.DecompressBatchMixed(outs)
    for (cd, buf, _), (n, e), r in zip(outs, back, raws):
        assert e is None and n == len(r) and bytes(buf) == r
    # an unknown codec id fails alone; its neighbours still decode
    lib = L.load()
    import ctypes
    nb = 3
    iov = (L.JfsIov * nb)()
    keep = []
    for i in range(nb):
        src = comp[i]
        dst = bytearray(len(raws[i]))
        keep.append((src, dst))
        iov[i].src = ctypes.cast(ctypes.c_char_p(src), ctypes.c_void_p)
        iov[i].src_len = len(src)
        iov[i].dst = ctypes.addressof((ctypes.c_char * len(dst)).from_buffer(dst))
        iov[i].dst_cap = len(dst)
    algos = (ctypes.c_int32 * nb)(cds[0].algo, 7, cds[2].algo)
    out = (ctypes.c_int64 * nb)()
    assert lib.jfs_decompress_batch_mixed(algos, nb, iov, out, 0) == 0
    assert out[0] == len(raws[0]) and out[1] == L.JFS_ERR_INVALID and out[2] == len(raws[2])
    assert bytes(keep[0][1]) == raws[0] and bytes(keep[2][1]) == raws[2]
