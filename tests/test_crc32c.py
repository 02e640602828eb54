"""CRC-32C: the oracle pinned on CPU by published vectors,
the HIP kernel (jfs_crc32c_device) bit-exact against the oracle on GPU.

Reference: pkg/object/checksum.go:30-45 (crc32.Update(0, crc32c, data)) and
pkg/chunk/disk_cache_file.go:139-152 (big-endian CRC-32C per 32 KiB piece)."""
import random

import numpy as np
import pytest

from juicefs_amd.blockgen import gen_block


def crc32c_bitwise(data: bytes, crc: int = 0) -> int:
    """Go hash/crc32 Castagnoli, bit at a time (independent of the oracle)."""
    c = crc ^ 0xFFFFFFFF
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ 0x82F63B78 if c & 1 else c >> 1
    return c ^ 0xFFFFFFFF


def test_oracle_check_value_and_rfc3720_vectors(oracle):
    assert oracle.crc32c(b"123456789") == 0xE3069283  # the CRC catalogue's check value
    # RFC 3720 appendix B.4 (iSCSI CRC32C examples; CRC bytes listed LSB first)
    assert oracle.crc32c(bytes(32)) == 0x8A9136AA
    assert oracle.crc32c(b"\xff" * 32) == 0x62A8AB43
    assert oracle.crc32c(bytes(range(32))) == 0x46DD794E
    assert oracle.crc32c(bytes(range(31, -1, -1))) == 0x113FDB5C
    assert oracle.crc32c(b"") == 0


def test_oracle_vs_bitwise_and_update_chaining(oracle):
    rng = random.Random(3)
    for n in (1, 3, 15, 16, 17, 255, 1000, 4099):
        d = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.crc32c(d) == crc32c_bitwise(d)
        k = rng.randrange(n + 1)  # crc32.Update chaining (checksumReader.Read)
        assert oracle.crc32c(d[k:], oracle.crc32c(d[:k])) == oracle.crc32c(d)


def test_oracle_segments_layout(oracle):
    d = gen_block("T", 9, 100000)
    s = oracle.crc32c_segments(d)
    assert len(s) == 4 * ((len(d) - 1) // 32768 + 1)
    for k in range(len(s) // 4):
        assert int.from_bytes(s[4 * k:4 * k + 4], "big") == crc32c_bitwise(d[32768 * k:32768 * (k + 1)])
    assert oracle.crc32c_segments(b"") == bytes(4)  # Go: ((0-1)/csBlock+1)*4 = 4 zero bytes


def _run_gpu(gpu, datas, seg, src_mis=0, extra_cap=0):
    import torch
    from juicefs_amd import device as D
    so, off = [], 0
    for i, d in enumerate(datas):
        m = (src_mis * (i + 1)) % 16 if src_mis else 0
        so.append(off + m)
        off = (off + m + len(d) + 64 + 15) & ~15
    host = np.zeros(off + 64, dtype=np.uint8)
    for d, o in zip(datas, so):
        host[o:o + len(d)] = np.frombuffer(d, dtype=np.uint8)
    src = torch.from_numpy(host).to(gpu)
    words = [((len(d) - 1) // seg + 1 if len(d) else 1) if seg else 0 for d in datas]
    caps = [4 * w + extra_cap for w in words]
    doffs = np.cumsum([0] + [c + 16 for c in caps[:-1]]).tolist()
    dst = torch.full((sum(c + 16 for c in caps) + 16,), 0xEE, dtype=torch.uint8, device=gpu)
    desc = D.make_desc(src, so, [len(d) for d in datas], dst, doffs, caps)
    crc = torch.zeros(len(datas), dtype=torch.int32, device=gpu)
    ret = torch.zeros(len(datas), dtype=torch.int32, device=gpu)
    D.crc32c(desc, crc, ret, seg_bytes=seg)
    torch.cuda.synchronize()
    c = [x & 0xFFFFFFFF for x in crc.cpu().tolist()]
    dh = dst.cpu().numpy()
    segs = [dh[o:o + 4 * w].tobytes() for o, w in zip(doffs, words)]
    return c, ret.cpu().tolist(), segs


@pytest.mark.gpu
def test_crc32c_gpu_vs_oracle(gpu, oracle, golden):
    rng = random.Random(11)
    datas = [b"123456789", bytes(32), b"", b"\x01"]
    for b in golden["lz4"]["blocks"][:24]:  # the golden block set (all classes, 1 B .. 4 MiB)
        datas.append(gen_block(b["cls"], b["seed"], min(b["size"], 1 << 20)))
    for n in (4095, 4096, 4097, 32767, 32768, 32769, 65536 + 7, 300001):
        datas.append(bytes(rng.randrange(256) for _ in range(n)))
    for mis in (0, 3):
        c, r, segs = _run_gpu(gpu, datas, 32 << 10, src_mis=mis)
        for d, ci, ri, si in zip(datas, c, r, segs):
            assert ci == oracle.crc32c(d), (len(d), mis)
            assert si == oracle.crc32c_segments(d), (len(d), mis)
            assert ri == len(si)
    assert _run_gpu(gpu, [b"123456789"], 0)[0] == [0xE3069283]


@pytest.mark.gpu
def test_crc32c_gpu_4mib_blocks_and_segment_sizes(gpu, oracle):
    import torch
    from juicefs_amd import device as D
    n, U = 64, 4 << 20
    raw = torch.empty(n * U, dtype=torch.uint8, device=gpu)
    D.gen_blocks(raw, n, U, "T", 555)
    host = raw.cpu().numpy()
    datas = [host[i * U:(i + 1) * U].tobytes() for i in (0, 1, 63)]
    for seg in (4096, 32 << 10, 1 << 20):
        c, r, segs = _run_gpu(gpu, datas, seg)
        for d, ci, si in zip(datas, c, segs):
            assert ci == oracle.crc32c(d)
            assert si == oracle.crc32c_segments(d, seg)
    # whole batch in place: every block's CRC vs the oracle
    desc = D.make_desc(raw, [i * U for i in range(n)], [U] * n, raw, [0] * n, [0] * n)
    crc = torch.zeros(n, dtype=torch.int32, device=gpu)
    D.crc32c(desc, crc)
    torch.cuda.synchronize()
    got = [x & 0xFFFFFFFF for x in crc.cpu().tolist()]
    for i in range(n):
        assert got[i] == oracle.crc32c(host[i * U:(i + 1) * U].tobytes()), i


@pytest.mark.gpu
def test_crc32c_bad_descriptor(gpu):
    # dst too small for the segment sums -> ret -1, nothing written past cap
    c, r, segs = _run_gpu(gpu, [bytes(100000)], 32 << 10, extra_cap=-4)
    assert r == [-1]


def test_none_codec_batch_checksum_on_host(oracle):
    """jfs_compress_batch_crc with the "none" codec: the payload is the block
    itself (noOp, compress.go:55-68), summed on the host; no GPU needed."""
    from juicefs_amd import compress as C
    c = C.NewCompressor("none")
    srcs = [b"", b"a", gen_block("T", 3, 70000), gen_block("R", 4, 4097)]
    pairs = [(bytearray(len(s)), s) for s in srcs] + [(bytearray(1), b"toolong")]
    res = c.CompressBatchChecksum(pairs)
    for (d, s), (n, e, crc) in zip(pairs[:-1], res[:-1]):
        assert e is None and n == len(s) and crc == oracle.crc32c(s)
    assert res[-1][1] is not None and res[-1][2] == 0
