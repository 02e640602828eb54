"""GPU: the segment-parallel LZ4 encoder (lz4_encode.hip, segment mode) must
write exactly LZ4_compress_default's bytes -- the serial parse of
pkg/compress/compress.go:115-117 -- on every input: it cuts a block into
segments, re-parses each from the state the segment before it stopped in, and
uses the result only once a round changes nothing; blocks that do not settle
(or overflow a segment's sequence list) are encoded by the serial kernel.
Checked against the CPU oracle (oracle/lz4_oracle.c, pinned by liblz4 1.9.3
golden vectors) and against the serial GPU kernel, on text, zero, random and
mixed blocks whose content changes at the segment boundaries."""
import os
import random

import numpy as np
import pytest
import torch

from juicefs_amd import compress as C
from juicefs_amd import device as D
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu


def _encode_both(srcs, caps=None):
    """(segment-mode results, serial-kernel results) as lists of bytes / 0."""
    dev = torch.device("cuda:0")
    n = len(srcs)
    caps = caps or [D.lz4_bound(len(s)) for s in srcs]
    soff = np.cumsum([0] + [(len(s) + 255) // 256 * 256 for s in srcs])
    doff = np.cumsum([0] + [(c + 255) // 256 * 256 for c in caps])
    raw = torch.zeros(int(soff[-1]) + 256, dtype=torch.uint8)
    for i, s in enumerate(srcs):
        if s:
            raw[int(soff[i]):int(soff[i]) + len(s)] = torch.frombuffer(bytearray(s), dtype=torch.uint8)
    raw = raw.to(dev)
    outs = []
    for small in (True, False):
        comp = torch.zeros(int(doff[-1]) + 256, dtype=torch.uint8, device=dev)
        desc = D.make_desc(raw, soff[:-1], [len(s) for s in srcs], comp, doff[:-1], caps)
        ret = torch.zeros(n, dtype=torch.int32, device=dev)
        if small:
            D.lz4_compress_small(desc, ret, [len(s) for s in srcs])
        else:
            D.lz4_compress(desc, ret)
        torch.cuda.synchronize()
        r = ret.cpu().numpy()
        host = comp.cpu().numpy()
        outs.append([bytes(host[int(doff[i]):int(doff[i]) + int(r[i])]) if r[i] > 0 else int(r[i]) for i in range(n)])
    return outs


def _mixed(seed, n, pieces):
    """Text with zero runs and random runs placed across 64 KiB boundaries."""
    rng = random.Random(seed)
    b = bytearray(gen_block("T", seed, n))
    for _ in range(pieces):
        at = (rng.randrange(1, max(2, n >> 16)) << 16) + rng.randrange(-3000, 3000)
        ln = rng.choice([40, 300, 5000, 70000])
        at = max(0, min(at, n - ln))
        fill = bytes(ln) if rng.random() < 0.5 else gen_block("R", seed + at, ln)
        b[at:at + ln] = fill
    return bytes(b)


def test_eseg_matches_oracle_and_serial(gpu, oracle):
    D.lz4_eseg_counts(reset=True)
    srcs = [gen_block("T", 11, 4 << 20), gen_block("T", 12, (4 << 20) - 7), gen_block("T", 13, 1 << 20),
            gen_block("T", 14, 65547), gen_block("T", 15, 65546), gen_block("T", 16, 200001),
            gen_block("Z", 17, 4 << 20), gen_block("R", 18, 1 << 20), b"", gen_block("T", 19, 5),
            _mixed(20, 4 << 20, 12), _mixed(21, 3 << 20, 30), _mixed(22, 1 << 20, 6)]
    seg, ser = _encode_both(srcs)
    for i, s in enumerate(srcs):
        want = oracle.lz4_compress(s)[1]
        assert seg[i] == want, (i, len(s))
        assert ser[i] == want, (i, len(s))
    cnt = D.lz4_eseg_counts()
    # every text block of >= 65547 bytes settles (the random block is handed to
    # the serial kernel after its first segment finds no match)
    assert sum(v for k, v in cnt.items() if k > 0) >= 8, cnt


def test_eseg_limited_output(gpu, oracle):
    """dst_cap below the bound: the whole output or 0, like LZ4_compress_default."""
    src = gen_block("T", 31, 1 << 20)
    full = oracle.lz4_compress(src)[1]
    caps = [len(full), len(full) - 1, len(full) + 1, 1000, D.lz4_bound(len(src))]
    seg, ser = _encode_both([src] * len(caps), caps)
    for c, a, b in zip(caps, seg, ser):
        want = full if c >= len(full) else 0
        assert a == want and b == want, c


def test_eseg_dense_sequences_overflow_to_serial(gpu, oracle):
    """4-byte words from a small vocabulary: a sequence every ~5 bytes, more
    than a segment's sequence list holds -> the serial kernel takes the block,
    same bytes."""
    rng = random.Random(5)
    words = [bytes(rng.randrange(256) for _ in range(4)) for _ in range(64)]
    src = b"".join(rng.choice(words) for _ in range((2 << 20) // 4))
    D.lz4_eseg_counts(reset=True)
    seg, ser = _encode_both([src])
    want = oracle.lz4_compress(src)[1]
    assert seg[0] == want and ser[0] == want
    assert D.lz4_eseg_counts().get(0, 0) == 1


def test_eseg_many_blocks_and_batch_api(gpu, oracle):
    """A 64-block batch through the host batch ABI (segment path below
    JFS_LZ4E_SEG_MAX blocks), ragged sizes."""
    rng = random.Random(9)
    srcs = [gen_block("TTTZ"[i % 4], 400 + i, rng.randrange(60000, 1 << 20)) for i in range(64)]
    c = C.LZ4()
    pairs = [(bytearray(c.CompressBound(len(s))), s) for s in srcs]
    res = c.CompressBatch(pairs)
    for (d, s), (n, err) in zip(pairs, res):
        assert err is None and bytes(d[:n]) == oracle.lz4_compress(s)[1]


def _encode_device(srcs, caps=None):
    """jfs_lz4_compress_device results (bytes / 0): the large-batch path, whose
    byU32 blocks take the compact-table kernel (lz4_encode.hip, Smem<true>)."""
    dev = torch.device("cuda:0")
    caps = caps or [D.lz4_bound(len(s)) for s in srcs]
    soff = np.cumsum([0] + [(len(s) + 255) // 256 * 256 for s in srcs])
    doff = np.cumsum([0] + [(c + 255) // 256 * 256 for c in caps])
    raw = torch.zeros(int(soff[-1]) + 256, dtype=torch.uint8)
    for i, s in enumerate(srcs):
        if s:
            raw[int(soff[i]):int(soff[i]) + len(s)] = torch.frombuffer(bytearray(s), dtype=torch.uint8)
    raw = raw.to(dev)
    comp = torch.zeros(int(doff[-1]) + 256, dtype=torch.uint8, device=dev)
    desc = D.make_desc(raw, soff[:-1], [len(s) for s in srcs], comp, doff[:-1], caps)
    ret = torch.zeros(len(srcs), dtype=torch.int32, device=dev)
    D.lz4_compress(desc, ret)
    torch.cuda.synchronize()
    r = ret.cpu().numpy()
    host = comp.cpu().numpy()
    return [bytes(host[int(doff[i]):int(doff[i]) + int(r[i])]) if r[i] > 0 else int(r[i]) for i in range(len(srcs))]


def test_compact_table_kernel_exact(gpu, oracle):
    """The large-batch kernel keeps 17-bit position entries (u16 + a bit plane)
    refreshed every 32 KiB, a 512-byte output ring and a 1 KiB source window
    (16 blocks per CU); its output must stay LZ4_compress_default's: matches at
    exactly 65,535 / 65,536 bytes back, entries going stale across long
    matches and long skip-schedule jumps, a long literal run right before a
    long match (the ring's room), the byU16/byU32 switch at 65,547."""
    srcs = []
    r = gen_block("R", 61, 65535)
    srcs.append(r + r + r[:3000])                       # distance 65,535: matches allowed
    r = gen_block("R", 62, 65536)
    srcs.append(r + r + r[:3000])                       # distance 65,536: too far
    r = gen_block("R", 63, 65537)
    srcs.append(r + gen_block("T", 64, 40000) + r)      # stale entries, then text
    for lit in (430, 470, 500, 1990, 2040):
        b = bytearray(gen_block("T", 40 + lit, 300000))
        b[100000:100000 + lit] = gen_block("R", lit, lit)
        b[100000 + lit:100000 + lit + 5000] = bytes(5000)
        srcs.append(bytes(b))
    for i, z in enumerate((70000, 140000, 300000)):    # long matches jump past refreshes
        srcs.append(gen_block("T", 70 + i, 200000) + bytes(z) + gen_block("T", 70 + i, 150000))
    srcs += [_mixed(80 + i, (4 << 20) - 13 * i, 20) for i in range(3)]
    srcs += [gen_block("R", 90, 1 << 20), gen_block("Z", 91, 1 << 20), gen_block("T", 92, 65547),
             gen_block("T", 93, 65546), gen_block("T", 94, 3 * 131072 + 5), gen_block("T", 95, 16 << 20),
             gen_block("R", 96, 300000) + gen_block("T", 96, 300000)]
    os.environ["JFS_LZ4E_COMPACT"] = "1"  # small batches take the check-bit kernel by default
    try:
        got = _encode_device(srcs)
    finally:
        del os.environ["JFS_LZ4E_COMPACT"]
    for i, s in enumerate(srcs):
        assert got[i] == oracle.lz4_compress(s)[1], (i, len(s))


def test_compact_table_kernel_golden_and_limited_output(gpu, golden):
    """liblz4 1.9.3's own bytes (golden sha256) and its limited-output results
    (0 when the block does not fit in dst_cap) through the compact kernel."""
    import hashlib
    cache, srcs, caps, want = {}, [], [], []
    for b in golden["lz4"]["blocks"]:
        srcs.append(gen_block(b["cls"], b["seed"], b["size"]))
        caps.append(D.lz4_bound(b["size"]))
        want.append(("sha", b["csize"], b["comp_sha"]))
    for e in golden["lz4"]["limited"]:
        key = (e["cls"], e["seed"], e["size"])
        if key not in cache:
            cache[key] = gen_block(*key)
        srcs.append(cache[key])
        caps.append(e["cap"])
        want.append(("ret", e["ret"], None))
    os.environ["JFS_LZ4E_COMPACT"] = "1"
    try:
        got = _encode_device(srcs, caps)
    finally:
        del os.environ["JFS_LZ4E_COMPACT"]
    for i, (kind, n, sh) in enumerate(want):
        if kind == "sha":
            assert isinstance(got[i], bytes) and len(got[i]) == n and hashlib.sha256(got[i]).hexdigest() == sh, i
        elif n == 0:
            assert got[i] == 0, (i, caps[i])
        else:
            assert isinstance(got[i], bytes) and len(got[i]) == n, (i, caps[i])
