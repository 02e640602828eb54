"""GPU parity: the HIP Zstd decoder (through the C ABI) vs the CPU oracle
(oracle/zstd_oracle.c, pinned to libzstd 1.4.9 fixtures).  Bar: identical
decoded bytes and identical result codes (size / -1 corrupt / -2 dst too
small / -3 source size wrong) on every fixture and corpus case."""
import hashlib
import os

import numpy as np
import pytest
import torch

from juicefs_amd import compress as C
from juicefs_amd import device as D

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def frames_bin(golden):
    with open(os.path.join(GOLD, golden["zstd"]["bin"]), "rb") as f:
        return f.read()


def run_device(srcs, caps, dev, src_mis=0, dst_mis=0):
    """Decode each src into its own dst (cap bytes) on the GPU; returns
    (rets, outputs[:ret])."""
    n = len(srcs)
    so, do, off, doff = [], [], 0, 0
    for i, s in enumerate(srcs):
        m = (src_mis + 7 * i) % 16 if src_mis else 0
        so.append(off + m)
        off += m + len(s) + 64
        off = (off + 15) & ~15
        dm = (dst_mis + 5 * i) % 16 if dst_mis else 0
        do.append(doff + dm)
        doff += dm + caps[i] + 64
        doff = (doff + 15) & ~15
    host = np.zeros(off + 64, dtype=np.uint8)
    for s, o in zip(srcs, so):
        host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
    src_t = torch.from_numpy(host).to(dev)
    dst_t = torch.full((doff + 64,), 0xAB, dtype=torch.uint8, device=dev)
    desc = D.make_desc(src_t, so, [len(s) for s in srcs], dst_t, do, caps)
    ret = torch.zeros(n, dtype=torch.int32, device=dev)
    D.zstd_decompress_sync(desc, ret)
    r = ret.cpu().tolist()
    dh = dst_t.cpu().numpy()
    outs = [dh[o:o + max(x, 0)].tobytes() for o, x in zip(do, r)]
    # nothing written at or past cap
    for o, c in zip(do, caps):
        assert (dh[o + c:o + c + 16] == 0xAB).all()
    return r, outs


def test_zstd_frames_vs_golden(gpu, golden, frames_bin):
    ents = golden["zstd"]["frames"] + golden["zstd"]["special"]
    srcs = [frames_bin[f["off"]:f["off"] + f["csize"]] for f in ents]
    caps = [f["size"] for f in ents]
    r, outs = run_device(srcs, caps, gpu)
    for f, x, o in zip(ents, r, outs):
        assert x == f["size"] and sha(o) == f["src_sha"], (f.get("name"), f["cls"], f.get("level"), f["size"], x)


def test_zstd_frames_one_wave_path(gpu, golden, frames_bin):
    """The golden frames in one batch larger than JFS_ZSTD_SPLIT_MAX (128):
    the one-wave-per-input kernels (zlit / zseqa / zseqb / zexec) decode them
    (smaller batches take zstd_split.inc, tests/test_zstd_split_gpu.py)."""
    ents = golden["zstd"]["frames"] + golden["zstd"]["special"]
    srcs = [frames_bin[f["off"]:f["off"] + f["csize"]] for f in ents]
    caps = [f["size"] for f in ents]
    k = 129 // len(srcs) + 1
    r, outs = run_device(srcs * k, caps * k, gpu, src_mis=2, dst_mis=5)
    assert len(r) > 128
    for f, x, o in zip(ents * k, r, outs):
        assert x == f["size"] and sha(o) == f["src_sha"], (f.get("name"), f["cls"], f.get("level"), f["size"], x)


def test_zstd_frames_unaligned_and_short(gpu, golden, frames_bin, oracle):
    ents = [f for f in golden["zstd"]["frames"] if f["size"] <= 300000]
    srcs = [frames_bin[f["off"]:f["off"] + f["csize"]] for f in ents]
    caps = [f["size"] for f in ents]
    r, outs = run_device(srcs, caps, gpu, src_mis=3, dst_mis=9)
    for f, x, o in zip(ents, r, outs):
        assert x == f["size"] and sha(o) == f["src_sha"]
    # one byte short -> dstSize_tooSmall, exactly like the oracle
    caps2 = [max(c - 1, 0) for c in caps]
    r2, _ = run_device(srcs, caps2, gpu)
    for s, c, x in zip(srcs, caps2, r2):
        assert x == oracle.zstd_decompress(s, c)[0]


def test_zstd_accept_and_corpus_vs_oracle(gpu, golden, oracle):
    cases = golden["zstd"]["accept"] + golden["zstd"]["corpus"]
    srcs = [bytes.fromhex(a["src"]) for a in cases]
    caps = [a["cap"] for a in cases]
    r, outs = run_device(srcs, caps, gpu, src_mis=1, dst_mis=2)
    bad = []
    for s, c, x, o in zip(srcs, caps, r, outs):
        want, wo = oracle.zstd_decompress(s, c)
        if x != want or (x >= 0 and o != wo):
            bad.append((s.hex(), c, want, x))
    assert not bad, bad[:5]


def test_zstd_baseline_block_batch(gpu, golden, frames_bin, oracle):
    """configs[3] shape: 4 MiB level-3 frames, many per launch."""
    f = [e for e in golden["zstd"]["frames"] if e["size"] == 4 << 20][0]
    c = frames_bin[f["off"]:f["off"] + f["csize"]]
    n, ref = oracle.zstd_decompress(c, f["size"])
    assert n == f["size"]
    nb = 96
    r, outs = run_device([c] * nb, [f["size"]] * nb, gpu, dst_mis=0)
    assert r == [f["size"]] * nb
    assert all(o == ref for o in outs)


def test_zstandard_decompress_contract(gpu, golden):
    """compress.go:94-103 through DataDog v1.5.6 semantics (size hint)."""
    z = C.ZStandard()
    kat = {bytes.fromhex(k["src"]): bytes.fromhex(k["comp_l1"]) for k in golden["zstd"]["kat"]}
    frame = kat[b"Zstd"]
    out = bytearray(4)
    n, err = z.Decompress(out, frame)
    assert err is None and n == 4 and bytes(out) == b"Zstd"
    n, err = z.Decompress(bytearray(1), frame)          # cap < hint -> "buffer too short"
    assert err is not None
    n, err = z.Decompress(bytearray(0), kat[b""])       # empty content -> (0, nil)
    assert err is None and n == 0
    n, err = z.Decompress(bytearray(100), b"")          # ErrEmptySlice
    assert err is not None
    big = kat[b"hello world" * 8]
    out = bytearray(200)
    n, err = z.Decompress(out, big)
    assert err is None and bytes(out[:n]) == b"hello world" * 8
    n, err = z.Decompress(bytearray(100), big[:-1])     # truncated frame
    assert err is not None


def test_zstd_device_call_is_async_and_stream_safe(gpu, golden, frames_bin, oracle):
    """jfs_zstd_decompress_device enqueues the decode on the caller's stream;
    after zscan/zplan it waits once for the planned scratch sizes and grows
    the device scratch itself, so the result is always final (never a -4
    "resubmit", jfs_gpucodec.h); two streams sharing the device scratch stay
    correct."""
    import torch
    f = [e for e in golden["zstd"]["frames"] if e["size"] == 4 << 20][0]
    c = frames_bin[f["off"]:f["off"] + f["csize"]]
    n, ref = oracle.zstd_decompress(c, f["size"])
    nb = 48
    host = np.zeros(nb * (len(c) + 256), dtype=np.uint8)
    slot = len(c) + 256
    for i in range(nb):
        host[i * slot:i * slot + len(c)] = np.frombuffer(c, dtype=np.uint8)
    src = torch.from_numpy(host).to(gpu)
    outs, descs, rets = [], [], []
    for k in range(2):
        out = torch.zeros(nb * n, dtype=torch.uint8, device=gpu)
        outs.append(out)
        descs.append(D.make_desc(src, [i * slot for i in range(nb)], [len(c)] * nb, out, [i * n for i in range(nb)],
                                 [n] * nb))
        rets.append(torch.zeros(nb, dtype=torch.int32, device=gpu))
    D.zstd_decompress_sync(descs[0], rets[0])  # sizes the scratch
    assert (rets[0] == n).all()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    for k, st in enumerate((s1, s2)):
        outs[k].zero_()
        rets[k].zero_()
    torch.cuda.synchronize()
    for _ in range(3):  # interleaved launches on two streams, same scratch
        for k, st in enumerate((s1, s2)):
            D.zstd_decompress(descs[k], rets[k], st)
    torch.cuda.synchronize()
    for k in range(2):
        assert (rets[k] == n).all()
        assert all(outs[k][i * n:(i + 1) * n].cpu().numpy().tobytes() == ref for i in (0, nb // 2, nb - 1))


def test_zstd_host_batch_chunks(gpu, golden, frames_bin):
    """Zstd through the batch ABI in many pipeline chunks (host-planned
    scratch per staging slot, no device round trip per chunk)."""
    import subprocess
    import sys
    child = r'''
import sys, hashlib
sys.path.insert(0, sys.argv[1])
from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block
z = C.ZStandard()
srcs = [gen_block("TZR"[i % 3], 300 + i, (1 << 20) + 4097 * i) for i in range(40)]
pairs = [(bytearray(z.CompressBound(len(s))), s) for s in srcs]
res = z.CompressBatch(pairs)
frames = [bytes(d[:n]) for (d, _), (n, e) in zip(pairs, res)]
assert all(e is None for _, e in res)
outs = [bytearray(len(s)) for s in srcs]
back = z.DecompressBatch(list(zip(outs, frames)))
assert all(e is None and n == len(s) and bytes(o) == s for s, o, (n, e) in zip(srcs, outs, back))
print("OK")
'''
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, JFS_HOST_CHUNK_MB="24")
    r = subprocess.run([sys.executable, "-c", child, root], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-2000:])


def _block_spans(fr):
    """(block start, block type, literal section type, literal section end)
    for each block of a single-segment-or-windowed frame."""
    p = 4
    fhd = fr[p]; p += 1
    ss, did, fcs = (fhd >> 5) & 1, fhd & 3, fhd >> 6
    p += (0 if ss else 1) + [0, 1, 2, 4][did] + [1 if ss else 0, 2, 4, 8][fcs]
    out, last = [], 0
    while not last:
        h = int.from_bytes(fr[p:p + 3], "little"); p += 3
        last, bt, bs = h & 1, (h >> 1) & 3, h >> 3
        q = p
        p += bs if bt != 1 else 1
        if bt != 2:
            out.append((q, bt, -1, q))
            continue
        b0 = fr[q]; lt, sf = b0 & 3, (b0 >> 2) & 3
        if lt >= 2:
            hs = 3 if sf <= 1 else 4 if sf == 2 else 5
            v = int.from_bytes(fr[q:q + hs], "little")
            cs = (v >> 14) & 0x3FF if hs == 3 else (v >> 18) if hs == 4 else (v >> 22)
            out.append((q, bt, lt, q + hs + cs))
        else:
            out.append((q, bt, lt, q))
    return out


def test_zstd_literal_pairs_corrupt_vs_oracle(gpu, golden, frames_bin, oracle):
    """Literal sections decoded two blocks at a time (JFS_ZLIT_PAIR): a damaged
    Huffman table description or stream in either block of a pair (and in a
    treeless block) gives the oracle's result, through the one-wave path."""
    f = [e for e in golden["zstd"]["frames"] if e["size"] == 4 << 20 and e["level"] == 3][0]
    fr = frames_bin[f["off"]:f["off"] + f["csize"]]
    spans = _block_spans(fr)
    huf = [s for s in spans if s[2] == 2]
    tl = [s for s in spans if s[2] == 3]
    assert len(huf) >= 4
    variants = []
    for q, _, lt, lend in huf[:4] + tl[:2]:
        hs = 3 if ((fr[q] >> 2) & 3) <= 1 else 4 if ((fr[q] >> 2) & 3) == 2 else 5
        for pos, x in ((q + hs + 1, 0x5A), ((q + lend) // 2, 0xFF), (lend - 2, 0x11)):
            b = bytearray(fr)
            b[pos] ^= x
            variants.append(bytes(b))
    k = 129 // len(variants) + 1
    srcs = variants * k
    caps = [f["size"]] * len(srcs)
    r, outs = run_device(srcs, caps, gpu)
    assert len(r) > 128
    want = [oracle.zstd_decompress(v, f["size"]) for v in variants]
    for i, (x, o) in enumerate(zip(r, outs)):
        wr, wo = want[i % len(variants)]
        assert x == wr, (i % len(variants), wr, x)
        if x >= 0:
            assert o == wo


def _bits_le(fields):
    """LSB-first bit packing of (value, nbits) fields into bytes."""
    acc, n, out = 0, 0, bytearray()
    for v, nb in fields:
        acc |= (v & ((1 << nb) - 1)) << n
        n += nb
    while n > 0:
        out.append(acc & 0xFF)
        acc >>= 8
        n -= 8
    return bytes(out)


def _frame_weight_symbol(sym_hi, regen=100):
    """One-block frame whose literals are Huffman-compressed with FSE-coded
    weights, the weights' table description (RFC 8878 4.1.1, accuracy log 5)
    counting symbol 0 once and symbol `sym_hi` 31 times: every decoded weight
    is sym_hi, a corrupt description (symbols >= 64 must take the
    serial table build, like libzstd and the oracle)."""
    zeros = sym_hi - 2  # zero-count symbols after symbol 1's zero (repeat flags)
    f = [(0, 4), (2, 5), (1, 5)]  # AL - 5; symbol 0: count 1 (v=2); symbol 1: count 0 (v=1)
    while zeros >= 3:
        f.append((3, 2))
        zeros -= 3
    f.append((zeros, 2))
    f.append((63, 6))  # symbol sym_hi: count 31 (v=32 >= max=31: 6 bits, x - max = 32)
    ncount = _bits_le(f)
    wstream = bytes([0x5A, 0xA5, 0x33, 0x81])
    hb = len(ncount) + len(wstream)
    huf = bytes([hb]) + ncount + wstream
    stream = bytes([0x3C, 0x99, 0x17, 0x80])
    csize = len(huf) + len(stream)
    # literals header, Compressed, size format 00 (one stream, 10-bit sizes)
    h = 2 | (0 << 2) | ((regen & 0xF) << 4) | ((regen >> 4) << 8) | (csize << 14)
    lit = bytes([h & 0xFF, (h >> 8) & 0xFF, (h >> 16) & 0xFF]) + huf + stream
    body = lit + bytes([0])  # no sequences
    bh = 1 | (2 << 1) | (len(body) << 3)
    blk = bytes([bh & 0xFF, (bh >> 8) & 0xFF, (bh >> 16) & 0xFF]) + body
    return bytes([0x28, 0xB5, 0x2F, 0xFD, 0x20, regen]) + blk


@pytest.mark.parametrize("nb", [3, 140])
def test_zstd_huffman_weight_symbol_ge64_vs_oracle(gpu, oracle, nb):
    """A Huffman weight description that counts FSE symbols 64 / 100 / 255
    (and 40 / 63, the lane-parallel builder's range) decodes to the oracle's
    result on the small-batch (3 inputs) and the large-batch (140) paths."""
    frames = [_frame_weight_symbol(s) for s in (40, 63, 64, 100, 255)]
    want = [oracle.zstd_decompress(f, 100) for f in frames]
    assert all(w[0] < 0 for w in want[2:]), want  # the oracle rejects them
    srcs = [frames[i % len(frames)] for i in range(nb)]
    r, outs = run_device(srcs, [100] * nb, gpu)
    for i, (x, o) in enumerate(zip(r, outs)):
        wr, wo = want[i % len(frames)]
        assert x == wr, (i % len(frames), wr, x)
        if x >= 0:
            assert o == wo
