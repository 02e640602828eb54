"""GPU parity: the HIP LZ4 kernels (through the C ABI) vs the CPU oracle and the
liblz4 1.9.3 golden vectors.  Bar: bit-exact bytes and exact return values."""
import hashlib
import random

import numpy as np
import pytest

from juicefs_amd import compress as C
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.mark.parametrize("name", ["lz4", "none", "zstd"])
def test_compressor_contract(gpu, name):
    """compress_test.go:25-64 (testCompress), replayed verbatim for every
    codec of compress_test.go:66-76 (TestUncompressed, TestZstd, TestLZ4)."""
    for name in (name,):
        c = C.NewCompressor(name)
        src0 = c.Name().encode()
        for src in (src0, b""):
            if len(src) > 1:
                _, err = c.Compress(bytearray(1), src)
                assert err is not None, "expect short buffer error"
            dst = bytearray(c.CompressBound(len(src)))
            n, err = c.Compress(dst, src)
            assert err is None, err
            if len(src) > 1:
                _, err = c.Decompress(bytearray(1), bytes(dst[:n]))
                assert err is not None, "expect short buffer error"
            src2 = bytearray(len(src))
            n2, err = c.Decompress(src2, bytes(dst[:n]))
            assert err is None, err
            assert bytes(src2[:n2]) == src
        if c.CompressBound(0) > 0:
            n, err = c.Decompress(bytearray(100), src0[:0])
            assert err is not None and n <= 0


def test_lz4_kats_on_gpu(gpu, golden):
    c = C.LZ4()
    for k in golden["lz4"]["kat"]:
        src = bytes.fromhex(k["src"])
        dst = bytearray(k["bound"])
        n, err = c.Compress(dst, src)
        assert err is None and bytes(dst[:n]).hex() == k["comp"]
        out = bytearray(len(src))
        if n:
            m, err = c.Decompress(out, bytes(dst[:n]))
            assert err is None and m == len(src) and bytes(out) == src


BLOCK_CASES = [(cls, n) for cls in "TZR" for n in (1, 12, 13, 100, 4096, 65535, 65547, 131072, 1 << 20)] + [
    ("T", 4 << 20), ("Z", 4 << 20), ("R", 4 << 20)]


def test_lz4_decode_blocks_vs_oracle(gpu, oracle):
    c = C.LZ4()
    pairs, want = [], []
    for i, (cls, n) in enumerate(BLOCK_CASES):
        src = gen_block(cls, 900 + i, n)
        _, comp = oracle.lz4_compress(src)
        for cap in (n, n + 77):
            pairs.append((bytearray(cap), comp))
            want.append((n, src))
        if n > 1:  # short destination: exact negative value from the oracle
            r, _ = oracle.lz4_decompress(comp, n - 1)
            pairs.append((bytearray(n - 1), comp))
            want.append((r, None))
    res = c.DecompressBatch(pairs)
    for (dst, comp), (n_exp, src), (n, err) in zip(pairs, want, res):
        if n_exp >= 0:
            assert err is None and n == n_exp
            assert bytes(dst[:n]) == src
        else:
            assert err is not None and n == n_exp


def test_lz4_decode_corpus_exact(gpu, golden):
    """Every case of the liblz4 1.9.3 acceptance corpus: same return value
    (success size or negative error position), same bytes on success."""
    c = C.LZ4()
    cases = golden["lz4"]["decode_corpus"]
    pairs = [(bytearray(max(e["cap"], 0)), bytes.fromhex(e["src"])) for e in cases]
    res = c.DecompressBatch(pairs)
    bad = []
    for e, (dst, _), (n, err) in zip(cases, pairs, res):
        if e["ret"] >= 0:
            if not (err is None and n == e["ret"] and sha(bytes(dst[:n])) == e["out_sha"]):
                bad.append((e, n))
        else:
            if not (err is not None and n == e["ret"]):
                bad.append((e, n))
    assert not bad, f"{len(bad)} mismatches, first: {bad[:3]}"


def test_lz4_encode_golden(gpu, golden):
    """Byte-identical LZ4_compress_default output (sha256 of liblz4 1.9.3 output),
    including 4 MiB text blocks and the byU16/byU32 table switch at 65547."""
    c = C.LZ4()
    pairs, ents = [], []
    for b in golden["lz4"]["blocks"]:
        src = gen_block(b["cls"], b["seed"], b["size"])
        pairs.append((bytearray(c.CompressBound(len(src))), src))
        ents.append(b)
    res = c.CompressBatch(pairs)
    for (dst, _), b, (n, err) in zip(pairs, ents, res):
        assert err is None, b
        assert n == b["csize"] and sha(bytes(dst[:n])) == b["comp_sha"], (b["cls"], b["size"], b["seed"])


def test_lz4_encode_limited_output(gpu, golden):
    c = C.LZ4()
    cache, pairs, ents = {}, [], []
    for e in golden["lz4"]["limited"]:
        key = (e["cls"], e["seed"], e["size"])
        if key not in cache:
            cache[key] = gen_block(*key)
        pairs.append((bytearray(e["cap"]), cache[key]))
        ents.append(e)
    res = c.CompressBatch(pairs)
    for e, (n, err) in zip(ents, res):
        if e["ret"] == 0:
            assert err is not None
        else:
            assert err is None and n == e["ret"]


def test_lz4_encode_vs_oracle_random_sizes(gpu, oracle):
    rng = random.Random(7)
    c = C.LZ4()
    pairs, srcs = [], []
    for i in range(48):
        n = rng.choice([rng.randrange(0, 300), rng.randrange(300, 70000), rng.randrange(70000, 600000)])
        cls = rng.choice("TTTRZ")
        src = gen_block(cls, 5000 + i, n)
        if rng.random() < 0.3 and n > 100:  # mixed content
            k = rng.randrange(n)
            src = src[:k] + gen_block("R", i, min(5000, n - k)) + src[k + min(5000, n - k):]
        srcs.append(src)
        pairs.append((bytearray(c.CompressBound(n)), src))
    res = c.CompressBatch(pairs)
    for src, (dst, _), (n, err) in zip(srcs, pairs, res):
        m, ref = oracle.lz4_compress(src)
        assert err is None and n == m and bytes(dst[:n]) == ref


def test_lz4_single_block_calls_concurrent(gpu, oracle):
    """One call per block from many threads (pkg/chunk's 200 concurrent
    downloads); the coalescer batches them."""
    import threading
    c = C.LZ4()
    srcs = [gen_block("T", 70 + i, 65536 + 1000 * i) for i in range(32)]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    errs = []

    def work(i):
        out = bytearray(len(srcs[i]))
        n, err = c.Decompress(out, comps[i])
        if err is not None or n != len(srcs[i]) or bytes(out) != srcs[i]:
            errs.append(i)
        dst = bytearray(c.CompressBound(len(srcs[i])))
        n, err = c.Compress(dst, srcs[i])
        if err is not None or bytes(dst[:n]) != comps[i]:
            errs.append(100 + i)

    th = [threading.Thread(target=work, args=(i,)) for i in range(32)]
    [t.start() for t in th]
    [t.join() for t in th]
    assert not errs


def test_lz4_device_resident_roundtrip(gpu, oracle):
    """HBM-resident batch (the bench path): generate -> GPU compress -> GPU
    decompress; compressed bytes checked against the oracle on a sample."""
    import torch
    from juicefs_amd import device as D
    b = D.Lz4Batch(24, 4 << 20, "T", seed_base=11)
    b.decompress()
    assert b.verify()
    raw = b.raw.cpu().numpy()
    comp = b.comp.cpu().numpy()
    for i in (0, 7, 23):
        src = raw[i * b.U:(i + 1) * b.U].tobytes()
        m, ref = oracle.lz4_compress(src)
        assert m == b.csize[i]
        assert comp[i * b.slot:i * b.slot + m].tobytes() == ref
    # a different output placement: unaligned destinations and sources
    out = torch.zeros(24 * (b.U + 32), dtype=torch.uint8, device=gpu)
    src_copy = torch.zeros(24 * (b.slot + 32), dtype=torch.uint8, device=gpu)
    offs_s = np.array([i * (b.slot + 32) + (i % 13) for i in range(24)])
    for i in range(24):
        src_copy[offs_s[i]:offs_s[i] + b.csize[i]] = b.comp[i * b.slot:i * b.slot + b.csize[i]]
    offs_d = np.array([i * (b.U + 32) + (i * 7) % 16 for i in range(24)])
    desc = D.make_desc(src_copy, offs_s, b.csize, out, offs_d, [b.U] * 24)
    ret = torch.empty(24, dtype=torch.int32, device=gpu)
    D.lz4_decompress(desc, ret)
    torch.cuda.synchronize()
    assert (ret == b.U).all()
    for i in range(24):
        assert torch.equal(out[offs_d[i]:offs_d[i] + b.U], b.raw[i * b.U:(i + 1) * b.U])


def _dense_tokens(seed, ntok):
    """A valid LZ4 block made of 3..5-byte sequences (more tokens per input
    window than the per-window table holds): exercises windows that end at the
    table capacity and restart at the next token."""
    rng = random.Random(seed)
    out = bytearray([0x80]) + bytes(rng.randrange(256) for _ in range(8)) + (rng.randrange(1, 9)).to_bytes(2, "little")
    for _ in range(ntok):
        k = rng.randrange(10)
        if k < 6:      # ll 0, ml 4: 3 bytes
            out += bytes([0x00]) + rng.randrange(1, 9).to_bytes(2, "little")
        elif k < 8:    # ll 1, ml 5: 4 bytes
            out += bytes([0x11, rng.randrange(256)]) + rng.randrange(1, 9).to_bytes(2, "little")
        else:          # ll 0, ml 15+4+e: 4 bytes
            out += bytes([0x0F]) + rng.randrange(1, 9).to_bytes(2, "little") + bytes([rng.randrange(0, 40)])
    out += bytes([0xF0, 1]) + bytes(rng.randrange(256) for _ in range(16))
    return bytes(out)


def test_lz4_decode_dense_tokens(gpu, oracle):
    c = C.LZ4()
    comps = [_dense_tokens(70 + i, n) for i, n in enumerate((10, 700, 5000, 60000, 250000))]
    pairs, want = [], []
    for comp in comps:
        r, out = oracle.lz4_decompress(comp, 8 << 20)
        assert r > 0
        pairs.append((bytearray(r), comp))
        want.append((r, out[:r]))
    res = c.DecompressBatch(pairs)
    for (dst, _), (r, out), (n, err) in zip(pairs, want, res):
        assert err is None and n == r and bytes(dst[:n]) == out


def _far_head_stream(rng, pre, src_pos, ml):
    """Filler tokens up to output `pre`, then one token whose match reads from
    output position src_pos (0..3) -- a far source in the first dword of dst
    once the output passes the 4 KiB LDS ring -- then filler and a literal tail."""
    out = bytearray()
    produced = 0

    def tok(lits, off, mlen):
        nonlocal produced
        ll = len(lits)
        mcode = mlen - 4
        t = (min(ll, 15) << 4) | min(mcode, 15)
        b = bytearray([t])
        if ll >= 15:
            r = ll - 15
            while r >= 255:
                b.append(255)
                r -= 255
            b.append(r)
        b += lits + off.to_bytes(2, "little")
        if mcode >= 15:
            r = mcode - 15
            while r >= 255:
                b.append(255)
                r -= 255
            b.append(r)
        produced += ll + mlen
        return b

    lits = bytes(rng.randrange(256) for _ in range(12))
    out += tok(lits, 5, 4)
    while produced + 14 + 40 < pre:
        out += tok(bytes(rng.randrange(256) for _ in range(10)), rng.randrange(1, 9), 4)
    ll = max(1, pre - produced)
    ms = produced + ll
    out += tok(bytes(rng.randrange(256) for _ in range(ll)), ms - src_pos, ml)
    for _ in range(20):
        out += tok(bytes(rng.randrange(256) for _ in range(10)), rng.randrange(1, 9), 4)
    out += bytes([0xF0, 1]) + bytes(rng.randrange(256) for _ in range(16))
    return bytes(out)


def test_lz4_far_source_at_block_start(gpu, oracle):
    """Far matches whose source starts in dst's first dword (the far loads must
    not read below the block's first dword), every dst alignment."""
    import torch
    from juicefs_amd import device as D
    rng = random.Random(5)
    streams = []
    for pre in range(4070, 4112, 3):
        for sp in range(4):
            streams.append(_far_head_stream(rng, pre, sp, 4 + rng.randrange(40)))
    want = []
    for st in streams:
        r, o = oracle.lz4_decompress(st, 1 << 16)
        assert r > 0
        want.append(o[:r])
    n = len(streams)
    cap = max(len(w) for w in want)
    src = torch.zeros(n * (len(max(streams, key=len)) + 32), dtype=torch.uint8, device=gpu)
    slot_s = len(max(streams, key=len)) + 32
    offs_s = [i * slot_s for i in range(n)]
    host = np.zeros(src.numel(), dtype=np.uint8)
    for i, st in enumerate(streams):
        host[offs_s[i]:offs_s[i] + len(st)] = np.frombuffer(st, dtype=np.uint8)
    src.copy_(torch.from_numpy(host))
    for mis in (0, 1, 2, 3, 5, 13):
        out = torch.full((n * (cap + 64) + 64,), 0xEE, dtype=torch.uint8, device=gpu)
        offs_d = [i * (cap + 64) + mis for i in range(n)]
        desc = D.make_desc(src, offs_s, [len(s) for s in streams], out, offs_d, [len(w) for w in want])
        ret = torch.empty(n, dtype=torch.int32, device=gpu)
        D.lz4_decompress(desc, ret)
        torch.cuda.synchronize()
        r = ret.cpu().tolist()
        oh = out.cpu().numpy()
        for i, w in enumerate(want):
            assert r[i] == len(w), (mis, i, r[i], len(w))
            assert oh[offs_d[i]:offs_d[i] + len(w)].tobytes() == w, (mis, i)


def test_lz4_encode_long_literal_runs(gpu, oracle):
    """Literal runs around the encoder's output-ring sizes (the token stays
    pending while the run streams out) inside text blocks, byte-exact."""
    c = C.LZ4()
    srcs = []
    for i, run in enumerate((960, 1000, 1024, 1040, 1100, 1984, 2000, 2048, 2100, 4000, 4096, 9000)):
        base = bytearray(gen_block("T", 80 + i, 300000))
        k = 1000 + 17 * i
        base[k:k + run] = gen_block("R", 90 + i, run)
        k2 = 150000 + 31 * i
        base[k2:k2 + run] = gen_block("R", 190 + i, run)
        srcs.append(bytes(base))
    srcs.append(gen_block("R", 7, 2048) + gen_block("T", 8, 5000))
    pairs = [(bytearray(c.CompressBound(len(s))), s) for s in srcs]
    res = c.CompressBatch(pairs)
    for s, (d, _), (n, err) in zip(srcs, pairs, res):
        m, ref = oracle.lz4_compress(s)
        assert err is None and n == m and bytes(d[:n]) == ref


def test_lz4_long_literal_runs_then_far_and_near_matches(gpu, oracle):
    """Literal runs >= 8 KiB take the HBM-to-HBM path (lz4_decode.hip
    direct_lit); later matches must find the run's bytes in the ring (last 4 KiB)
    and in HBM (older), right after the run and far behind it; short
    destinations must still fail exactly where liblz4 fails."""
    rng = np.random.default_rng(77)
    c = C.LZ4()
    pairs, want = [], []
    for k, run in enumerate((8192, 8193, 12345, 40000, 65536, 200000)):
        r = rng.integers(0, 256, run, dtype=np.uint8).tobytes()
        text = gen_block("T", 300 + k, 3000)
        # copies out of the run: just behind its end (ring), mid-run and near its start (HBM, < 64 KiB back)
        src = (r + r[-600:-100] + text + r[run // 2:run // 2 + 700] + text[:900] + r[max(0, run - 60000):][:1500]
               + gen_block("R", 400 + k, 9000 + 37 * k) + text)
        _, comp = oracle.lz4_compress(src)
        n = len(src)
        for cap in (n, n + 5):
            pairs.append((bytearray(cap), comp))
            want.append((n, src))
        rr, _ = oracle.lz4_decompress(comp, n - 1)
        pairs.append((bytearray(n - 1), comp))
        want.append((rr, None))
    res = c.DecompressBatch(pairs)
    for (dst, comp), (n_exp, src), (n, err) in zip(pairs, want, res):
        if n_exp >= 0:
            assert err is None and n == n_exp
            assert bytes(dst[:n]) == src
        else:
            assert err is not None and n == n_exp


def test_lz4_long_periodic_matches(gpu, oracle):
    """Long matches with offsets 1/2/4/8/16 are written as pure stores
    (lz4_decode.hip direct_fill); other offsets take the ring path.  Text
    around the runs makes later tokens read both the run's tail (ring) and
    its body (HBM); short destinations fail where liblz4 fails."""
    c = C.LZ4()
    pairs, want = [], []
    for k, (period, reps) in enumerate(((1, 20000), (2, 9000), (4, 5000), (8, 3000), (16, 1500), (3, 7000),
                                        (16, 300), (1, 70000))):
        pat = gen_block("R", 500 + k, period)
        text = gen_block("T", 600 + k, 2500)
        src = text[:700] + pat * reps + text + (pat * reps)[:5000 + 13 * k] + text[1000:2400] + pat * 40 + text[:300]
        _, comp = oracle.lz4_compress(src)
        n = len(src)
        for cap in (n, n + 9):
            pairs.append((bytearray(cap), comp))
            want.append((n, src))
        rr, _ = oracle.lz4_decompress(comp, n - 3)
        pairs.append((bytearray(n - 3), comp))
        want.append((rr, None))
    res = c.DecompressBatch(pairs)
    for (dst, comp), (n_exp, src), (n, err) in zip(pairs, want, res):
        if n_exp >= 0:
            assert err is None and n == n_exp
            assert bytes(dst[:n]) == src
        else:
            assert err is not None and n == n_exp
