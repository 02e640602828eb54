"""GPU parity of the small-batch LZ4 decoder (lz4_split.hip, reached through
jfs_lz4_decompress_device_small and, for batches of <= JFS_LZ4_SPLIT_MAX
blocks, through jfs_decompress / jfs_decompress_batch) against the CPU oracle
and the liblz4 1.9.3 acceptance corpus.  Bar: identical return values on every
case and identical bytes on success -- whether a block is decoded by the split
path itself or handed to the one-workgroup kernel.  The diagnostic counters
check that well-formed text blocks stay on the split path."""
import hashlib
import random

import numpy as np
import pytest
import torch

from juicefs_amd import compress as C
from juicefs_amd import device as D
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu


def sha(b):
    return hashlib.sha256(b).hexdigest()


def run_small(srcs, caps, dev, group=64, mis=0):
    """Decode srcs into caps-sized outputs with the small-batch device API in
    groups of `group`; returns (rets, outputs[:ret])."""
    rets, outs = [], []
    for g0 in range(0, len(srcs), group):
        ss, cc = srcs[g0:g0 + group], caps[g0:g0 + group]
        so, do, off, doff = [], [], 0, 0
        for i, (s, c) in enumerate(zip(ss, cc)):
            m = (mis * (i + 1)) % 16 if mis else 0
            so.append(off + m)
            off = (off + m + len(s) + 64 + 15) & ~15
            dm = (mis * (i + 3)) % 16 if mis else 0
            do.append(doff + dm)
            doff = (doff + dm + c + 64 + 15) & ~15
        host = np.zeros(off + 64, dtype=np.uint8)
        for s, o in zip(ss, so):
            host[o:o + len(s)] = np.frombuffer(s, dtype=np.uint8)
        src_t = torch.from_numpy(host).to(dev)
        dst_t = torch.full((doff + 64,), 0xEE, dtype=torch.uint8, device=dev)
        desc = D.make_desc(src_t, so, [len(s) for s in ss], dst_t, do, cc)
        ret = torch.zeros(len(ss), dtype=torch.int32, device=dev)
        D.lz4_decompress_small(desc, ret, [len(s) for s in ss], cc)
        torch.cuda.synchronize()
        r = ret.cpu().tolist()
        dh = dst_t.cpu().numpy()
        for o, c in zip(do, cc):  # nothing written at or past cap
            assert (dh[o + c:o + c + 16] == 0xEE).all()
        rets += r
        outs += [dh[o:o + max(x, 0)].tobytes() for o, x in zip(do, r)]
    return rets, outs


def test_split_text_blocks_stay_on_the_split_path(gpu, oracle):
    """4 MiB text blocks (the cache-miss shape): exact bytes, and decoded by
    the split path itself (no hand-off)."""
    srcs = [gen_block("T", 4100 + i, 4 << 20) for i in range(3)] + [gen_block("T", 4200, 1 << 20),
                                                                    gen_block("T", 4201, 65536 + 333)]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    D.lz4_split_counts(reset=True)
    for mis in (0, 5):
        r, outs = run_small(comps, [len(s) for s in srcs], gpu, mis=mis)
        assert r == [len(s) for s in srcs]
        assert all(o == s for o, s in zip(outs, srcs))
    done, handed = D.lz4_split_counts()[:2]
    assert done == 2 * len(srcs) and handed == 0, (done, handed)


def test_split_many_text_blocks_thread_emit(gpu, oracle):
    """Eight 4 MiB text blocks in one launch (~130 k segments: past
    EMIT_WAVE_MAX, the thread-per-segment emit): exact, and on the split path."""
    srcs = [gen_block("T", 4400 + i, 4 << 20) for i in range(8)]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    assert sum((len(c) + 127) // 128 for c in comps) > 65536
    D.lz4_split_counts(reset=True)
    r, outs = run_small(comps, [len(s) for s in srcs], gpu, mis=3)
    assert r == [len(s) for s in srcs]
    assert all(o == s for o, s in zip(outs, srcs))
    done, handed = D.lz4_split_counts()[:2]
    assert done == len(srcs) and handed == 0, (done, handed)


def test_split_blocks_vs_oracle_all_classes(gpu, oracle):
    cases = [(cls, n) for cls in "TZR" for n in (1, 12, 13, 100, 4096, 65535, 65547, 131072, 1 << 20)] + [
        ("T", 4 << 20), ("Z", 4 << 20), ("R", 4 << 20)]
    srcs, caps, want = [], [], []
    for i, (cls, n) in enumerate(cases):
        src = gen_block(cls, 1900 + i, n)
        _, comp = oracle.lz4_compress(src)
        for cap in (n, n + 77, max(n - 1, 0)):
            r, o = oracle.lz4_decompress(comp, cap)
            srcs.append(comp)
            caps.append(cap)
            want.append((r, o))
    got, outs = run_small(srcs, caps, gpu, group=40)
    for (r, o), g, out, cap in zip(want, got, outs, caps):
        assert g == r, (g, r, cap)
        if r >= 0:
            assert out == o[:r]


def test_split_corpus_exact(gpu, golden):
    """The 3,000-case liblz4 1.9.3 acceptance corpus through the split path:
    same return value on every case, same bytes on success."""
    cases = golden["lz4"]["decode_corpus"]
    srcs = [bytes.fromhex(e["src"]) for e in cases]
    caps = [max(e["cap"], 0) for e in cases]
    got, outs = run_small(srcs, caps, gpu)
    bad = [(e["ret"], g) for e, g, o in zip(cases, got, outs)
           if g != e["ret"] or (g >= 0 and sha(o) != e["out_sha"])]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:5]}"


def _dense_tokens(seed, ntok):
    rng = random.Random(seed)
    out = bytearray([0x80]) + bytes(rng.randrange(256) for _ in range(8)) + (rng.randrange(1, 9)).to_bytes(2, "little")
    for _ in range(ntok):
        k = rng.randrange(10)
        if k < 6:
            out += bytes([0x00]) + rng.randrange(1, 9).to_bytes(2, "little")
        elif k < 8:
            out += bytes([0x11, rng.randrange(256)]) + rng.randrange(1, 9).to_bytes(2, "little")
        else:
            out += bytes([0x0F]) + rng.randrange(1, 9).to_bytes(2, "little") + bytes([rng.randrange(0, 40)])
    out += bytes([0xF0, 1]) + bytes(rng.randrange(256) for _ in range(16))
    return bytes(out)


def test_split_dense_tokens_and_long_runs(gpu, oracle):
    """Back-to-back 3-byte tokens, literal runs spanning many segments, long
    periodic matches, matches into a random run: exact against the oracle."""
    rng = np.random.default_rng(9)
    srcs, caps, want = [], [], []

    def add(comp, cap):
        r, o = oracle.lz4_decompress(comp, cap)
        srcs.append(comp)
        caps.append(cap)
        want.append((r, o[:max(r, 0)]))
    for i, n in enumerate((10, 700, 5000, 60000, 250000)):
        comp = _dense_tokens(70 + i, n)
        r, _ = oracle.lz4_decompress(comp, 8 << 20)
        add(comp, r)
    for k, run in enumerate((300, 1000, 2000, 8192, 40000, 200000)):
        r = rng.integers(0, 256, run, dtype=np.uint8).tobytes()
        text = gen_block("T", 300 + k, 3000)
        src = text + r + text[:900] + r[run // 2:run // 2 + 700] + text + r[:1500] + text
        _, comp = oracle.lz4_compress(src)
        add(comp, len(src))
        add(comp, len(src) - 1)
    for k, (period, reps) in enumerate(((1, 20000), (2, 9000), (3, 7000), (16, 1500), (1, 70000))):
        pat = gen_block("R", 500 + k, period)
        text = gen_block("T", 600 + k, 2500)
        src = text[:700] + pat * reps + text + (pat * reps)[:5000] + text[1000:2400] + pat * 40 + text[:300]
        _, comp = oracle.lz4_compress(src)
        add(comp, len(src))
        add(comp, len(src) - 3)
    got, outs = run_small(srcs, caps, gpu, group=16)
    for (r, o), g, out in zip(want, got, outs):
        assert g == r
        if r >= 0:
            assert out == o


def test_split_through_one_call_api(gpu, oracle):
    """jfs_decompress (the cachedStore.load call) goes through the coalescer,
    whose small batches take the split path: exact bytes and return values."""
    c = C.LZ4()
    src = gen_block("T", 4300, 4 << 20)
    comp = oracle.lz4_compress(src)[1]
    D.lz4_split_counts(reset=True)
    out = bytearray(len(src))
    n, err = c.Decompress(out, comp)
    assert err is None and n == len(src) and bytes(out) == src
    short = bytearray(len(src) - 1)
    r, _ = oracle.lz4_decompress(comp, len(src) - 1)
    n, err = c.Decompress(short, comp)
    assert err is not None and n == r
    done, handed = D.lz4_split_counts()[:2]
    assert done + handed == 2 and done >= 1, (done, handed)


def test_split_one_segment_exact_cap_stays_on_split_path(gpu, oracle):
    """A block of <= 256 compressed bytes decoded into exactly its size (the
    one-call path's dst) is decoded by the split path itself: the count of a
    segment that ends exactly at dst_cap is not an overflow."""
    srcs = [gen_block("T", 5100 + i, n) for i, n in enumerate((40, 100, 200, 250))] + [b"a" * 200, b"ab" * 150]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    assert all(len(c) <= 256 for c in comps), [len(c) for c in comps]
    D.lz4_split_counts(reset=True)
    r, outs = run_small(comps, [len(s) for s in srcs], gpu)
    assert r == [len(s) for s in srcs]
    assert all(o == s for o, s in zip(outs, srcs))
    done, handed = D.lz4_split_counts()[:2]
    assert done == len(srcs) and handed == 0, (done, handed)


def test_split_device_sizes_beyond_host_budget_go_exact(gpu, oracle):
    """jfs_lz4_decompress_device_small sizes its scratch from the HOST
    (src_len, dst_cap) arrays; a device descriptor asking for more (a caller
    bug) must not overrun that scratch: the block is handed to the exact
    kernel, which decodes it from its descriptor."""
    srcs = [gen_block("T", 5200 + i, 65536 + 17 * i) for i in range(4)]
    comps = [oracle.lz4_compress(s)[1] for s in srcs]
    so, off = [], 0
    for c in comps:
        so.append(off)
        off = (off + len(c) + 64 + 15) & ~15
    host = np.zeros(off + 64, dtype=np.uint8)
    for c, o in zip(comps, so):
        host[o:o + len(c)] = np.frombuffer(c, dtype=np.uint8)
    src_t = torch.from_numpy(host).to(gpu)
    caps = [len(s) for s in srcs]
    do = [i * (70000 + 64) for i in range(len(srcs))]
    dst_t = torch.full((do[-1] + 70000 + 64,), 0xEE, dtype=torch.uint8, device=gpu)
    desc = D.make_desc(src_t, so, [len(c) for c in comps], dst_t, do, caps)
    ret = torch.zeros(len(srcs), dtype=torch.int32, device=gpu)
    # host copies claim much smaller inputs and outputs than the descriptors
    D.lz4_split_counts(reset=True)
    D.lz4_decompress_small(desc, ret, [64] * len(srcs), [1000] * len(srcs))
    torch.cuda.synchronize()
    assert ret.cpu().tolist() == caps
    dh = dst_t.cpu().numpy()
    for o, s in zip(do, srcs):
        assert dh[o:o + len(s)].tobytes() == s
    done, handed = D.lz4_split_counts()[:2]
    assert handed == len(srcs), (done, handed)


def _chain_stream(units, seed=7):
    """An LZ4 stream of `units` 11-byte output units, each one literal byte and
    a 10-byte match at offset 11: every match byte copies the same byte of the
    unit before, so its origin chain runs back through every earlier unit."""
    rng = random.Random(seed)
    first = bytes(rng.randrange(256) for _ in range(11))
    out = bytearray([0xB6]) + first + (11).to_bytes(2, "little")  # ll 11, ml 10
    for _ in range(units - 1):
        out += bytes([0x16, rng.randrange(256)]) + (11).to_bytes(2, "little")  # ll 1, ml 10
    out += bytes([0xF0, 1]) + bytes(rng.randrange(256) for _ in range(16))  # last: 16 literals
    return bytes(out)


def test_split_deep_origin_chains(gpu, oracle):
    """Origin chains ~380,000 steps deep (4 MiB of 11-byte units): the pointer
    jumping's round count, sized from the proven bound (a chain takes at most
    one step per token), settles them on the split path itself."""
    comps = [_chain_stream(381300), _chain_stream(20000, seed=8), _chain_stream(3, seed=9)]
    caps = []
    for c in comps:
        n, _ = oracle.lz4_decompress(c, 8 << 20)
        assert n > 0
        caps.append(n)
    assert caps[0] > 4_190_000
    D.lz4_split_counts(reset=True)
    r, outs = run_small(comps, caps, gpu)
    for c, cap, x, o in zip(comps, caps, r, outs):
        want_n, want = oracle.lz4_decompress(c, cap)
        assert x == want_n and o == want
    cnt = D.lz4_split_counts()
    assert cnt[0] == len(comps) and cnt[1] == 0, cnt
