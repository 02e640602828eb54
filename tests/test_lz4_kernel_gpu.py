"""GPU parity of the one-workgroup-per-block LZ4 decode kernel (the headline
kernel, lz4_decode.hip) called directly through jfs_lz4_decompress_device, so
that no batch routing (the small-batch split decoder) takes any case first.
Every stream shape the segment-walk parser must get right: liblz4 1.9.3
acceptance corpus (exact negative returns), dense 3..5-byte tokens (window
table cap), literal runs that jump over one or many 128-byte parser segments
and whole 8 KiB spans, long length extensions, periodic matches, every data
class at sizes around the span/window boundaries, short destinations.
Bar: the oracle's return value and bytes, for every case."""
import random

import numpy as np
import pytest

from juicefs_amd.blockgen import gen_block
from tests.test_lz4_gpu import _dense_tokens

pytestmark = pytest.mark.gpu


def _run_device(gpu, comps, caps, mis_s=0, mis_d=0):
    import torch
    from juicefs_amd import device as D
    n = len(comps)
    slot_s = [(len(c) + 64 + 15) // 16 * 16 for c in comps]
    offs_s = np.cumsum([0] + slot_s[:-1]) + mis_s
    host = np.zeros(int(sum(slot_s)) + 64, dtype=np.uint8)
    for i, c in enumerate(comps):
        host[offs_s[i]:offs_s[i] + len(c)] = np.frombuffer(c, dtype=np.uint8)
    src = torch.from_numpy(host).to(gpu)
    slot_d = [(max(cp, 0) + 64 + 15) // 16 * 16 for cp in caps]
    offs_d = np.cumsum([0] + slot_d[:-1]) + mis_d
    out = torch.full((int(sum(slot_d)) + 64,), 0xEE, dtype=torch.uint8, device=gpu)
    desc = D.make_desc(src, offs_s, [len(c) for c in comps], out, offs_d, caps)
    ret = torch.empty(n, dtype=torch.int32, device=gpu)
    D.lz4_decompress(desc, ret)
    torch.cuda.synchronize()
    return ret.cpu().tolist(), out.cpu().numpy(), offs_d


def _check(gpu, oracle, comps, caps, **kw):
    r, oh, offs_d = _run_device(gpu, comps, caps, **kw)
    bad = []
    for i, (c, cap) in enumerate(zip(comps, caps)):
        want, ref = oracle.lz4_decompress(c, cap)
        if r[i] != want:
            bad.append((i, len(c), cap, r[i], want))
        elif want > 0 and oh[offs_d[i]:offs_d[i] + want].tobytes() != ref[:want]:
            bad.append((i, len(c), cap, "bytes"))
    assert not bad, f"{len(bad)} of {len(comps)} mismatch, first: {bad[:4]}"


def _tok(lits, off, mlen):
    ll, mcode = len(lits), mlen - 4
    b = bytearray([(min(ll, 15) << 4) | min(mcode, 15)])
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
    return b


def _mixed_runs_stream(seed, n_tok):
    """Short text-like tokens interleaved with literal runs of 15..20000 bytes
    and matches with long length extensions: chains that jump over segment
    and span boundaries, tokens whose 255-extension bytes straddle them."""
    rng = random.Random(seed)
    out = bytearray()
    produced = 0
    for _ in range(n_tok):
        k = rng.randrange(20)
        if k == 0:
            ll = rng.choice([15, 16, 127, 128, 129, 255, 270, 1000, 4096, 8191, 8192, 8300, 20000])
        elif k < 3:
            ll = rng.randrange(15, 300)
        else:
            ll = rng.randrange(0, 15)
        if rng.randrange(25) == 0:
            ml = rng.choice([19, 19 + 254, 19 + 255, 19 + 600, 5000])
        else:
            ml = rng.randrange(4, 19)
        lits = bytes(rng.randrange(256) for _ in range(ll))
        produced += ll
        off = rng.randrange(1, min(produced, 65535) + 1) if produced > 0 else 0
        if off == 0:
            lits = lits + bytes([rng.randrange(256)])
            produced += 1
            off = 1
        out += _tok(lits, off, ml)
        produced += ml
    out += bytes([0xF0, 5]) + bytes(rng.randrange(256) for _ in range(20))
    return bytes(out)


def test_main_kernel_corpus_exact(gpu, golden, oracle):
    cases = golden["lz4"]["decode_corpus"]
    comps = [bytes.fromhex(e["src"]) for e in cases]
    caps = [max(e["cap"], 0) for e in cases]
    r, oh, offs_d = _run_device(gpu, comps, caps)
    from tests.test_lz4_gpu import sha
    bad = [(i, r[i], e["ret"]) for i, e in enumerate(cases)
           if r[i] != e["ret"] or (e["ret"] > 0 and sha(oh[offs_d[i]:offs_d[i] + r[i]].tobytes()) != e["out_sha"])]
    assert not bad, f"{len(bad)} mismatches, first: {bad[:3]}"


def test_main_kernel_classes_and_sizes(gpu, oracle):
    comps, caps = [], []
    sizes = [17, 100, 2047, 2048, 2049, 8191, 8192, 8193, 16384 + 77, 65547, 100000, 262144 + 5, 1 << 20]
    for i, n in enumerate(sizes):
        for cls in "TZR":
            src = gen_block(cls, 1300 + 3 * i + "TZR".index(cls), n)
            _, comp = oracle.lz4_compress(src)
            comps += [comp, comp, comp]
            caps += [n, n + 100, n - 1]
    _check(gpu, oracle, comps, caps)


def test_main_kernel_text_with_runs(gpu, oracle):
    """Text blocks with random runs of every length around the parser's 128-byte
    segments and 8 KiB spans inserted at many offsets."""
    comps, caps = [], []
    runs = [100, 127, 128, 129, 250, 256, 300, 1000, 4096, 8000, 8192, 8200, 9000, 17000, 40000]
    for i, run in enumerate(runs):
        base = bytearray(gen_block("T", 1500 + i, 200000))
        for k, at in enumerate((333, 5000 + 61 * i, 77777, 150001)):
            base[at:at + run] = gen_block("R", 1600 + 7 * i + k, run)
        s = bytes(base)
        _, comp = oracle.lz4_compress(s)
        comps += [comp, comp]
        caps += [len(s), len(s) - 3]
    _check(gpu, oracle, comps, caps)


def test_main_kernel_handmade_streams(gpu, oracle):
    comps = [_mixed_runs_stream(40 + i, n) for i, n in enumerate((50, 400, 3000, 12000, 30000))]
    comps += [_dense_tokens(90 + i, n) for i, n in enumerate((700, 5000, 60000, 250000))]
    caps = []
    outc = []
    for c in comps:
        r, _ = oracle.lz4_decompress(c, 16 << 20)
        assert r > 0
        caps.append(r)
    comps2, caps2 = [], []
    for c, r in zip(comps, caps):
        comps2 += [c, c, c]
        caps2 += [r, r + 64, r - 1]
    _check(gpu, oracle, comps2, caps2)
    _check(gpu, oracle, comps2, caps2, mis_s=5, mis_d=3)


def test_main_kernel_truncated_and_corrupt(gpu, oracle):
    """Truncated inputs and flipped bytes in text blocks: the exact negative
    returns (the chain ends at the span where the stream breaks)."""
    rng = random.Random(9)
    comps, caps = [], []
    for i in range(40):
        n = rng.choice([5000, 20000, 70000, 300000])
        src = gen_block("T", 1700 + i, n)
        _, comp = oracle.lz4_compress(src)
        c = bytearray(comp)
        kind = i % 3
        if kind == 0:
            c = c[:rng.randrange(1, len(c))]
        elif kind == 1:
            for _ in range(3):
                c[rng.randrange(len(c))] ^= 1 << rng.randrange(8)
        else:
            at = rng.randrange(len(c))
            c[at:at + 40] = bytes([255]) * min(40, len(c) - at)
        comps.append(bytes(c))
        caps.append(n)
    _check(gpu, oracle, comps, caps)
