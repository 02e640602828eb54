"""GPU parity of the Zstd small-batch decode path (juicefs_amd/csrc/zstd_split.inc:
one workgroup per block, origin-map replay, the exact one-wave replay for any
input outside its proven cases) -- the path of a lone frame through
jfs_decompress, i.e. pkg/chunk's one Decompress per cache miss
(cached_store.go:755-823 -> compress.go:94-103).  Bar: the decoded bytes and
result codes of the golden fixtures and of the CPU oracle (oracle/zstd_oracle.c)
on every case, and the path really replaying the well-formed frames itself."""
import hashlib
import os
import statistics
import time

import numpy as np
import pytest
import torch

from juicefs_amd import compress as C
from juicefs_amd import device as D
from tests.zstd_l1_cases import CASES, make_case

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def frames_bin(golden):
    with open(os.path.join(GOLD, golden["zstd"]["bin"]), "rb") as f:
        return f.read()


def run_device(srcs, caps, dev, src_mis=0, dst_mis=0):
    """Decode each src into its own dst (cap bytes) in ONE device call;
    returns (rets, outputs[:ret]) and checks nothing is written past cap."""
    n = len(srcs)
    so, do, off, doff = [], [], 0, 0
    for i, s in enumerate(srcs):
        m = (src_mis + 7 * i) % 16 if src_mis else 0
        so.append(off + m)
        off = (off + m + len(s) + 64 + 15) & ~15
        dm = (dst_mis + 5 * i) % 16 if dst_mis else 0
        do.append(doff + dm)
        doff = (doff + dm + caps[i] + 64 + 15) & ~15
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
    for o, c in zip(do, caps):
        assert (dh[o + c:o + c + 16] == 0xAB).all()
    return r, [dh[o:o + max(x, 0)].tobytes() for o, x in zip(do, r)]


def test_split_lone_golden_frames(gpu, golden, frames_bin):
    """Every golden frame (levels 1/3/..., classes T/Z/R, 1 B .. 4 MiB) alone
    in a call: the small-batch path replays each itself."""
    D.zstd_split_counts(reset=True)
    ents = golden["zstd"]["frames"]
    for f in ents:
        src = frames_bin[f["off"]:f["off"] + f["csize"]]
        r, outs = run_device([src], [f["size"]], gpu, src_mis=5, dst_mis=3)
        assert r[0] == f["size"] and sha(outs[0]) == f["src_sha"], (f["cls"], f.get("level"), f["size"], r[0])
    done, handed = D.zstd_split_counts()
    assert done == len(ents) and handed == 0, (done, handed)


def test_split_special_frames(gpu, golden, frames_bin):
    """The special fixtures (multi-frame, skippable, checksummed, ...):
    correct through the hand-over to the exact replay."""
    for f in golden["zstd"]["special"]:
        src = frames_bin[f["off"]:f["off"] + f["csize"]]
        r, outs = run_device([src], [f["size"]], gpu)
        assert r[0] == f["size"] and sha(outs[0]) == f["src_sha"], f.get("name")


def test_split_corpus_vs_oracle(gpu, golden, oracle):
    """Accept + corrupt corpus in batches of 7 (small-batch path): codes and
    bytes of the oracle; both the origin-map replay and the hand-over run."""
    cases = golden["zstd"]["accept"] + golden["zstd"]["corpus"]
    D.zstd_split_counts(reset=True)
    bad = []
    for i in range(0, len(cases), 7):
        part = cases[i:i + 7]
        srcs = [bytes.fromhex(a["src"]) for a in part]
        caps = [a["cap"] for a in part]
        r, outs = run_device(srcs, caps, gpu, src_mis=1 + i % 5, dst_mis=2)
        for s, c, x, o in zip(srcs, caps, r, outs):
            want, wo = oracle.zstd_decompress(s, c)
            if x != want or (x >= 0 and o != wo):
                bad.append((s.hex()[:80], c, want, x))
    assert not bad, bad[:5]
    done, handed = D.zstd_split_counts()
    assert done > 0 and handed > 0, (done, handed)


def test_split_short_caps_vs_oracle(gpu, golden, frames_bin, oracle):
    """One byte short, exact, and generous caps: dstSize_tooSmall exactly as
    the oracle, nothing written past cap."""
    ents = [f for f in golden["zstd"]["frames"] if f["size"] <= 300000][:12]
    for f in ents:
        src = frames_bin[f["off"]:f["off"] + f["csize"]]
        caps = [max(f["size"] - 1, 0), f["size"], f["size"] + 1000]
        r, outs = run_device([src] * 3, caps, gpu, dst_mis=7)
        for c, x, o in zip(caps, r, outs):
            want, wo = oracle.zstd_decompress(src, c)
            assert x == want and (x < 0 or o == wo), (f["size"], c, x, want)


def test_split_level1_cases_roundtrip(gpu):
    """The level-1 encode fixtures' inputs (4 MiB T/Z/R/mixed/skewed frames,
    size-tier edges, multi-block mixes: raw, RLE and compressed blocks,
    treeless literals, repeat tables), framed byte-exactly by the GPU encoder
    (tests/test_zstd_encode_gpu.py pins those frames to libzstd), each
    decoded alone."""
    z = C.ZStandard()
    srcs = [make_case(k, s, n) for k, s, n in CASES]
    pairs = [(bytearray(z.CompressBound(len(s))), s) for s in srcs]
    res = z.CompressBatch(pairs)
    assert all(e is None for _, e in res)
    frames = [bytes(d[:n]) for (d, _), (n, _) in zip(pairs, res)]
    D.zstd_split_counts(reset=True)
    for s, fr in zip(srcs, frames):
        r, outs = run_device([fr], [len(s)], gpu, dst_mis=1)
        assert r[0] == len(s) and outs[0] == s, len(s)
    done, handed = D.zstd_split_counts()
    assert done == len(srcs) and handed == 0, (done, handed)


def test_split_matches_exact_path(gpu, golden, frames_bin):
    """The same frames through the small-batch path (batch of 8) and the
    one-wave path (batch of 160 > JFS_ZSTD_SPLIT_MAX's default 128): identical
    results."""
    ents = [f for f in golden["zstd"]["frames"] if f["size"] >= 100000][:8]
    srcs = [frames_bin[f["off"]:f["off"] + f["csize"]] for f in ents]
    caps = [f["size"] for f in ents]
    r1, o1 = run_device(srcs, caps, gpu)
    k = (160 + len(srcs) - 1) // len(srcs)
    r2, o2 = run_device(srcs * k, caps * k, gpu)
    assert r1 == r2[:len(srcs)] and o1 == o2[:len(srcs)]
    for f, x, o in zip(ents, r1, o1):
        assert x == f["size"] and sha(o) == f["src_sha"]


def test_split_one_call_lone_latency(gpu, golden, frames_bin):
    """jfs_decompress of one 4 MiB frame (level 1 and level 3): correct, and
    its p50 latency (host buffers in and out) recorded."""
    z = C.ZStandard()
    cases = {}
    for f in golden["zstd"]["frames"]:  # libzstd frames (level 3 at 4 MiB)
        if f["size"] == 4 << 20:
            cases.setdefault("L%d-%s" % (f.get("level", 0), f["cls"]), (frames_bin[f["off"]:f["off"] + f["csize"]],
                                                                       f["size"], f["src_sha"]))
    for k in ("T", "M"):  # level 1, byte-exact GPU frames of the 4 MiB fixture inputs
        raw = make_case(k, 4100 if k == "T" else 4103, 4 << 20)
        d = bytearray(z.CompressBound(len(raw)))
        n, err = z.Compress(d, raw)
        assert err is None
        cases["L1-" + k] = (bytes(d[:n]), len(raw), sha(raw))
    lat = {}
    for name, (src, size, want) in cases.items():
        out = bytearray(b"\x01") * size
        ts = []
        for _ in range(12):
            t0 = time.perf_counter()
            n, err = z.Decompress(out, src)
            ts.append(time.perf_counter() - t0)
            assert err is None and n == size
        assert sha(bytes(out)) == want, name
        lat[name] = round(statistics.median(ts[2:]) * 1e3, 2)
    print("lone 4 MiB zstd decode p50 ms:", lat)
    assert lat and all(v < 40 for v in lat.values()), lat


def test_split_declines_block_heavy_inputs(gpu, oracle):
    """An input of thousands of tiny blocks (here 5,000 empty raw blocks
    before the data) would need a record per block: the batch takes the
    one-wave path instead (the split counters do not move), same result."""
    import struct
    data = bytes(range(100))
    frame = struct.pack("<I", 0xFD2FB528) + bytes([0x00, 0x00])  # no FCS, window 1 KiB
    frame += b"\x00\x00\x00" * 5000  # empty raw blocks
    frame += (1 | (len(data) << 3)).to_bytes(3, "little") + data
    want, wo = oracle.zstd_decompress(frame, 1000)
    assert want == len(data) and wo == data
    D.zstd_split_counts(reset=True)
    r, outs = run_device([frame], [1000], gpu)
    assert r[0] == want and outs[0] == data
    assert D.zstd_split_counts() == (0, 0)
