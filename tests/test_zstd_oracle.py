"""CPU: the Zstd oracle (oracle/zstd_oracle.c) against fixtures made with
libzstd 1.4.9 (tests/golden/make_golden.py): frames of every class / level /
header variant decode to the generator's bytes, and a 2,000-case mutation
corpus is accepted/rejected exactly as ZSTD_decompress does."""
import hashlib
import os

import pytest

from juicefs_amd.blockgen import gen_block

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(b):
    return hashlib.sha256(b).hexdigest()


@pytest.fixture(scope="module")
def frames_bin(golden):
    with open(os.path.join(GOLD, golden["zstd"]["bin"]), "rb") as f:
        return f.read()


def test_xxh64_known_answers(oracle):
    # XXH64 reference values (xxhash spec test vectors, seed 0)
    assert oracle.xxh64(b"") == 0xEF46DB3751D8E999
    assert oracle.xxh64(b"a") == 0xD24EC4F1A98C6E5B
    assert oracle.xxh64(b"abc") == 0x44BC2CF5AD770999
    import xxhash
    for n in (1, 3, 4, 7, 8, 31, 32, 33, 100, 1000):
        b = bytes(range(256)) * 4
        assert oracle.xxh64(b[:n]) == xxhash.xxh64(b[:n]).intdigest()


def test_zstd_kat(oracle, golden):
    for k in golden["zstd"]["kat"]:
        src = bytes.fromhex(k["src"])
        r, out = oracle.zstd_decompress(bytes.fromhex(k["comp_l1"]), len(src))
        assert r == len(src) and out == src


def test_zstd_frames(oracle, golden, frames_bin):
    """Level 1/3/9/19 frames, 1 B .. 4 MiB, text/zeros/random."""
    seen = set()
    for f in golden["zstd"]["frames"]:
        c = frames_bin[f["off"]:f["off"] + f["csize"]]
        assert sha(c) == f["comp_sha"]
        r, out = oracle.zstd_decompress(c, f["size"])
        assert r == f["size"] and sha(out) == f["src_sha"], (f["cls"], f["level"], f["size"], r)
        if f["size"] <= 300000:
            assert out == gen_block(f["cls"], f["seed"], f["size"])
        # one byte short -> dstSize_tooSmall
        if f["size"] > 0:
            assert oracle.zstd_decompress(c, f["size"] - 1)[0] == -2
        seen.add((f["cls"], f["level"]))
    assert len(seen) == 12


def test_zstd_header_variants(oracle, golden, frames_bin):
    """Checksum flag, no content size (window descriptor), small windows."""
    names = set()
    for f in golden["zstd"]["special"]:
        c = frames_bin[f["off"]:f["off"] + f["csize"]]
        r, out = oracle.zstd_decompress(c, f["size"])
        assert r == f["size"] and sha(out) == f["src_sha"], f["name"]
        names.add(f["name"])
        if "checksum" in f["name"]:  # a flipped checksum byte is rejected
            bad = bytearray(c)
            bad[-1] ^= 1
            assert oracle.zstd_decompress(bytes(bad), f["size"])[0] == -1
    assert {"checksum", "no_fcs", "wlog10", "wlog12"} <= names


def test_zstd_accept_cases(oracle, golden):
    """Multi-frame, skippable, trailing junk, truncation, short dst."""
    for a in golden["zstd"]["accept"]:
        r, out = oracle.zstd_decompress(bytes.fromhex(a["src"]), a["cap"])
        assert r == a["ret"], a
        if r >= 0:
            assert sha(out) == a["out_sha"]


def test_zstd_mutation_corpus(oracle, golden):
    """Accept/reject and output exactly as libzstd 1.4.9.  Error *categories*
    (dstSize_tooSmall / srcSize_wrong / other) match too, except where a
    corrupt sequence stream over-reads: libzstd's bit container then returns
    wrapped-around bits, this restatement returns zeros, and the first error
    hit can differ (both reject)."""
    oracle.zstd_strict_reserved(False)  # 1.4.9 ignores the reserved mode bits
    try:
        cat_diff = 0
        for a in golden["zstd"]["corpus"]:
            r, out = oracle.zstd_decompress(bytes.fromhex(a["src"]), a["cap"])
            assert (r >= 0) == (a["ret"] >= 0), a
            if r >= 0:
                assert r == a["ret"] and sha(out) == a["out_sha"], a
            elif r != a["ret"]:
                cat_diff += 1
        assert cat_diff <= 10, cat_diff
    finally:
        oracle.zstd_strict_reserved(True)


def test_zstd_reserved_bits_rejected(oracle):
    # zstd >= 1.5 (pinned 1.5.6) rejects non-zero reserved bits in the
    # Symbol_Compression_Modes byte; this frame is accepted by 1.4.9 only.
    f = bytes.fromhex("28b52ffd60d0064d00001000000102cbff000b")
    assert oracle.zstd_decompress(f, 2000)[0] == -1
    oracle.zstd_strict_reserved(False)
    try:
        assert oracle.zstd_decompress(f, 2000)[0] == 2000
    finally:
        oracle.zstd_strict_reserved(True)


def test_zstd_frame_content_size(oracle, golden, frames_bin):
    for f in golden["zstd"]["frames"][:20]:
        c = frames_bin[f["off"]:f["off"] + f["csize"]]
        assert oracle.lib.oracle_zstd_frame_content_size(c, len(c)) == f["size"]
