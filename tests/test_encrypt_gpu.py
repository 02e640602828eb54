"""GPU: the encrypted-object paths through the host batch ABI.

PUT = Compress (pkg/chunk/cached_store.go:372) then dataEncryptor.Encrypt
(pkg/object/encrypt.go:226-257); GET = Decrypt (:259-284) then Decompress
(cached_store.go:814).  jfs_compress_seal_batch must write exactly
Encrypt(Compress(block)): the envelope header (be16 wrapped-key length,
nonce length, wrapped key, nonce) and aead.Seal of the compressed bytes --
checked byte for byte against the CPU oracles (the LZ4 encoder is
byte-exact; Zstd frames are compared with the library's own Zstd encoder,
the ciphers with oracle/aead_oracle.c).  jfs_open_decompress_batch must give
the block back, JFS_ERR_AUTH on any tampering and JFS_ERR_CORRUPT for a
malformed header, per block."""
import random

import pytest

from juicefs_amd import _lib as L
from juicefs_amd import compress as C
from juicefs_amd import encrypt as E
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu
CIPHERS = {E.AES256GCM_RSA: "aes256gcm", E.CHACHA20_RSA: "chacha20", E.SM4GCM: "sm4gcm"}
CODECS = {"none": L.ALGO_NONE, "lz4": L.ALGO_LZ4, "zstd": L.ALGO_ZSTD}


def _blocks():
    sizes = [1, 100, 4096, 65536 + 11, 300000, 1 << 20, 4 << 20]
    return [gen_block("TZR"[i % 3] if i < 5 else "T", 800 + i, n) for i, n in enumerate(sizes)]


def _compressed(codec, raw):
    if codec == "none":
        return raw
    c = C.NewCompressor(codec)
    d = bytearray(c.CompressBound(len(raw)))
    n, e = c.Compress(d, raw)
    assert e is None
    return bytes(d[:n])


@pytest.mark.parametrize("algo", list(CIPHERS))
@pytest.mark.parametrize("codec", list(CODECS))
def test_compress_seal_then_open_decompress(gpu, oracle, algo, codec):
    rng = random.Random(hash((algo, codec)) & 0xFFFF)
    raws = _blocks()
    klen = E.key_size(algo)
    params = []
    for i in range(len(raws)):
        key = bytes(rng.randrange(256) for _ in range(klen))
        nonce = bytes(rng.randrange(256) for _ in range(12))
        wrapped = bytes(rng.randrange(256) for _ in range(256 + 7 * i))  # stands in for the RSA-wrapped key
        params.append((key, nonce, wrapped))
    pairs = [(bytearray(E.envelope_bound(CODECS[codec], len(r), len(p[2]))), r) for r, p in zip(raws, params)]
    res = E.compress_seal_batch(CODECS[codec], algo, pairs, params)
    envs = []
    for (dst, raw), (key, nonce, wrapped), (n, err) in zip(pairs, params, res):
        assert err is None, err
        comp = _compressed(codec, raw)
        want = oracle.envelope(wrapped, nonce, oracle.seal(CIPHERS[algo], key, nonce, comp))
        assert n == len(want) and bytes(dst[:n]) == want, (algo, codec, len(raw))
        envs.append(bytes(dst[:n]))
        w2, n2, off = E.parse_envelope(envs[-1])
        assert (w2, n2, off) == (wrapped, nonce, 3 + len(wrapped) + 12)
    # GET: open + decompress, then tampered / malformed objects next to good ones
    keys = [p[0] for p in params]
    outs = [bytearray(len(r)) for r in raws]
    back = E.open_decompress_batch(CODECS[codec], algo, list(zip(outs, envs)), keys)
    for o, raw, (n, err) in zip(outs, raws, back):
        assert err is None and n == len(raw) and bytes(o) == raw
    bad_env = bytearray(envs[3])
    bad_env[len(bad_env) // 2 + 200] ^= 1  # a payload byte
    bad_tag = bytearray(envs[2])
    bad_tag[-1] ^= 0x80
    trial = [(bytearray(len(raws[3])), bytes(bad_env)), (bytearray(len(raws[2])), bytes(bad_tag)),
             (bytearray(len(raws[4])), envs[4]), (bytearray(10), b"\x00\x01"),
             (bytearray(len(raws[1])), envs[1][:3 + 256 + 7 + 12])]
    tkeys = [keys[3], keys[2], keys[4], keys[0], keys[1]]
    tr = E.open_decompress_batch(CODECS[codec], algo, trial, tkeys)
    assert tr[0][1].code == L.JFS_ERR_AUTH and tr[1][1].code == L.JFS_ERR_AUTH
    assert tr[2][1] is None and bytes(trial[2][0]) == raws[4]
    assert tr[3][1].code == L.JFS_ERR_CORRUPT and tr[4][1].code == L.JFS_ERR_CORRUPT
    # a wrong key
    wk = E.open_decompress_batch(CODECS[codec], algo, [(bytearray(len(raws[5])), envs[5])], [bytes(klen)])
    assert wk[0][1].code == L.JFS_ERR_AUTH


def test_seal_short_dst_and_bad_cipher(gpu):
    raw = gen_block("T", 1, 5000)
    p = (bytes(32), bytes(12), b"w" * 10)
    bound = E.envelope_bound(L.ALGO_LZ4, len(raw), 10)
    r = E.compress_seal_batch(L.ALGO_LZ4, E.AES256GCM_RSA, [(bytearray(bound - 1), raw)], [p])
    assert r[0][1].code == L.JFS_ERR_SHORT_BUFFER
    with pytest.raises(ValueError):
        E.cipher_id("rot13")


@pytest.mark.parametrize("codec", ["lz4", "zstd"])
def test_put_payload_checksums(gpu, oracle, codec):
    """generateChecksum (pkg/object/checksum.go:30-45) of what is PUT: the
    compressed block (jfs_compress_batch_crc) or the whole envelope
    (jfs_compress_seal_batch), computed on the GPU; CRC-32C oracle pinned by
    RFC 3720."""
    raws = _blocks()
    c = C.NewCompressor(codec)
    pairs = [(bytearray(c.CompressBound(len(r))), r) for r in raws]
    res = c.CompressBatchChecksum(pairs)
    for (d, _), (n, e, crc) in zip(pairs, res):
        assert e is None and crc == oracle.crc32c(bytes(d[:n]))
    params = [(bytes(range(32)), bytes(range(12)), b"k" * (100 + i)) for i in range(len(raws))]
    spairs = [(bytearray(E.envelope_bound(CODECS[codec], len(r), 100 + i)), r) for i, r in enumerate(raws)]
    crcs = []
    sres = E.compress_seal_batch(CODECS[codec], E.CHACHA20_RSA, spairs, params, crcs=crcs)
    for (d, _), (n, e), crc in zip(spairs, sres, crcs):
        assert e is None and crc == oracle.crc32c(bytes(d[:n]))
