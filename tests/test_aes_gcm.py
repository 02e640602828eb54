"""AES-256-GCM: the oracle pinned on CPU by the GCM
specification's AES-256 test cases and by OpenSSL's EVP AES-256-GCM; the HIP
kernels (jfs_aes256gcm_{seal,open}_device) bit-exact against the oracle on GPU.

Reference: pkg/object/encrypt.go:178-189 (aes.NewCipher + cipher.NewGCM),
:226-257 Encrypt (aead.Seal, no additional data), :259-284 Decrypt (aead.Open)."""
import ctypes
import ctypes.util
import os
import random

import numpy as np
import pytest

from juicefs_amd.blockgen import gen_block

# The GCM specification (McGrew & Viega), AES-256 test cases without AAD.
SPEC = [
    ("00" * 32, "00" * 12, "", "", "530f8afbc74536b9a963b4f1c4cb738b"),
    ("00" * 32, "00" * 12, "00" * 16, "cea7403d4d606b6e074ec5d3baf39d18", "d0d1c8a799996bf0265b98b5d48ab919"),
    ("feffe9928665731c6d6a8f9467308308feffe9928665731c6d6a8f9467308308", "cafebabefacedbaddecaf888",
     "d9313225f88406e5a55909c5aff5269a86a7a9531534f7da2e4c303d8a318a72"
     "1c3c0c95956809532fcf0e2449a6b525b16aedf5aa0de657ba637b391aafd255",
     "522dc1f099567d07f47f37a32a84427d643a8cdcbfe5c0c97598a2bd2555d1aa"
     "8cb08e48590dbb3da7b08b1056828838c5f61e6393ba7a0abcc9f662898015ad",
     "b094dac5d93471bdec1a502270e3cc6c"),
]


def _openssl():
    for name in ("libcrypto.so.3", "libcrypto.so.1.1", ctypes.util.find_library("crypto")):
        if not name:
            continue
        try:
            return ctypes.CDLL(name)
        except OSError:
            continue
    return None


def openssl_seal(lib, key, nonce, pt):
    vp = ctypes.c_void_p
    lib.EVP_CIPHER_CTX_new.restype = vp
    lib.EVP_aes_256_gcm.restype = vp
    lib.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]
    lib.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    lib.EVP_EncryptUpdate.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    lib.EVP_EncryptFinal_ex.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    lib.EVP_CIPHER_CTX_free.argtypes = [vp]
    ctx = lib.EVP_CIPHER_CTX_new()
    assert lib.EVP_EncryptInit_ex(ctx, lib.EVP_aes_256_gcm(), None, None, None) == 1
    assert lib.EVP_CIPHER_CTX_ctrl(ctx, 0x9, 12, None) == 1  # EVP_CTRL_GCM_SET_IVLEN
    assert lib.EVP_EncryptInit_ex(ctx, None, None, key, nonce) == 1
    out = ctypes.create_string_buffer(len(pt) + 32)
    n = ctypes.c_int(0)
    assert lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
    n2 = ctypes.c_int(0)
    assert lib.EVP_EncryptFinal_ex(ctx, ctypes.cast(ctypes.addressof(out) + n.value, ctypes.c_char_p),
                                   ctypes.byref(n2)) == 1
    tag = ctypes.create_string_buffer(16)
    assert lib.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, ctypes.cast(tag, vp)) == 1  # EVP_CTRL_GCM_GET_TAG
    lib.EVP_CIPHER_CTX_free(ctx)
    return out.raw[:n.value + n2.value] + tag.raw


def test_oracle_spec_vectors(oracle):
    for k, iv, p, c, t in SPEC:
        k, iv, p = bytes.fromhex(k), bytes.fromhex(iv), bytes.fromhex(p)
        sealed = oracle.aes256gcm_seal(k, iv, p)
        assert sealed.hex() == c + t
        assert oracle.aes256gcm_open(k, iv, sealed) == p


def test_oracle_vs_openssl(oracle):
    lib = _openssl()
    if lib is None:
        pytest.skip("no libcrypto on this host")
    rng = random.Random(5)
    for n in (0, 1, 15, 16, 17, 31, 32, 33, 255, 4096, 4097, 70000):
        key = bytes(rng.randrange(256) for _ in range(32))
        nonce = bytes(rng.randrange(256) for _ in range(12))
        pt = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.aes256gcm_seal(key, nonce, pt) == openssl_seal(lib, key, nonce, pt), n


def test_oracle_open_rejects_tampering(oracle):
    key, nonce = bytes(range(32)), bytes(range(12))
    ct = bytearray(oracle.aes256gcm_seal(key, nonce, b"juicefs block" * 100))
    assert oracle.aes256gcm_open(key, nonce, bytes(ct)) == b"juicefs block" * 100
    for pos in (0, 700, len(ct) - 1):
        bad = bytearray(ct)
        bad[pos] ^= 1
        assert oracle.aes256gcm_open(key, nonce, bytes(bad)) is None
    assert oracle.aes256gcm_open(key, nonce, b"\x00" * 15) is None


def _run(gpu, items, seal, mis=0, raw=False):
    """items: list of (key, nonce, data); returns (ret list, outputs) and, with
    raw=True, also every block's whole dst region."""
    import torch
    from juicefs_amd import device as D
    so, off = [], 0
    for i, (_, _, d) in enumerate(items):
        m = (mis * (i + 1)) % 16 if mis else 0
        so.append(off + m)
        off = (off + m + len(d) + 64 + 15) & ~15
    host = np.zeros(off + 64, dtype=np.uint8)
    for (_, _, d), o in zip(items, so):
        host[o:o + len(d)] = np.frombuffer(d, dtype=np.uint8)
    src = torch.from_numpy(host).to(gpu)
    caps = [len(d) + 16 if seal else max(len(d) - 16, 0) for _, _, d in items]
    do, doff = [], 0
    for i, c in enumerate(caps):
        m = (mis * (i + 3)) % 16 if mis else 0
        do.append(doff + m)
        doff = (doff + m + c + 64 + 15) & ~15
    dst = torch.full((doff + 64,), 0xEE, dtype=torch.uint8, device=gpu)
    kn = np.zeros(64 * len(items), dtype=np.uint8)
    for i, (k, nc, _) in enumerate(items):
        kn[64 * i:64 * i + 32] = np.frombuffer(k, dtype=np.uint8)
        kn[64 * i + 32:64 * i + 44] = np.frombuffer(nc, dtype=np.uint8)
    knt = torch.from_numpy(kn).to(gpu)
    desc = D.make_aead_desc(src, so, [len(d) for _, _, d in items], dst, do, caps, knt,
                            [64 * i for i in range(len(items))], [64 * i + 32 for i in range(len(items))])
    ret = torch.zeros(len(items), dtype=torch.int32, device=gpu)
    D.aes256gcm(desc, ret, seal)
    torch.cuda.synchronize()
    r = ret.cpu().tolist()
    dh = dst.cpu().numpy()
    outs = [dh[o:o + max(x, 0)].tobytes() for o, x in zip(do, r)]
    for o, c in zip(do, caps):  # nothing written past the output
        assert (dh[o + c:o + c + 16] == 0xEE).all()
    if raw:
        return r, outs, [dh[o:o + c].tobytes() for o, c in zip(do, caps)]
    return r, outs


@pytest.mark.gpu
def test_gcm_gpu_vs_oracle(gpu, oracle):
    rng = random.Random(9)
    items = []
    for k, iv, p, _, _ in SPEC:
        items.append((bytes.fromhex(k), bytes.fromhex(iv), bytes.fromhex(p)))
    for n in (1, 15, 16, 17, 255, 4095, 4096, 4097, 65536 + 7, 300000, 1 << 20):
        key = bytes(rng.randrange(256) for _ in range(32))
        nonce = bytes(rng.randrange(256) for _ in range(12))
        items.append((key, nonce, gen_block("TZR"[n % 3], n, n)))
    for mis in (0, 5):
        r, outs = _run(gpu, items, True, mis)
        for (k, nc, d), x, o in zip(items, r, outs):
            want = oracle.aes256gcm_seal(k, nc, d)
            assert x == len(d) + 16 and o == want, (len(d), mis)
        # open what was sealed: plaintext back, ret = len
        sealed = [(k, nc, o) for (k, nc, _), o in zip(items, outs)]
        r2, outs2 = _run(gpu, sealed, False, mis)
        for (_, _, d), x, o in zip(items, r2, outs2):
            assert x == len(d) and o == d


@pytest.mark.gpu
def test_gcm_gpu_open_rejects_tampering(gpu, oracle):
    key, nonce = bytes(range(1, 33)), bytes(range(12))
    pt = gen_block("T", 4, 100000)
    ct = oracle.aes256gcm_seal(key, nonce, pt)
    bad = []
    for pos in (0, 50000, len(ct) - 1):
        b = bytearray(ct)
        b[pos] ^= 0x40
        bad.append((key, nonce, bytes(b)))
    bad.append((bytes(32), nonce, ct))  # wrong key
    r, _, regions = _run(gpu, [(key, nonce, ct)] + bad, False, raw=True)
    assert r[0] == len(pt) and r[1:] == [-1] * len(bad)
    # like Go's gcm.Open, a failed open leaves no plaintext behind: dst is zeroed
    assert regions[0] == pt
    for reg in regions[1:]:
        assert reg == bytes(len(pt))


@pytest.mark.gpu
def test_gcm_gpu_4mib_blocks(gpu, oracle):
    """JuiceFS's object shape: one random key and nonce per 4 MiB (compressed)
    block, many blocks per launch; a sample checked against the oracle."""
    import torch
    from juicefs_amd import device as D
    n, U = 32, 4 << 20
    rng = np.random.default_rng(3)
    raw = torch.empty(n * U, dtype=torch.uint8, device=gpu)
    D.gen_blocks(raw, n, U, "T", 77)
    kn = torch.from_numpy(rng.integers(0, 256, 64 * n, dtype=np.uint8)).to(gpu)
    out = torch.empty(n * (U + 16), dtype=torch.uint8, device=gpu)
    desc = D.make_aead_desc(raw, [i * U for i in range(n)], [U] * n, out, [i * (U + 16) for i in range(n)],
                            [U + 16] * n, kn, [64 * i for i in range(n)], [64 * i + 32 for i in range(n)])
    ret = torch.zeros(n, dtype=torch.int32, device=gpu)
    D.aes256gcm(desc, ret, True)
    torch.cuda.synchronize()
    assert (ret == U + 16).all()
    host, oh, kh = raw.cpu().numpy(), out.cpu().numpy(), kn.cpu().numpy()
    for i in (0, 17, 31):
        want = oracle.aes256gcm_seal(kh[64 * i:64 * i + 32].tobytes(), kh[64 * i + 32:64 * i + 44].tobytes(),
                                     host[i * U:(i + 1) * U].tobytes())
        assert oh[i * (U + 16):(i + 1) * (U + 16)].tobytes() == want, i


@pytest.mark.gpu
def test_fused_compress_seal_and_open_decompress(gpu, oracle):
    """SURVEY.md 8(f)3 fused paths: LZ4 compress -> seal and open -> LZ4
    decompress chained on one stream (lengths passed on the device).  The
    sealed objects equal oracle.seal(oracle.lz4_compress(block)); opening them
    gives the blocks back; a tampered object fails its block only."""
    import torch
    from juicefs_amd import device as D
    rng = np.random.default_rng(8)
    srcs = [gen_block("T", 70 + i, n) for i, n in enumerate((1 << 20, 300000, 4096, (1 << 20) + 7, 65536))]
    srcs.append(gen_block("R", 3, 200000))
    n = len(srcs)
    bound = [len(s) + len(s) // 255 + 16 for s in srcs]
    so = np.cumsum([0] + [(len(s) + 255) // 256 * 256 for s in srcs[:-1]])
    co = np.cumsum([0] + [(b + 255) // 256 * 256 for b in bound[:-1]])
    eo = np.cumsum([0] + [(b + 16 + 255) // 256 * 256 for b in bound[:-1]])
    raw = torch.zeros(int(so[-1]) + len(srcs[-1]) + 256, dtype=torch.uint8, device=gpu)
    for s, o in zip(srcs, so):
        raw[int(o):int(o) + len(s)] = torch.from_numpy(np.frombuffer(s, dtype=np.uint8).copy()).to(gpu)
    comp = torch.zeros(int(co[-1]) + bound[-1] + 256, dtype=torch.uint8, device=gpu)
    sealed = torch.zeros(int(eo[-1]) + bound[-1] + 16 + 256, dtype=torch.uint8, device=gpu)
    kn_h = rng.integers(0, 256, 64 * n, dtype=np.uint8)
    kn = torch.from_numpy(kn_h).to(gpu)
    cdesc = D.make_desc(raw, so, [len(s) for s in srcs], comp, co, bound)
    adesc = D.make_aead_desc(comp, co, [0] * n, sealed, eo, [b + 16 for b in bound], kn,
                             [64 * i for i in range(n)], [64 * i + 32 for i in range(n)])
    rc, rs = torch.zeros(n, dtype=torch.int32, device=gpu), torch.zeros(n, dtype=torch.int32, device=gpu)
    D.lz4_compress_seal(cdesc, adesc, rc, rs)
    torch.cuda.synchronize()
    csz, ssz = rc.cpu().tolist(), rs.cpu().tolist()
    sh = sealed.cpu().numpy()
    objs = []
    for i, s in enumerate(srcs):
        m, ref = oracle.lz4_compress(s)
        assert csz[i] == m and ssz[i] == m + 16
        key, nonce = kn_h[64 * i:64 * i + 32].tobytes(), kn_h[64 * i + 32:64 * i + 44].tobytes()
        obj = sh[int(eo[i]):int(eo[i]) + ssz[i]].tobytes()
        assert obj == oracle.aes256gcm_seal(key, nonce, ref), i
        objs.append(obj)
    # tamper with object 2, then open -> decompress everything
    sealed[int(eo[2]) + 5] ^= 1
    plain = torch.zeros_like(comp)
    out = torch.zeros_like(raw)
    odesc = D.make_aead_desc(sealed, eo, ssz, plain, co, bound, kn, [64 * i for i in range(n)],
                             [64 * i + 32 for i in range(n)])
    ddesc = D.make_desc(plain, co, [0] * n, out, so, [len(s) for s in srcs])
    ro, rd = torch.zeros(n, dtype=torch.int32, device=gpu), torch.zeros(n, dtype=torch.int32, device=gpu)
    D.open_lz4_decompress(odesc, ddesc, ro, rd)
    torch.cuda.synchronize()
    ro_h, rd_h, oh = ro.cpu().tolist(), rd.cpu().tolist(), out.cpu().numpy()
    for i, s in enumerate(srcs):
        if i == 2:
            assert ro_h[i] == -1 and rd_h[i] == D.JFS_CHAIN_FAILED
            continue
        assert ro_h[i] == csz[i] and rd_h[i] == len(s)
        assert oh[int(so[i]):int(so[i]) + len(s)].tobytes() == s, i
