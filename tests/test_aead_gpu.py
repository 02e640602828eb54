"""GPU: the three data ciphers of NewDataEncryptor (pkg/object/encrypt.go:176-202)
through jfs_aead_{seal,open}_device, bit-exact against the pinned oracle
(oracle/aes_gcm_oracle.c, oracle/aead_oracle.c): ciphertext || tag on seal,
plaintext and length on open, -1 and a zeroed output on any tampering (Go's
Open clears its output), every size class and misaligned buffers."""
import random

import numpy as np
import pytest
import torch

from juicefs_amd import device as D
from juicefs_amd.blockgen import gen_block

pytestmark = pytest.mark.gpu
KEYLEN = {"aes256gcm": 32, "chacha20": 32, "sm4gcm": 16}


def _run(gpu, cipher, items, seal, mis=0):
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
        kn[64 * i:64 * i + len(k)] = np.frombuffer(k, dtype=np.uint8)
        kn[64 * i + 32:64 * i + 44] = np.frombuffer(nc, dtype=np.uint8)
    knt = torch.from_numpy(kn).to(gpu)
    desc = D.make_aead_desc(src, so, [len(d) for _, _, d in items], dst, do, caps, knt,
                            [64 * i for i in range(len(items))], [64 * i + 32 for i in range(len(items))])
    ret = torch.zeros(len(items), dtype=torch.int32, device=gpu)
    D.aead(cipher, desc, ret, seal)
    torch.cuda.synchronize()
    r = ret.cpu().tolist()
    dh = dst.cpu().numpy()
    for o, c in zip(do, caps):  # nothing written past the output
        assert (dh[o + c:o + c + 16] == 0xEE).all()
    return r, [dh[o:o + c].tobytes() for o, c in zip(do, caps)]


@pytest.mark.parametrize("cipher", ["chacha20", "sm4gcm", "aes256gcm"])
def test_aead_gpu_vs_oracle(gpu, oracle, cipher):
    rng = random.Random(21)
    items = []
    for n in (0, 1, 15, 16, 17, 63, 64, 65, 255, 4095, 4096, 4097, 16383, 16384, 16385, 65536 + 7, 300000, 1 << 20):
        key = bytes(rng.randrange(256) for _ in range(KEYLEN[cipher]))
        nonce = bytes(rng.randrange(256) for _ in range(12))
        items.append((key, nonce, gen_block("TZR"[n % 3], n, n)))
    for mis in (0, 5):
        r, outs = _run(gpu, cipher, items, True, mis)
        for (k, nc, d), x, o in zip(items, r, outs):
            assert x == len(d) + 16 and o == oracle.seal(cipher, k, nc, d), (cipher, len(d), mis)
        sealed = [(k, nc, o) for (k, nc, _), o in zip(items, outs)]
        r2, outs2 = _run(gpu, cipher, sealed, False, mis)
        for (_, _, d), x, o in zip(items, r2, outs2):
            assert x == len(d) and o == d


@pytest.mark.parametrize("cipher", ["chacha20", "sm4gcm"])
def test_aead_gpu_open_rejects_tampering_and_clears(gpu, oracle, cipher):
    key, nonce = bytes(range(1, 1 + KEYLEN[cipher])), bytes(range(12))
    pt = gen_block("T", 4, 100000)
    ct = oracle.seal(cipher, key, nonce, pt)
    bad = []
    for pos in (0, 50000, len(ct) - 17, len(ct) - 1):
        b = bytearray(ct)
        b[pos] ^= 0x40
        bad.append((key, nonce, bytes(b)))
    bad.append((bytes(len(key)), nonce, ct))  # wrong key
    r, outs = _run(gpu, cipher, [(key, nonce, ct)] + bad, False)
    assert r[0] == len(pt) and outs[0] == pt
    assert r[1:] == [-1] * len(bad)
    assert all(o == bytes(len(pt)) for o in outs[1:])


@pytest.mark.parametrize("cipher", ["chacha20", "sm4gcm"])
def test_aead_gpu_4mib_objects(gpu, oracle, cipher):
    """JuiceFS's object shape: one random key and nonce per compressed 4 MiB block."""
    rng = random.Random(5)
    items = [(bytes(rng.randrange(256) for _ in range(KEYLEN[cipher])), bytes(rng.randrange(256) for _ in range(12)),
              gen_block("T", 700 + i, (4 << 20) - 977 * i)) for i in range(6)]
    r, outs = _run(gpu, cipher, items, True)
    for (k, nc, d), x, o in zip(items, r, outs):
        assert x == len(d) + 16 and o == oracle.seal(cipher, k, nc, d)
