"""Python mirror of JuiceFS's object-encryption data path over libjfsgpu.so,
fused with the codec.

    AES256GCM_RSA / CHACHA20_RSA / SM4GCM          pkg/object/encrypt.go:172-176
    NewDataEncryptor(keyEncryptor, algo)           :178-203 (here: cipher id)
    dataEncryptor.Encrypt / Decrypt                :226-284

The PUT path of an encrypted volume compresses a block (cached_store.go:372)
and then Encrypt()s it into the object envelope; the GET path Decrypt()s and
decompresses (:814).  ``compress_seal_batch`` / ``open_decompress_batch`` do
both steps on the GPU for many blocks at once.  The random data key, the
nonce and the key wrap (RSA / SM2 keyEncryptor, encrypt.go:234) stay with the
caller: seal takes (key, nonce, wrapped_key) per block, open takes the data
key the caller unwrapped from the envelope header (``parse_envelope``).
Results are ``(n, err)`` pairs like compress.py's batch helpers.
"""
from __future__ import annotations

import ctypes

from . import _lib as L
from .compress import CompressError, _addr, _err

AES256GCM_RSA = "aes256gcm-rsa"
CHACHA20_RSA = "chacha20-rsa"
SM4GCM = "sm4gcm"


def cipher_id(algo: str) -> int:
    """NewDataEncryptor's names ("" = AES-256-GCM); raises for an unsupported one."""
    c = L.load().jfs_cipher_from_name(algo.encode())
    if c < 0:
        raise ValueError(f"unsupport cipher: {algo}")
    return c


def key_size(algo: str) -> int:
    return L.load().jfs_cipher_key_size(cipher_id(algo))


def envelope_bound(codec: int, n: int, wrapped_len: int) -> int:
    return int(L.load().jfs_envelope_bound(codec, n, wrapped_len))


def parse_envelope(env: bytes):
    """(wrapped key, nonce, payload offset); raises CompressError like Decrypt's header checks."""
    i64 = ctypes.c_int64
    wo, wl, no, nl = i64(), i64(), i64(), i64()
    a, n, keep = _addr(env, False)
    r = int(L.load().jfs_envelope_parse(a, n, ctypes.byref(wo), ctypes.byref(wl), ctypes.byref(no), ctypes.byref(nl)))
    if r < 0:
        raise CompressError("malformed ciphertext", r)
    return bytes(env[wo.value:wo.value + wl.value]), bytes(env[no.value:no.value + nl.value]), r


def _err_of(code: int, dst_len: int, src_len: int, op: str) -> CompressError:
    if code == L.JFS_ERR_AUTH:
        return CompressError("cipher: message authentication failed", code)
    return _err(code, dst_len, src_len, op)


NONCE_SIZE = 12  # encrypt.go:239: aead.NonceSize() of all three ciphers


def _check_keys(algo: str, keys, nonces) -> None:
    """The C ABI reads jfs_cipher_key_size() key bytes and 12 nonce bytes per
    block through plain pointers; a shorter buffer would be read past its end.
    dataEncryptor.aead (encrypt.go:182-202, used at :235, :276) refuses a wrong key size with an
    error, and so does this, before anything reaches the library."""
    ks = key_size(algo)
    for i, k in enumerate(keys):
        if len(k) != ks:
            raise ValueError(f"block {i}: {algo or 'aes256gcm-rsa'} needs a {ks}-byte key, got {len(k)}")
    for i, n in enumerate(nonces or ()):
        if len(n) != NONCE_SIZE:
            raise ValueError(f"block {i}: nonce must be {NONCE_SIZE} bytes, got {len(n)}")


def compress_seal_batch(codec: int, algo: str, pairs, params, device_mask: int = 0, crcs: list | None = None):
    """pairs: [(dst, raw block)], params: [(key, nonce, wrapped_key)] -> [(envelope bytes, err)];
    with crcs=[], it receives each envelope's CRC-32C (generateChecksum)."""
    lib = L.load()
    nb = len(pairs)
    _check_keys(algo, [p[0] for p in params], [p[1] for p in params])
    iov = (L.JfsIov * max(nb, 1))()
    sp = (L.JfsSealParam * max(nb, 1))()
    keep = []
    for i, ((dst, src), (key, nonce, wrapped)) in enumerate(zip(pairs, params)):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        kk, _, k1 = _addr(key, False)
        nn, _, k2 = _addr(nonce, False)
        ww, wn, k3 = _addr(wrapped, False)
        keep.append((kd, ks, k1, k2, k3))
        iov[i].src, iov[i].src_len, iov[i].dst, iov[i].dst_cap = s, sn, d, dn
        sp[i].key, sp[i].nonce, sp[i].wrapped, sp[i].wrapped_len = kk, nn, ww, wn
    out = (ctypes.c_int64 * max(nb, 1))()
    crc = (ctypes.c_uint32 * max(nb, 1))() if crcs is not None else None
    rc = lib.jfs_compress_seal_batch(codec, cipher_id(algo), nb, iov, sp, out, crc, device_mask)
    if rc != 0:
        raise _err_of(rc, 0, 0, "seal batch")
    if crcs is not None:
        crcs[:] = [int(crc[i]) for i in range(nb)]
    return [(int(out[i]), None) if out[i] >= 0 else
            (0, _err_of(int(out[i]), iov[i].dst_cap, iov[i].src_len, "compress+seal")) for i in range(nb)]


def open_decompress_batch(codec: int, algo: str, pairs, keys, device_mask: int = 0):
    """pairs: [(dst, envelope)], keys: [data key] -> [(n, err)] (n as jfs_decompress returns it)"""
    lib = L.load()
    nb = len(pairs)
    _check_keys(algo, keys, None)
    iov = (L.JfsIov * max(nb, 1))()
    kp = (ctypes.c_void_p * max(nb, 1))()
    keep = []
    for i, ((dst, src), key) in enumerate(zip(pairs, keys)):
        d, dn, kd = _addr(dst, True)
        s, sn, ks = _addr(src, False)
        kk, _, k1 = _addr(key, False)
        keep.append((kd, ks, k1))
        iov[i].src, iov[i].src_len, iov[i].dst, iov[i].dst_cap = s, sn, d, dn
        kp[i] = kk.value if isinstance(kk, ctypes.c_void_p) else kk
    out = (ctypes.c_int64 * max(nb, 1))()
    rc = lib.jfs_open_decompress_batch(codec, cipher_id(algo), nb, iov, kp, out, device_mask)
    if rc != 0:
        raise _err_of(rc, 0, 0, "open batch")
    res = []
    for i in range(nb):
        r = int(out[i])
        if r < 0:
            n = r if (codec == L.ALGO_LZ4 and r > L.JFS_ERR_BASE) else 0
            res.append((n, _err_of(r, iov[i].dst_cap, iov[i].src_len, "open+decompress")))
        else:
            res.append((r, None))
    return res
