"""The other two data ciphers of JuiceFS object encryption and the object
envelope, CPU part: the oracle (oracle/aead_oracle.c) pinned
by published vectors and by OpenSSL.

  pkg/object/encrypt.go:190      CHACHA20_RSA  chacha20poly1305.New
  pkg/object/encrypt.go:192-201  SM4GCM        sm4.NewCipher + cipher.NewGCM
  pkg/object/encrypt.go:226-257  Encrypt: be16 wrapped-key length, nonce length,
                                 wrapped key, nonce, aead.Seal(.., nil)
  pkg/object/encrypt.go:259-284  Decrypt: header checks, aead.Open

SM4 by the GB/T 32907-2016 example (one block, and the 1,000,000-fold
encryption); ChaCha20 / Poly1305 / the AEAD by RFC 8439 sections 2.3.2, 2.5.2
and 2.8.2; both against OpenSSL 3 (SM4-ECB; ChaCha20-Poly1305) on random
inputs.  SM4-GCM is the GCM of aes_gcm_oracle.c (pinned by the GCM spec
vectors) over the pinned SM4 block."""
import ctypes
import ctypes.util
import random

import pytest

from tests.test_aes_gcm import _openssl

RFC_PT = (b"Ladies and Gentlemen of the class of '99: If I could offer you only one tip for the future, "
          b"sunscreen would be it.")


def _evp(lib, cipher_name, key, iv, pt, aead_tag=False, aad=b""):
    vp = ctypes.c_void_p
    lib.EVP_CIPHER_fetch.restype = vp
    lib.EVP_CIPHER_fetch.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p]
    lib.EVP_CIPHER_CTX_new.restype = vp
    lib.EVP_EncryptInit_ex.argtypes = [vp, vp, vp, ctypes.c_char_p, ctypes.c_char_p]
    lib.EVP_CIPHER_CTX_ctrl.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
    lib.EVP_CIPHER_CTX_set_padding.argtypes = [vp, ctypes.c_int]
    lib.EVP_EncryptUpdate.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p, ctypes.c_int]
    lib.EVP_EncryptFinal_ex.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int)]
    lib.EVP_CIPHER_CTX_free.argtypes = [vp]
    ciph = lib.EVP_CIPHER_fetch(None, cipher_name, None)
    if not ciph:
        pytest.skip(f"OpenSSL has no {cipher_name!r}")
    ctx = lib.EVP_CIPHER_CTX_new()
    assert lib.EVP_EncryptInit_ex(ctx, ciph, None, key, iv) == 1
    lib.EVP_CIPHER_CTX_set_padding(ctx, 0)
    n = ctypes.c_int(0)
    if aad:
        assert lib.EVP_EncryptUpdate(ctx, None, ctypes.byref(n), aad, len(aad)) == 1
    out = ctypes.create_string_buffer(len(pt) + 32)
    assert lib.EVP_EncryptUpdate(ctx, out, ctypes.byref(n), pt, len(pt)) == 1
    n2 = ctypes.c_int(0)
    assert lib.EVP_EncryptFinal_ex(ctx, ctypes.cast(ctypes.addressof(out) + n.value, ctypes.c_char_p),
                                   ctypes.byref(n2)) == 1
    res = out.raw[:n.value + n2.value]
    if aead_tag:
        tag = ctypes.create_string_buffer(16)
        assert lib.EVP_CIPHER_CTX_ctrl(ctx, 0x10, 16, ctypes.cast(tag, vp)) == 1  # EVP_CTRL_AEAD_GET_TAG
        res += tag.raw
    lib.EVP_CIPHER_CTX_free(ctx)
    return res


def test_sm4_gbt32907_example(oracle):
    k = bytes.fromhex("0123456789abcdeffedcba9876543210")
    assert oracle.sm4_block(k, k).hex() == "681edf34d206965e86b3e94f536e4246"


def test_sm4_gbt32907_million_encryptions(oracle):
    k = bytes.fromhex("0123456789abcdeffedcba9876543210")
    x = k
    for _ in range(1000000):
        x = oracle.sm4_block(k, x)
    assert x.hex() == "595298c7c6fd271f0402f804c33d3f66"


def test_sm4_vs_openssl(oracle):
    lib = _openssl()
    if lib is None:
        pytest.skip("no libcrypto")
    rng = random.Random(11)
    for _ in range(64):
        k = bytes(rng.randrange(256) for _ in range(16))
        blk = bytes(rng.randrange(256) for _ in range(16))
        assert oracle.sm4_block(k, blk) == _evp(lib, b"SM4-ECB", k, None, blk)


def test_sm4gcm_roundtrip_and_tamper(oracle):
    rng = random.Random(3)
    for n in (0, 1, 15, 16, 17, 100, 4096, 70001):
        k = bytes(rng.randrange(256) for _ in range(16))
        iv = bytes(rng.randrange(256) for _ in range(12))
        pt = bytes(rng.randrange(256) for _ in range(n))
        ct = oracle.seal("sm4gcm", k, iv, pt)
        assert len(ct) == n + 16 and oracle.open("sm4gcm", k, iv, ct) == pt
        bad = bytearray(ct)
        bad[rng.randrange(len(bad))] ^= 4
        assert oracle.open("sm4gcm", k, iv, bytes(bad)) is None


def test_chacha20_block_rfc8439_2_3_2(oracle):
    key = bytes(range(32))
    nonce = bytes.fromhex("000000090000004a00000000")
    assert oracle.chacha20_block(key, 1, nonce).hex() == (
        "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
        "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


def test_poly1305_rfc8439_2_5_2(oracle):
    key = bytes.fromhex("85d6be7857556d337f4452fe42d506a80103808afb0db2fd4abff6af4149f51b")
    assert oracle.poly1305(key, b"Cryptographic Forum Research Group").hex() == "a8061dc1305136c6c22b8baf0c0127a9"


def test_chacha20poly1305_aead_rfc8439_2_8_2(oracle):
    key = bytes(range(0x80, 0xa0))
    nonce = bytes.fromhex("070000004041424344454647")
    aad = bytes.fromhex("50515253c0c1c2c3c4c5c6c7")
    sealed = oracle.seal("chacha20", key, nonce, RFC_PT, aad)
    assert sealed[:16].hex() == "d31a8d34648e60db7b86afbc53ef7ec2"
    assert sealed[-16:].hex() == "1ae10b594f09e26a7e902ecbd0600691"
    assert oracle.open("chacha20", key, nonce, sealed, aad) == RFC_PT


def test_chacha20poly1305_vs_openssl(oracle):
    lib = _openssl()
    if lib is None:
        pytest.skip("no libcrypto")
    rng = random.Random(8)
    for n in (0, 1, 15, 16, 17, 63, 64, 65, 1000, 70000):
        k = bytes(rng.randrange(256) for _ in range(32))
        iv = bytes(rng.randrange(256) for _ in range(12))
        pt = bytes(rng.randrange(256) for _ in range(n))
        assert oracle.seal("chacha20", k, iv, pt) == _evp(lib, b"ChaCha20-Poly1305", k, iv, pt, aead_tag=True), n
        ct = oracle.seal("chacha20", k, iv, pt)
        assert oracle.open("chacha20", k, iv, ct) == pt
        bad = bytearray(ct)
        bad[-1] ^= 1
        assert oracle.open("chacha20", k, iv, bytes(bad)) is None


def test_envelope_layout(oracle):
    """encrypt.go:244-254: be16(len(cipherkey)) || u8(len(nonce)) || cipherkey ||
    nonce || sealed; Decrypt's checks (:260-267)."""
    wrapped = bytes(range(256)) + b"\x01" * 44  # e.g. a 2048-bit RSA-OAEP key wrap: 256 bytes; here 300
    nonce = bytes(range(12))
    sealed = b"\xaa" * 50
    env = oracle.envelope(wrapped, nonce, sealed)
    assert env[:3] == bytes([300 >> 8, 300 & 255, 12]) and env[3:303] == wrapped and env[303:315] == nonce
    assert env[315:] == sealed
    assert oracle.envelope_parse(env) == (315, 300, 12)
    assert oracle.envelope_parse(env[:2])[0] == -1               # "length is less than 3"
    assert oracle.envelope_parse(env[:315])[0] == -2             # "malformed ciphertext": 3+k+n >= len
