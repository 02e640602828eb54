/*
 * CPU oracle (TEST INFRASTRUCTURE ONLY -- never linked into libjfsgpu.so):
 * AES-256-GCM as JuiceFS's object encryption applies it.
 *
 *   pkg/object/encrypt.go:178-189   AES256GCM_RSA: aes.NewCipher(key) + cipher.NewGCM(block)
 *                                   (12-byte nonce, 16-byte tag)
 *   pkg/object/encrypt.go:226-257   Encrypt: random 32-byte key and nonce per object;
 *                                   aead.Seal(p[:0], nonce, plaintext, nil) -- no
 *                                   additional data; output = ciphertext || tag
 *   pkg/object/encrypt.go:259-284   Decrypt: aead.Open(...), error on a bad tag
 *
 * Restated from FIPS-197 (AES, byte-oriented: SubBytes / ShiftRows /
 * MixColumns / AddRoundKey, 14 rounds, AES-256 key expansion) and NIST
 * SP 800-38D (GCM: J0 = nonce || 0^31 1, CTR from inc32(J0), GHASH with the
 * bit-at-a-time multiply of Algorithm 1).  Pinned in tests/test_aes_gcm.py by
 * the GCM specification's AES-256 test cases and by OpenSSL's EVP AES-256-GCM
 * (libcrypto, loaded with ctypes) on random inputs.
 */
#include <stdint.h>
#include <string.h>

static const uint8_t SBOX[256] = {
    0x63, 0x7c, 0x77, 0x7b, 0xf2, 0x6b, 0x6f, 0xc5, 0x30, 0x01, 0x67, 0x2b, 0xfe, 0xd7, 0xab, 0x76, 0xca, 0x82, 0xc9,
    0x7d, 0xfa, 0x59, 0x47, 0xf0, 0xad, 0xd4, 0xa2, 0xaf, 0x9c, 0xa4, 0x72, 0xc0, 0xb7, 0xfd, 0x93, 0x26, 0x36, 0x3f,
    0xf7, 0xcc, 0x34, 0xa5, 0xe5, 0xf1, 0x71, 0xd8, 0x31, 0x15, 0x04, 0xc7, 0x23, 0xc3, 0x18, 0x96, 0x05, 0x9a, 0x07,
    0x12, 0x80, 0xe2, 0xeb, 0x27, 0xb2, 0x75, 0x09, 0x83, 0x2c, 0x1a, 0x1b, 0x6e, 0x5a, 0xa0, 0x52, 0x3b, 0xd6, 0xb3,
    0x29, 0xe3, 0x2f, 0x84, 0x53, 0xd1, 0x00, 0xed, 0x20, 0xfc, 0xb1, 0x5b, 0x6a, 0xcb, 0xbe, 0x39, 0x4a, 0x4c, 0x58,
    0xcf, 0xd0, 0xef, 0xaa, 0xfb, 0x43, 0x4d, 0x33, 0x85, 0x45, 0xf9, 0x02, 0x7f, 0x50, 0x3c, 0x9f, 0xa8, 0x51, 0xa3,
    0x40, 0x8f, 0x92, 0x9d, 0x38, 0xf5, 0xbc, 0xb6, 0xda, 0x21, 0x10, 0xff, 0xf3, 0xd2, 0xcd, 0x0c, 0x13, 0xec, 0x5f,
    0x97, 0x44, 0x17, 0xc4, 0xa7, 0x7e, 0x3d, 0x64, 0x5d, 0x19, 0x73, 0x60, 0x81, 0x4f, 0xdc, 0x22, 0x2a, 0x90, 0x88,
    0x46, 0xee, 0xb8, 0x14, 0xde, 0x5e, 0x0b, 0xdb, 0xe0, 0x32, 0x3a, 0x0a, 0x49, 0x06, 0x24, 0x5c, 0xc2, 0xd3, 0xac,
    0x62, 0x91, 0x95, 0xe4, 0x79, 0xe7, 0xc8, 0x37, 0x6d, 0x8d, 0xd5, 0x4e, 0xa9, 0x6c, 0x56, 0xf4, 0xea, 0x65, 0x7a,
    0xae, 0x08, 0xba, 0x78, 0x25, 0x2e, 0x1c, 0xa6, 0xb4, 0xc6, 0xe8, 0xdd, 0x74, 0x1f, 0x4b, 0xbd, 0x8b, 0x8a, 0x70,
    0x3e, 0xb5, 0x66, 0x48, 0x03, 0xf6, 0x0e, 0x61, 0x35, 0x57, 0xb9, 0x86, 0xc1, 0x1d, 0x9e, 0xe1, 0xf8, 0x98, 0x11,
    0x69, 0xd9, 0x8e, 0x94, 0x9b, 0x1e, 0x87, 0xe9, 0xce, 0x55, 0x28, 0xdf, 0x8c, 0xa1, 0x89, 0x0d, 0xbf, 0xe6, 0x42,
    0x68, 0x41, 0x99, 0x2d, 0x0f, 0xb0, 0x54, 0xbb, 0x16};

static uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

/* AES-256 key expansion: 15 round keys of 16 bytes (FIPS-197 5.2, Nk = 8) */
static void expand(const uint8_t key[32], uint8_t rk[240]) {
    memcpy(rk, key, 32);
    uint8_t rc = 1;
    for (int i = 8; i < 60; i++) {
        uint8_t t[4];
        memcpy(t, rk + 4 * (i - 1), 4);
        if (i % 8 == 0) {
            uint8_t r = t[0];
            t[0] = (uint8_t)(SBOX[t[1]] ^ rc);
            t[1] = SBOX[t[2]];
            t[2] = SBOX[t[3]];
            t[3] = SBOX[r];
            rc = xtime(rc);
        } else if (i % 8 == 4) {
            for (int k = 0; k < 4; k++) t[k] = SBOX[t[k]];
        }
        for (int k = 0; k < 4; k++) rk[4 * i + k] = rk[4 * (i - 8) + k] ^ t[k];
    }
}

/* one block (FIPS-197 5.1; state column-major: s[4c + r]) */
static void encrypt_block(const uint8_t rk[240], const uint8_t in[16], uint8_t out[16]) {
    uint8_t s[16];
    for (int i = 0; i < 16; i++) s[i] = in[i] ^ rk[i];
    for (int round = 1; round <= 14; round++) {
        uint8_t t[16];
        for (int i = 0; i < 16; i++) t[i] = SBOX[s[i]];
        /* ShiftRows: row r rotates left by r */
        for (int c = 0; c < 4; c++)
            for (int r = 0; r < 4; r++) s[4 * c + r] = t[4 * ((c + r) % 4) + r];
        if (round < 14) { /* MixColumns */
            for (int c = 0; c < 4; c++) {
                uint8_t a0 = s[4 * c], a1 = s[4 * c + 1], a2 = s[4 * c + 2], a3 = s[4 * c + 3];
                uint8_t all = a0 ^ a1 ^ a2 ^ a3;
                s[4 * c] ^= all ^ xtime(a0 ^ a1);
                s[4 * c + 1] ^= all ^ xtime(a1 ^ a2);
                s[4 * c + 2] ^= all ^ xtime(a2 ^ a3);
                s[4 * c + 3] ^= all ^ xtime(a3 ^ a0);
            }
        }
        for (int i = 0; i < 16; i++) s[i] ^= rk[16 * round + i];
    }
    memcpy(out, s, 16);
}

/* X * Y in GF(2^128), SP 800-38D Algorithm 1 (bit 0 = MSB of byte 0) */
static void gf_mul(const uint8_t X[16], const uint8_t Y[16], uint8_t Z[16]) {
    uint8_t V[16], R[16];
    memset(R, 0, 16);
    memcpy(V, Y, 16);
    for (int i = 0; i < 128; i++) {
        if (X[i / 8] & (0x80 >> (i % 8)))
            for (int k = 0; k < 16; k++) R[k] ^= V[k];
        int lsb = V[15] & 1;
        for (int k = 15; k > 0; k--) V[k] = (uint8_t)((V[k] >> 1) | (V[k - 1] << 7));
        V[0] >>= 1;
        if (lsb) V[0] ^= 0xE1;
    }
    memcpy(Z, R, 16);
}

static void ghash_block(uint8_t Y[16], const uint8_t H[16], const uint8_t *blk, int len) {
    for (int k = 0; k < len; k++) Y[k] ^= blk[k];
    gf_mul(Y, H, Y);
}

/* CTR keystream xor + GHASH over the ciphertext; tag into tag[16] */
static void gcm(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *in, int64_t n, uint8_t *out,
                int decrypt, uint8_t tag[16]) {
    uint8_t rk[240], H[16], J0[16], ctr[16], ks[16], Y[16];
    expand(key, rk);
    memset(H, 0, 16);
    encrypt_block(rk, H, H);
    memcpy(J0, nonce, 12);
    J0[12] = J0[13] = J0[14] = 0;
    J0[15] = 1;
    memset(Y, 0, 16);
    uint32_t c = 2;
    for (int64_t o = 0; o < n; o += 16, c++) {
        int len = n - o < 16 ? (int)(n - o) : 16;
        memcpy(ctr, nonce, 12);
        ctr[12] = (uint8_t)(c >> 24);
        ctr[13] = (uint8_t)(c >> 16);
        ctr[14] = (uint8_t)(c >> 8);
        ctr[15] = (uint8_t)c;
        encrypt_block(rk, ctr, ks);
        if (decrypt) ghash_block(Y, H, in + o, len);
        for (int k = 0; k < len; k++) out[o + k] = in[o + k] ^ ks[k];
        if (!decrypt) ghash_block(Y, H, out + o, len);
    }
    uint8_t L[16];
    memset(L, 0, 16);
    uint64_t bits = (uint64_t)n * 8; /* len(A) = 0 */
    for (int k = 0; k < 8; k++) L[15 - k] = (uint8_t)(bits >> (8 * k));
    ghash_block(Y, H, L, 16);
    encrypt_block(rk, J0, ks);
    for (int k = 0; k < 16; k++) tag[k] = ks[k] ^ Y[k];
}

/* aead.Seal: dst receives n + 16 bytes (ciphertext || tag) */
int64_t oracle_aes256gcm_seal(const uint8_t *key, const uint8_t *nonce, const uint8_t *src, int64_t n, uint8_t *dst) {
    gcm(key, nonce, src, n, dst, 0, dst + n);
    return n + 16;
}

/* aead.Open: src = ciphertext || tag (n >= 16); dst receives n - 16 bytes;
 * returns n - 16, or -1 when the tag does not verify */
int64_t oracle_aes256gcm_open(const uint8_t *key, const uint8_t *nonce, const uint8_t *src, int64_t n, uint8_t *dst) {
    if (n < 16) return -1;
    uint8_t tag[16];
    gcm(key, nonce, src, n - 16, dst, 1, tag);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= (uint8_t)(tag[k] ^ src[n - 16 + k]);
    return d ? -1 : n - 16;
}
