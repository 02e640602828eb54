/*
 * CPU oracle (TEST INFRASTRUCTURE ONLY -- never linked into libjfsgpu.so):
 * the other two data ciphers of JuiceFS's object encryption and the object
 * envelope.
 *
 *   pkg/object/encrypt.go:190   CHACHA20_RSA: chacha20poly1305.New (32-byte key,
 *                               12-byte nonce, 16-byte tag)
 *   pkg/object/encrypt.go:192-201 SM4GCM: sm4.NewCipher(key) + cipher.NewGCM
 *                               (16-byte key, 12-byte nonce, 16-byte tag)
 *   pkg/object/encrypt.go:226-257 Encrypt: header = be16(len(wrapped key)) ||
 *                               u8(len(nonce)) || wrapped key || nonce, then
 *                               aead.Seal(..., nonce, plaintext, nil)
 *   pkg/object/encrypt.go:259-284 Decrypt: the header checks, aead.Open
 *
 * Restated from GB/T 32907-2016 (SM4: 32 rounds, tau = S-box per byte,
 * L(B) = B ^ B<<<2 ^ B<<<10 ^ B<<<18 ^ B<<<24, key schedule with FK, CK and
 * L'(B) = B ^ B<<<13 ^ B<<<23), NIST SP 800-38D (GCM, as in aes_gcm_oracle.c)
 * and RFC 8439 (ChaCha20 block function, Poly1305, the AEAD construction).
 * Pinned in tests/test_aead.py by the GB/T 32907 example, RFC 8439's test
 * vectors and OpenSSL (SM4-ECB, ChaCha20-Poly1305) on random inputs.
 */
#include <stdint.h>
#include <string.h>

/* ---- SM4 ------------------------------------------------------------------ */
static const uint8_t SM4_S[256] = {
    0xd6, 0x90, 0xe9, 0xfe, 0xcc, 0xe1, 0x3d, 0xb7, 0x16, 0xb6, 0x14, 0xc2, 0x28, 0xfb, 0x2c, 0x05, 0x2b, 0x67, 0x9a,
    0x76, 0x2a, 0xbe, 0x04, 0xc3, 0xaa, 0x44, 0x13, 0x26, 0x49, 0x86, 0x06, 0x99, 0x9c, 0x42, 0x50, 0xf4, 0x91, 0xef,
    0x98, 0x7a, 0x33, 0x54, 0x0b, 0x43, 0xed, 0xcf, 0xac, 0x62, 0xe4, 0xb3, 0x1c, 0xa9, 0xc9, 0x08, 0xe8, 0x95, 0x80,
    0xdf, 0x94, 0xfa, 0x75, 0x8f, 0x3f, 0xa6, 0x47, 0x07, 0xa7, 0xfc, 0xf3, 0x73, 0x17, 0xba, 0x83, 0x59, 0x3c, 0x19,
    0xe6, 0x85, 0x4f, 0xa8, 0x68, 0x6b, 0x81, 0xb2, 0x71, 0x64, 0xda, 0x8b, 0xf8, 0xeb, 0x0f, 0x4b, 0x70, 0x56, 0x9d,
    0x35, 0x1e, 0x24, 0x0e, 0x5e, 0x63, 0x58, 0xd1, 0xa2, 0x25, 0x22, 0x7c, 0x3b, 0x01, 0x21, 0x78, 0x87, 0xd4, 0x00,
    0x46, 0x57, 0x9f, 0xd3, 0x27, 0x52, 0x4c, 0x36, 0x02, 0xe7, 0xa0, 0xc4, 0xc8, 0x9e, 0xea, 0xbf, 0x8a, 0xd2, 0x40,
    0xc7, 0x38, 0xb5, 0xa3, 0xf7, 0xf2, 0xce, 0xf9, 0x61, 0x15, 0xa1, 0xe0, 0xae, 0x5d, 0xa4, 0x9b, 0x34, 0x1a, 0x55,
    0xad, 0x93, 0x32, 0x30, 0xf5, 0x8c, 0xb1, 0xe3, 0x1d, 0xf6, 0xe2, 0x2e, 0x82, 0x66, 0xca, 0x60, 0xc0, 0x29, 0x23,
    0xab, 0x0d, 0x53, 0x4e, 0x6f, 0xd5, 0xdb, 0x37, 0x45, 0xde, 0xfd, 0x8e, 0x2f, 0x03, 0xff, 0x6a, 0x72, 0x6d, 0x6c,
    0x5b, 0x51, 0x8d, 0x1b, 0xaf, 0x92, 0xbb, 0xdd, 0xbc, 0x7f, 0x11, 0xd9, 0x5c, 0x41, 0x1f, 0x10, 0x5a, 0xd8, 0x0a,
    0xc1, 0x31, 0x88, 0xa5, 0xcd, 0x7b, 0xbd, 0x2d, 0x74, 0xd0, 0x12, 0xb8, 0xe5, 0xb4, 0xb0, 0x89, 0x69, 0x97, 0x4a,
    0x0c, 0x96, 0x77, 0x7e, 0x65, 0xb9, 0xf1, 0x09, 0xc5, 0x6e, 0xc6, 0x84, 0x18, 0xf0, 0x7d, 0xec, 0x3a, 0xdc, 0x4d,
    0x20, 0x79, 0xee, 0x5f, 0x3e, 0xd7, 0xcb, 0x39, 0x48};

static const uint32_t SM4_FK[4] = {0xa3b1bac6u, 0x56aa3350u, 0x677d9197u, 0xb27022dcu};

static uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static uint32_t be32(const uint8_t *p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
static void put_be32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}
static uint32_t tau(uint32_t a) {
    return ((uint32_t)SM4_S[a >> 24] << 24) | ((uint32_t)SM4_S[(a >> 16) & 255] << 16) |
           ((uint32_t)SM4_S[(a >> 8) & 255] << 8) | SM4_S[a & 255];
}

static void sm4_keys(const uint8_t key[16], uint32_t rk[32]) {
    uint32_t k[36];
    for (int i = 0; i < 4; i++) k[i] = be32(key + 4 * i) ^ SM4_FK[i];
    for (int i = 0; i < 32; i++) {
        uint32_t ck = 0;
        for (int j = 0; j < 4; j++) ck = (ck << 8) | (uint32_t)(((4 * i + j) * 7) & 255);
        const uint32_t b = tau(k[i + 1] ^ k[i + 2] ^ k[i + 3] ^ ck);
        k[i + 4] = k[i] ^ b ^ rol(b, 13) ^ rol(b, 23);
        rk[i] = k[i + 4];
    }
}

static void sm4_block(const uint32_t rk[32], const uint8_t in[16], uint8_t out[16]) {
    uint32_t x[36];
    for (int i = 0; i < 4; i++) x[i] = be32(in + 4 * i);
    for (int i = 0; i < 32; i++) {
        const uint32_t b = tau(x[i + 1] ^ x[i + 2] ^ x[i + 3] ^ rk[i]);
        x[i + 4] = x[i] ^ b ^ rol(b, 2) ^ rol(b, 10) ^ rol(b, 18) ^ rol(b, 24);
    }
    for (int i = 0; i < 4; i++) put_be32(out + 4 * i, x[35 - i]);
}

void oracle_sm4_encrypt_block(const uint8_t key[16], const uint8_t in[16], uint8_t out[16]) {
    uint32_t rk[32];
    sm4_keys(key, rk);
    sm4_block(rk, in, out);
}

/* ---- GCM over SM4 (SP 800-38D; the bit-at-a-time multiply) ---------------- */
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

static void sm4gcm(const uint8_t key[16], const uint8_t nonce[12], const uint8_t *in, int64_t n, uint8_t *out,
                   int decrypt, uint8_t tag[16]) {
    uint32_t rk[32];
    uint8_t H[16], J0[16], ctr[16], ks[16], Y[16];
    sm4_keys(key, rk);
    memset(H, 0, 16);
    sm4_block(rk, H, H);
    memcpy(J0, nonce, 12);
    J0[12] = J0[13] = J0[14] = 0;
    J0[15] = 1;
    memset(Y, 0, 16);
    uint32_t c = 2;
    for (int64_t o = 0; o < n; o += 16, c++) {
        int len = n - o < 16 ? (int)(n - o) : 16;
        memcpy(ctr, nonce, 12);
        put_be32(ctr + 12, c);
        sm4_block(rk, ctr, ks);
        if (decrypt) ghash_block(Y, H, in + o, len);
        for (int k = 0; k < len; k++) out[o + k] = in[o + k] ^ ks[k];
        if (!decrypt) ghash_block(Y, H, out + o, len);
    }
    uint8_t L[16];
    memset(L, 0, 16);
    uint64_t bits = (uint64_t)n * 8;
    for (int k = 0; k < 8; k++) L[15 - k] = (uint8_t)(bits >> (8 * k));
    ghash_block(Y, H, L, 16);
    sm4_block(rk, J0, ks);
    for (int k = 0; k < 16; k++) tag[k] = ks[k] ^ Y[k];
}

int64_t oracle_sm4gcm_seal(const uint8_t *key, const uint8_t *nonce, const uint8_t *src, int64_t n, uint8_t *dst) {
    sm4gcm(key, nonce, src, n, dst, 0, dst + n);
    return n + 16;
}

int64_t oracle_sm4gcm_open(const uint8_t *key, const uint8_t *nonce, const uint8_t *src, int64_t n, uint8_t *dst) {
    if (n < 16) return -1;
    uint8_t tag[16];
    sm4gcm(key, nonce, src, n - 16, dst, 1, tag);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= (uint8_t)(tag[k] ^ src[n - 16 + k]);
    return d ? -1 : n - 16;
}

/* ---- ChaCha20-Poly1305 (RFC 8439) ------------------------------------------ */
static uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static void put_le32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

#define QR(a, b, c, d)                 \
    a += b, d ^= a, d = rol(d, 16);    \
    c += d, b ^= c, b = rol(b, 12);    \
    a += b, d ^= a, d = rol(d, 8);     \
    c += d, b ^= c, b = rol(b, 7)

/* RFC 8439 2.3: the 64-byte block for (key, counter, nonce) */
void oracle_chacha20_block(const uint8_t key[32], uint32_t counter, const uint8_t nonce[12], uint8_t out[64]) {
    uint32_t s[16], x[16];
    s[0] = 0x61707865u;
    s[1] = 0x3320646eu;
    s[2] = 0x79622d32u;
    s[3] = 0x6b206574u;
    for (int i = 0; i < 8; i++) s[4 + i] = le32(key + 4 * i);
    s[12] = counter;
    for (int i = 0; i < 3; i++) s[13 + i] = le32(nonce + 4 * i);
    memcpy(x, s, sizeof(x));
    for (int r = 0; r < 10; r++) {
        QR(x[0], x[4], x[8], x[12]);
        QR(x[1], x[5], x[9], x[13]);
        QR(x[2], x[6], x[10], x[14]);
        QR(x[3], x[7], x[11], x[15]);
        QR(x[0], x[5], x[10], x[15]);
        QR(x[1], x[6], x[11], x[12]);
        QR(x[2], x[7], x[8], x[13]);
        QR(x[3], x[4], x[9], x[14]);
    }
    for (int i = 0; i < 16; i++) put_le32(out + 4 * i, x[i] + s[i]);
}

/* Poly1305 (RFC 8439 2.5) with 26-bit limbs */
typedef struct {
    uint32_t r[5], h[5], pad[4];
} poly_t;

static void poly_init(poly_t *p, const uint8_t key[32]) {
    p->r[0] = (le32(key + 0)) & 0x3ffffff;
    p->r[1] = (le32(key + 3) >> 2) & 0x3ffff03;
    p->r[2] = (le32(key + 6) >> 4) & 0x3ffc0ff;
    p->r[3] = (le32(key + 9) >> 6) & 0x3f03fff;
    p->r[4] = (le32(key + 12) >> 8) & 0x00fffff;
    for (int i = 0; i < 5; i++) p->h[i] = 0;
    for (int i = 0; i < 4; i++) p->pad[i] = le32(key + 16 + 4 * i);
}

/* one 16-byte block m (already padded), plus 2^128 */
static void poly_block(poly_t *p, const uint8_t m[16]) {
    const uint32_t r0 = p->r[0], r1 = p->r[1], r2 = p->r[2], r3 = p->r[3], r4 = p->r[4];
    const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
    uint32_t h0 = p->h[0], h1 = p->h[1], h2 = p->h[2], h3 = p->h[3], h4 = p->h[4];
    h0 += (le32(m + 0)) & 0x3ffffff;
    h1 += (le32(m + 3) >> 2) & 0x3ffffff;
    h2 += (le32(m + 6) >> 4) & 0x3ffffff;
    h3 += (le32(m + 9) >> 6) & 0x3ffffff;
    h4 += (le32(m + 12) >> 8) | (1u << 24);
    const uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
    uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
    uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
    uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
    uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
    uint32_t c = (uint32_t)(d0 >> 26);
    h0 = (uint32_t)d0 & 0x3ffffff;
    d1 += c;
    c = (uint32_t)(d1 >> 26);
    h1 = (uint32_t)d1 & 0x3ffffff;
    d2 += c;
    c = (uint32_t)(d2 >> 26);
    h2 = (uint32_t)d2 & 0x3ffffff;
    d3 += c;
    c = (uint32_t)(d3 >> 26);
    h3 = (uint32_t)d3 & 0x3ffffff;
    d4 += c;
    c = (uint32_t)(d4 >> 26);
    h4 = (uint32_t)d4 & 0x3ffffff;
    h0 += c * 5;
    c = h0 >> 26;
    h0 &= 0x3ffffff;
    h1 += c;
    p->h[0] = h0, p->h[1] = h1, p->h[2] = h2, p->h[3] = h3, p->h[4] = h4;
}

static void poly_update(poly_t *p, const uint8_t *m, int64_t n) { /* zero-padded to 16 (AEAD) */
    for (int64_t o = 0; o < n; o += 16) {
        uint8_t b[16];
        memset(b, 0, 16);
        memcpy(b, m + o, (size_t)(n - o < 16 ? n - o : 16));
        poly_block(p, b);
    }
}

static void poly_finish(poly_t *p, uint8_t tag[16]) {
    uint32_t h0 = p->h[0], h1 = p->h[1], h2 = p->h[2], h3 = p->h[3], h4 = p->h[4], c;
    c = h1 >> 26, h1 &= 0x3ffffff, h2 += c;
    c = h2 >> 26, h2 &= 0x3ffffff, h3 += c;
    c = h3 >> 26, h3 &= 0x3ffffff, h4 += c;
    c = h4 >> 26, h4 &= 0x3ffffff, h0 += c * 5;
    c = h0 >> 26, h0 &= 0x3ffffff, h1 += c;
    /* h - p */
    uint32_t g0 = h0 + 5;
    c = g0 >> 26, g0 &= 0x3ffffff;
    uint32_t g1 = h1 + c;
    c = g1 >> 26, g1 &= 0x3ffffff;
    uint32_t g2 = h2 + c;
    c = g2 >> 26, g2 &= 0x3ffffff;
    uint32_t g3 = h3 + c;
    c = g3 >> 26, g3 &= 0x3ffffff;
    uint32_t g4 = h4 + c - (1u << 26);
    uint32_t mask = (g4 >> 31) - 1; /* all ones if h >= p */
    h0 = (h0 & ~mask) | (g0 & mask);
    h1 = (h1 & ~mask) | (g1 & mask);
    h2 = (h2 & ~mask) | (g2 & mask);
    h3 = (h3 & ~mask) | (g3 & mask);
    h4 = (h4 & ~mask) | (g4 & mask);
    const uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14),
                   w3 = (h3 >> 18) | (h4 << 8);
    uint64_t f = (uint64_t)w0 + p->pad[0];
    put_le32(tag, (uint32_t)f);
    f = (uint64_t)w1 + p->pad[1] + (f >> 32);
    put_le32(tag + 4, (uint32_t)f);
    f = (uint64_t)w2 + p->pad[2] + (f >> 32);
    put_le32(tag + 8, (uint32_t)f);
    f = (uint64_t)w3 + p->pad[3] + (f >> 32);
    put_le32(tag + 12, (uint32_t)f);
}

/* RFC 8439 2.5 Poly1305 MAC of an arbitrary message (last block with its own 1 bit) */
void oracle_poly1305(const uint8_t key[32], const uint8_t *m, int64_t n, uint8_t tag[16]) {
    poly_t p;
    poly_init(&p, key);
    int64_t o = 0;
    for (; o + 16 <= n; o += 16) poly_block(&p, m + o);
    if (o < n) { /* partial: append 1, pad with zeros, no 2^128 */
        uint8_t b[17];
        memset(b, 0, 17);
        memcpy(b, m + o, (size_t)(n - o));
        b[n - o] = 1;
        /* poly_block adds 2^128; emulate the 2^(8*len) bit instead by subtracting it back */
        uint32_t save = p.h[4];
        (void)save;
        const uint32_t r0 = p.r[0], r1 = p.r[1], r2 = p.r[2], r3 = p.r[3], r4 = p.r[4];
        const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
        uint32_t h0 = p.h[0], h1 = p.h[1], h2 = p.h[2], h3 = p.h[3], h4 = p.h[4];
        h0 += (le32(b + 0)) & 0x3ffffff;
        h1 += (le32(b + 3) >> 2) & 0x3ffffff;
        h2 += (le32(b + 6) >> 4) & 0x3ffffff;
        h3 += (le32(b + 9) >> 6) & 0x3ffffff;
        h4 += (le32(b + 12) >> 8);
        uint64_t d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 + (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
        uint64_t d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 + (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
        uint64_t d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 + (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
        uint64_t d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 + (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
        uint64_t d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 + (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
        uint32_t c = (uint32_t)(d0 >> 26);
        h0 = (uint32_t)d0 & 0x3ffffff;
        d1 += c, c = (uint32_t)(d1 >> 26), h1 = (uint32_t)d1 & 0x3ffffff;
        d2 += c, c = (uint32_t)(d2 >> 26), h2 = (uint32_t)d2 & 0x3ffffff;
        d3 += c, c = (uint32_t)(d3 >> 26), h3 = (uint32_t)d3 & 0x3ffffff;
        d4 += c, c = (uint32_t)(d4 >> 26), h4 = (uint32_t)d4 & 0x3ffffff;
        h0 += c * 5, c = h0 >> 26, h0 &= 0x3ffffff, h1 += c;
        p.h[0] = h0, p.h[1] = h1, p.h[2] = h2, p.h[3] = h3, p.h[4] = h4;
    }
    poly_finish(&p, tag);
}

static void chacha_xor(const uint8_t key[32], const uint8_t nonce[12], uint32_t counter, const uint8_t *in, int64_t n,
                       uint8_t *out) {
    uint8_t ks[64];
    for (int64_t o = 0; o < n; o += 64, counter++) {
        oracle_chacha20_block(key, counter, nonce, ks);
        const int64_t len = n - o < 64 ? n - o : 64;
        for (int64_t k = 0; k < len; k++) out[o + k] = in[o + k] ^ ks[k];
    }
}

static void aead_tag(const uint8_t key[32], const uint8_t nonce[12], const uint8_t *aad, int64_t alen,
                     const uint8_t *ct, int64_t n, uint8_t tag[16]) {
    uint8_t otk[64], lens[16];
    oracle_chacha20_block(key, 0, nonce, otk);
    poly_t p;
    poly_init(&p, otk);
    poly_update(&p, aad, alen);
    poly_update(&p, ct, n);
    for (int k = 0; k < 8; k++) lens[k] = (uint8_t)((uint64_t)alen >> (8 * k));
    for (int k = 0; k < 8; k++) lens[8 + k] = (uint8_t)((uint64_t)n >> (8 * k));
    poly_block(&p, lens);
    poly_finish(&p, tag);
}

/* chacha20poly1305 Seal / Open (RFC 8439 2.8) with optional additional data
 * (JuiceFS passes none) */
int64_t oracle_chacha20poly1305_seal(const uint8_t *key, const uint8_t *nonce, const uint8_t *aad, int64_t alen,
                                     const uint8_t *src, int64_t n, uint8_t *dst) {
    chacha_xor(key, nonce, 1, src, n, dst);
    aead_tag(key, nonce, aad, alen, dst, n, dst + n);
    return n + 16;
}

int64_t oracle_chacha20poly1305_open(const uint8_t *key, const uint8_t *nonce, const uint8_t *aad, int64_t alen,
                                     const uint8_t *src, int64_t n, uint8_t *dst) {
    if (n < 16) return -1;
    uint8_t tag[16];
    aead_tag(key, nonce, aad, alen, src, n - 16, tag);
    uint8_t d = 0;
    for (int k = 0; k < 16; k++) d |= (uint8_t)(tag[k] ^ src[n - 16 + k]);
    if (d) return -1;
    chacha_xor(key, nonce, 1, src, n - 16, dst);
    return n - 16;
}

/* ---- the object envelope (encrypt.go:226-284) ------------------------------ */
/* Encrypt's layout: returns the envelope size written to dst */
int64_t oracle_envelope_write(const uint8_t *wrapped, int64_t wlen, const uint8_t *nonce, int64_t nlen,
                              const uint8_t *sealed, int64_t slen, uint8_t *dst) {
    dst[0] = (uint8_t)(wlen >> 8);
    dst[1] = (uint8_t)(wlen & 0xFF);
    dst[2] = (uint8_t)nlen;
    memcpy(dst + 3, wrapped, (size_t)wlen);
    memcpy(dst + 3 + wlen, nonce, (size_t)nlen);
    memcpy(dst + 3 + wlen + nlen, sealed, (size_t)slen);
    return 3 + wlen + nlen + slen;
}

/* Decrypt's header checks: returns the payload offset (wrapped key at 3,
 * nonce after it), or -1 ("length is less than 3") / -2 ("malformed") */
int64_t oracle_envelope_parse(const uint8_t *src, int64_t n, int64_t *wlen, int64_t *nlen) {
    if (n < 3) return -1;
    *wlen = ((int64_t)src[0] << 8) + src[1];
    *nlen = src[2];
    if (3 + *wlen + *nlen >= n) return -2;
    return 3 + *wlen + *nlen;
}
