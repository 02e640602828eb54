// The AEADs of JuiceFS object encryption for device-resident blocks, gfx950 --
// SURVEY.md section 8(f)3, applied to every object right after compression
// (pkg/object/encrypt.go:176-202 NewDataEncryptor; Encrypt :226-257
// aead.Seal(p[:0], nonce, plaintext, nil), Decrypt :259-284 aead.Open):
//   AES256GCM_RSA  aes.NewCipher(32-byte key) + cipher.NewGCM
//   SM4GCM         sm4.NewCipher(16-byte key) + cipher.NewGCM
//   CHACHA20_RSA   chacha20poly1305.New(32-byte key)
// all with a 12-byte nonce, a 16-byte tag and no additional data.  The
// per-object key wrap (RSA / SM2 of the random data key, :234-237) stays on
// the host; the object envelope around the sealed bytes is written by the
// host batch path (capi.hip).
// CPU restatements (test infrastructure): oracle/aes_gcm_oracle.c,
// oracle/aead_oracle.c.
//
// GCM (AES or SM4): one workgroup of 256 lanes per block.  Lane t takes the
// 16-byte blocks t, t+256, t+512, ... (every row of 4 KiB is one coalesced
// read and write):
//   CTR:   C_i = P_i ^ E_K(nonce || be32(i + 2)), the cipher's tables in LDS
//          (AES: T-tables; SM4: the S-box composed with L, four rotations);
//   GHASH: Y_m = sum_i C_i * H^(m+1-i) over GF(2^128).  Each lane folds its
//          blocks by Horner with the constant H^256 (multiply by a constant =
//          16 lookups in a 256-entry table of b*H^256 built per block), then
//          multiplies its sum by H^(m - i_last) and the lanes XOR-reduce;
//          tag = E_K(J0) ^ (Y_m ^ L) * H,  L = bit lengths (0 || 8n).
// Elements of GF(2^128) are held as four big-endian words (GCM bit order:
// the first bit of the block is the x^0 coefficient = the MSB of word 0).
// ChaCha20-Poly1305: see chacha_kernel below.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace gcm {

constexpr int LANES = 256;

constexpr uint8_t SBOX[256] = {
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

constexpr uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0)); }

constexpr uint8_t SM4_S[256] = {
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

constexpr uint32_t rotl_c(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// Block-cipher tables + the GHASH reduction table, one layout for both GCMs.
// AES: te[k][x] = the T-table (2s, s, s, 3s) rotated right 8k.  SM4: te[k][x] =
// L(S(x) << (24 - 8k)), L(B) = B ^ B<<<2 ^ B<<<10 ^ B<<<18 ^ B<<<24, so a
// round's T(w) is four lookups xor-ed.
struct Tables {
    uint32_t te[4][256];
    uint32_t sb[256];     // S-box (a word per entry: no sub-dword LDS reads)
    uint32_t r8[256];     // GHASH: top 16 bits added when a byte d is shifted out by a multiply by x^8
};

constexpr void fill_r8(Tables &T) {
    for (int x = 0; x < 256; x++) {
        // r8: the 128-bit value with only its last byte = x, times x^8
        uint32_t v0 = 0, v1 = 0, v2 = 0, v3 = (uint32_t)x;
        for (int k = 0; k < 8; k++) {
            const uint32_t lsb = v3 & 1u;
            v3 = (v3 >> 1) | (v2 << 31);
            v2 = (v2 >> 1) | (v1 << 31);
            v1 = (v1 >> 1) | (v0 << 31);
            v0 >>= 1;
            if (lsb) v0 ^= 0xE1000000u;
        }
        T.r8[x] = v0 >> 16;  // (v1..v3 are zero)
    }
}

constexpr Tables make_tables() {
    Tables T{};
    for (int x = 0; x < 256; x++) {
        const uint32_t s = SBOX[x], m2 = xtime((uint8_t)s), m3 = m2 ^ s;
        const uint32_t w = (m2 << 24) | (s << 16) | (s << 8) | m3;
        T.te[0][x] = w;
        T.te[1][x] = (w >> 8) | (w << 24);
        T.te[2][x] = (w >> 16) | (w << 16);
        T.te[3][x] = (w >> 24) | (w << 8);
        T.sb[x] = s;
    }
    fill_r8(T);
    return T;
}

constexpr Tables make_sm4_tables() {
    Tables T{};
    for (int x = 0; x < 256; x++) {
        for (int k = 0; k < 4; k++) {
            const uint32_t b = (uint32_t)SM4_S[x] << (24 - 8 * k);
            T.te[k][x] = b ^ rotl_c(b, 2) ^ rotl_c(b, 10) ^ rotl_c(b, 18) ^ rotl_c(b, 24);
        }
        T.sb[x] = SM4_S[x];
    }
    fill_r8(T);
    return T;
}

__constant__ Tables g_tab = make_tables();
__constant__ Tables g_tab_sm4 = make_sm4_tables();

struct G128 {
    uint32_t w[4];
};

__device__ __forceinline__ G128 gxor(G128 a, const G128 &b) {
#pragma unroll
    for (int k = 0; k < 4; k++) a.w[k] ^= b.w[k];
    return a;
}

// a * x (GCM order): the 128-bit big-endian integer shifted right by one, reduced
__device__ __forceinline__ G128 mulx(G128 a) {
    const uint32_t lsb = a.w[3] & 1u;
    a.w[3] = (a.w[3] >> 1) | (a.w[2] << 31);
    a.w[2] = (a.w[2] >> 1) | (a.w[1] << 31);
    a.w[1] = (a.w[1] >> 1) | (a.w[0] << 31);
    a.w[0] = (a.w[0] >> 1) ^ (lsb ? 0xE1000000u : 0u);
    return a;
}

// generic product (SP 800-38D Algorithm 1); used a few times per block
__device__ G128 gmul(const G128 &x, G128 v) {
    G128 z = {{0, 0, 0, 0}};
    for (int i = 0; i < 128; i++) {
        if ((x.w[i >> 5] >> (31 - (i & 31))) & 1u) z = gxor(z, v);
        v = mulx(v);
    }
    return z;
}

struct Smem {
    Tables T;
    uint32_t rk[60];
    uint4 M[256];   // M[b] = b * H^256, b = the first byte (x^0..x^7 coefficients)
    G128 H, H256, EJ0;
    uint32_t red[LANES / 64][4];
    int32_t tag_ok;
};

__device__ __forceinline__ uint32_t sbw(const Smem &s, uint32_t w) {  // SubWord
    return (s.T.sb[w >> 24] << 24) | (s.T.sb[(w >> 16) & 255] << 16) | (s.T.sb[(w >> 8) & 255] << 8) | s.T.sb[w & 255];
}

// AES-256 of one block given as big-endian words
__device__ __forceinline__ void aes_enc(const Smem &s, uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    const uint32_t *rk = s.rk;
    const Tables &T = s.T;
    s0 ^= rk[0];
    s1 ^= rk[1];
    s2 ^= rk[2];
    s3 ^= rk[3];
#pragma unroll 1
    for (int r = 1; r < 14; r++) {
        const uint32_t t0 = T.te[0][s0 >> 24] ^ T.te[1][(s1 >> 16) & 255] ^ T.te[2][(s2 >> 8) & 255] ^ T.te[3][s3 & 255] ^ rk[4 * r];
        const uint32_t t1 = T.te[0][s1 >> 24] ^ T.te[1][(s2 >> 16) & 255] ^ T.te[2][(s3 >> 8) & 255] ^ T.te[3][s0 & 255] ^ rk[4 * r + 1];
        const uint32_t t2 = T.te[0][s2 >> 24] ^ T.te[1][(s3 >> 16) & 255] ^ T.te[2][(s0 >> 8) & 255] ^ T.te[3][s1 & 255] ^ rk[4 * r + 2];
        const uint32_t t3 = T.te[0][s3 >> 24] ^ T.te[1][(s0 >> 16) & 255] ^ T.te[2][(s1 >> 8) & 255] ^ T.te[3][s2 & 255] ^ rk[4 * r + 3];
        s0 = t0;
        s1 = t1;
        s2 = t2;
        s3 = t3;
    }
    const uint32_t *sb = T.sb;
    const uint32_t o0 = (sb[s0 >> 24] << 24) ^ (sb[(s1 >> 16) & 255] << 16) ^ (sb[(s2 >> 8) & 255] << 8) ^ sb[s3 & 255] ^ rk[56];
    const uint32_t o1 = (sb[s1 >> 24] << 24) ^ (sb[(s2 >> 16) & 255] << 16) ^ (sb[(s3 >> 8) & 255] << 8) ^ sb[s0 & 255] ^ rk[57];
    const uint32_t o2 = (sb[s2 >> 24] << 24) ^ (sb[(s3 >> 16) & 255] << 16) ^ (sb[(s0 >> 8) & 255] << 8) ^ sb[s1 & 255] ^ rk[58];
    const uint32_t o3 = (sb[s3 >> 24] << 24) ^ (sb[(s0 >> 16) & 255] << 16) ^ (sb[(s1 >> 8) & 255] << 8) ^ sb[s2 & 255] ^ rk[59];
    s0 = o0;
    s1 = o1;
    s2 = o2;
    s3 = o3;
}

// SM4 of one block given as big-endian words (GB/T 32907: 32 rounds
// X_{i+4} = X_i ^ T(X_{i+1} ^ X_{i+2} ^ X_{i+3} ^ rk_i), output reversed)
__device__ __forceinline__ void sm4_enc(const Smem &s, uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    const Tables &T = s.T;
    uint32_t x0 = s0, x1 = s1, x2 = s2, x3 = s3;
#pragma unroll 4
    for (int r = 0; r < 32; r++) {
        const uint32_t w = x1 ^ x2 ^ x3 ^ s.rk[r];
        const uint32_t t = T.te[0][w >> 24] ^ T.te[1][(w >> 16) & 255] ^ T.te[2][(w >> 8) & 255] ^ T.te[3][w & 255];
        const uint32_t y = x0 ^ t;
        x0 = x1;
        x1 = x2;
        x2 = x3;
        x3 = y;
    }
    s0 = x3;
    s1 = x2;
    s2 = x1;
    s3 = x0;
}

template <int C>
__device__ __forceinline__ void blk_enc(const Smem &s, uint32_t &s0, uint32_t &s1, uint32_t &s2, uint32_t &s3) {
    if (C == JFS_CIPHER_SM4GCM) sm4_enc(s, s0, s1, s2, s3);
    else aes_enc(s, s0, s1, s2, s3);
}

// a * H^256 with the byte table (16 lookups, a shift by 8 bits + reduction between them)
__device__ __forceinline__ G128 mul_h256(const Smem &s, const G128 &a) {
    uint4 z = s.M[a.w[3] & 255];
#pragma unroll
    for (int k = 14; k >= 0; k--) {
        const uint32_t d = z.w & 255u;
        z.w = (z.w >> 8) | (z.z << 24);
        z.z = (z.z >> 8) | (z.y << 24);
        z.y = (z.y >> 8) | (z.x << 24);
        z.x = (z.x >> 8) ^ (s.T.r8[d] << 16);
        const uint32_t byte = (a.w[k >> 2] >> (24 - 8 * (k & 3))) & 255u;
        const uint4 m = s.M[byte];
        z.x ^= m.x;
        z.y ^= m.y;
        z.z ^= m.z;
        z.w ^= m.w;
    }
    return G128{{z.x, z.y, z.z, z.w}};
}

__device__ __forceinline__ uint32_t bswap(uint32_t v) { return __builtin_bswap32(v); }

// 16 bytes at p of which [0, len) are real (the rest read as 0); little-endian words
__device__ __forceinline__ uint4 load_part(const gc_u8 *p, int len, bool aligned) {
    if (aligned && len == 16) return *(const gc_u4 *)p;
    uint32_t d[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++)
        if (i < len) d[i >> 2] |= (uint32_t)p[i] << (8 * (i & 3));
    return make_uint4(d[0], d[1], d[2], d[3]);
}
__device__ __forceinline__ void store_part(g_u8 *p, const uint4 &v, int len, bool aligned) {
    if (aligned && len == 16) {
        *(g_u4 *)p = v;
        return;
    }
    const uint32_t d[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 16; i++)
        if (i < len) p[i] = (uint8_t)(d[i >> 2] >> (8 * (i & 3)));
}

// mode 0 = seal (src = plaintext, n = src_len; dst = ciphertext || tag),
// mode 1 = open (src = ciphertext || tag, n = src_len - 16; dst = plaintext)
// lens (optional): per-block input lengths produced on the device by the
// previous kernel of a fused chain (LZ4 compress: <= 0 = it failed).
template <int C>
__global__ __launch_bounds__(LANES) void gcm_kernel(const jfs_aead_block *__restrict__ blocks, int nblk, int mode,
                                                     int32_t *__restrict__ ret, const int32_t *__restrict__ lens) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    const int t = threadIdx.x, l = t & 63, wv = t >> 6;
    {
        const uint32_t *g = (const uint32_t *)(C == JFS_CIPHER_SM4GCM ? &g_tab_sm4 : &g_tab);
        uint32_t *d = (uint32_t *)&s.T;
        for (int i = t; i < (int)(sizeof(Tables) / 4); i += LANES) d[i] = g[i];
    }
    if (b >= nblk) return;
    jfs_aead_block blk = ((JFS_GLOBAL const jfs_aead_block *)blocks)[b];
    if (lens) {
        const int32_t ln = lens[b];
        if (ln <= 0) {  // the chained step failed
            if (t == 0) ret[b] = JFS_CHAIN_FAILED;
            return;
        }
        blk.src_len = ln;
    }
    const gc_u8 *src = (const gc_u8 *)blk.src;
    g_u8 *dst = (g_u8 *)blk.dst;
    const int64_t n = mode == 0 ? (int64_t)blk.src_len : (int64_t)blk.src_len - 16;
    const int64_t need = mode == 0 ? n + 16 : n;
    const bool bad = blk.src_len < 0 || n < 0 || (int64_t)blk.dst_cap < need || blk.key == nullptr || blk.nonce == nullptr;
    if (bad) {
        if (t == 0) ret[b] = -2;
        return;
    }
    const gc_u8 *key = (const gc_u8 *)blk.key, *nonce = (const gc_u8 *)blk.nonce;
    const uint32_t n0 = ((uint32_t)nonce[0] << 24) | ((uint32_t)nonce[1] << 16) | ((uint32_t)nonce[2] << 8) | nonce[3];
    const uint32_t n1 = ((uint32_t)nonce[4] << 24) | ((uint32_t)nonce[5] << 16) | ((uint32_t)nonce[6] << 8) | nonce[7];
    const uint32_t n2 = ((uint32_t)nonce[8] << 24) | ((uint32_t)nonce[9] << 16) | ((uint32_t)nonce[10] << 8) | nonce[11];
    __syncthreads();
    if (t == 0 && C == JFS_CIPHER_SM4GCM) {  // SM4 key schedule (GB/T 32907 7.3)
        const uint32_t FK[4] = {0xa3b1bac6u, 0x56aa3350u, 0x677d9197u, 0xb27022dcu};
        uint32_t k[4];
        for (int i = 0; i < 4; i++)
            k[i] = (((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) |
                    key[4 * i + 3]) ^ FK[i];
        for (int i = 0; i < 32; i++) {
            uint32_t ck = 0;
            for (int j = 0; j < 4; j++) ck = (ck << 8) | (uint32_t)(((4 * i + j) * 7) & 255);
            const uint32_t w = sbw(s, k[1] ^ k[2] ^ k[3] ^ ck);
            const uint32_t nk = k[0] ^ w ^ ((w << 13) | (w >> 19)) ^ ((w << 23) | (w >> 9));
            s.rk[i] = nk;
            k[0] = k[1];
            k[1] = k[2];
            k[2] = k[3];
            k[3] = nk;
        }
    } else if (t == 0) {  // AES-256 key expansion (FIPS-197 5.2, Nk = 8)
        for (int i = 0; i < 8; i++)
            s.rk[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) | ((uint32_t)key[4 * i + 2] << 8) |
                      key[4 * i + 3];
        uint32_t rc = 1;
        for (int i = 8; i < 60; i++) {
            uint32_t x = s.rk[i - 1];
            if (i % 8 == 0) {
                x = sbw(s, (x << 8) | (x >> 24)) ^ (rc << 24);
                rc = xtime((uint8_t)rc);
            } else if (i % 8 == 4) {
                x = sbw(s, x);
            }
            s.rk[i] = s.rk[i - 8] ^ x;
        }
    }
    __syncthreads();
    if (t == 0) {
        uint32_t h0 = 0, h1 = 0, h2 = 0, h3 = 0;
        blk_enc<C>(s, h0, h1, h2, h3);
        G128 H = {{h0, h1, h2, h3}};
        s.H = H;
        uint32_t j0 = n0, j1 = n1, j2 = n2, j3 = 1;
        blk_enc<C>(s, j0, j1, j2, j3);
        s.EJ0 = G128{{j0, j1, j2, j3}};
        G128 P = H;
        for (int k = 0; k < 8; k++) P = gmul(P, P);  // H^256
        s.H256 = P;
    }
    __syncthreads();
    {  // M[t] = t * H^256 (byte t in the x^0..x^7 position)
        G128 v = s.H256, m = {{0, 0, 0, 0}};
        for (int j = 0; j < 8; j++) {
            if (t & (0x80 >> j)) m = gxor(m, v);
            v = mulx(v);
        }
        s.M[t] = make_uint4(m.w[0], m.w[1], m.w[2], m.w[3]);
    }
    __syncthreads();
    const int64_t nb = (n + 15) >> 4;  // AES blocks
    const bool aligned = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0;
    G128 A = {{0, 0, 0, 0}};
    int64_t last = -1;
    for (int64_t i = t; i < nb; i += LANES) {
        const int len = n - 16 * i < 16 ? (int)(n - 16 * i) : 16;
        const uint4 in = load_part(src + 16 * i, len, aligned);
        uint32_t k0 = n0, k1 = n1, k2 = n2, k3 = (uint32_t)(i + 2);
        blk_enc<C>(s, k0, k1, k2, k3);
        const uint4 out = make_uint4(in.x ^ bswap(k0), in.y ^ bswap(k1), in.z ^ bswap(k2), in.w ^ bswap(k3));
        // the ciphertext block, zero padded, big-endian words
        const uint4 c = mode == 0 ? out : in;
        uint32_t cw[4] = {bswap(c.x), bswap(c.y), bswap(c.z), bswap(c.w)};
        if (len < 16) {  // bytes past len are zero in `in`, not in `out`
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const int keep = len - 4 * k;  // bytes of word k kept (big-endian: the high ones)
                cw[k] = keep >= 4 ? cw[k] : keep <= 0 ? 0u : (cw[k] & (0xFFFFFFFFu << (8 * (4 - keep))));
            }
        }
        A = gxor(mul_h256(s, A), G128{{cw[0], cw[1], cw[2], cw[3]}});
        store_part(dst + 16 * i, out, len, aligned);
        last = i;
    }
    // this lane's sum times H^(nb - last): H^e by square-and-multiply (e <= 256)
    G128 v = {{0, 0, 0, 0}};
    if (last >= 0) {
        uint32_t e = (uint32_t)(nb - last);
        G128 p = s.H, r = {{0, 0, 0, 0}};
        bool have = false;
        while (e) {
            if (e & 1u) {
                r = have ? gmul(r, p) : p;
                have = true;
            }
            e >>= 1;
            if (e) p = gmul(p, p);
        }
        v = gmul(A, r);
    }
#pragma unroll
    for (int k = 0; k < 4; k++) {
        uint32_t x = v.w[k];
        x ^= (uint32_t)__shfl_xor((int)x, 32, 64);
        x ^= (uint32_t)__shfl_xor((int)x, 16, 64);
        x ^= (uint32_t)__shfl_xor((int)x, 8, 64);
        x ^= (uint32_t)__shfl_xor((int)x, 4, 64);
        x ^= (uint32_t)__shfl_xor((int)x, 2, 64);
        x ^= (uint32_t)__shfl_xor((int)x, 1, 64);
        if (l == 0) s.red[wv][k] = x;
    }
    __syncthreads();
    if (t == 0) {
        G128 Y = {{0, 0, 0, 0}};
        for (int w = 0; w < LANES / 64; w++) Y = gxor(Y, G128{{s.red[w][0], s.red[w][1], s.red[w][2], s.red[w][3]}});
        const uint64_t bits = (uint64_t)n * 8u;
        Y = gxor(Y, G128{{0u, 0u, (uint32_t)(bits >> 32), (uint32_t)bits}});
        Y = gmul(Y, s.H);
        const G128 tag = gxor(Y, s.EJ0);
        if (mode == 0) {
            for (int k = 0; k < 16; k++) dst[n + k] = (uint8_t)(tag.w[k >> 2] >> (24 - 8 * (k & 3)));
            ret[b] = (int32_t)(n + 16);
        } else {
            uint32_t diff = 0;
            for (int k = 0; k < 16; k++) diff |= (uint32_t)src[n + k] ^ ((tag.w[k >> 2] >> (24 - 8 * (k & 3))) & 255u);
            ret[b] = diff ? -1 : (int32_t)n;
            s.tag_ok = diff == 0;
        }
    }
    if (mode == 1) {
        // Go's gcm.Open clears its output when the tag does not verify: no
        // unauthenticated plaintext is left in dst (only the failure path pays)
        __syncthreads();
        if (!s.tag_ok)
            for (int64_t i = t; i < nb; i += LANES) {
                const int len = n - 16 * i < 16 ? (int)(n - 16 * i) : 16;
                store_part(dst + 16 * i, make_uint4(0, 0, 0, 0), len, aligned);
            }
    }
}

}  // namespace gcm

// ---------------------------------------------------------------------------
// ChaCha20-Poly1305 (RFC 8439 2.8; golang.org/x/crypto/chacha20poly1305 as
// encrypt.go:190 uses it).  One workgroup of 256 lanes per block; lane t
// takes the 64-byte keystream blocks t, t+256, ... (counter = index + 1):
// the ChaCha20 block function in registers, xor, coalesced 16-byte loads and
// stores.  Poly1305 over the ciphertext (zero-padded to 16, then the 16-byte
// lengths block, every block with its 2^128 bit): tag = sum_i m_i r^(M-i) + s
// mod 2^130-5.  A lane folds its own 16-byte blocks by Horner (r between the
// four blocks of a keystream block, r^1021 to its next one), multiplies its
// sum by r^(M - its last block), and the lanes' sums are added in LDS.
// Numbers mod 2^130-5 are five 26-bit limbs (the poly1305-donna layout).
// ---------------------------------------------------------------------------
namespace cc {

constexpr int LANES = 256;

struct P130 {
    uint32_t h[5];
};

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// a * b mod 2^130-5 (a limbs < 2^27, b limbs < 2^26 + small); result limbs < 2^26 (+ a small h1 excess)
__device__ __forceinline__ P130 pmul(const P130 &a, const P130 &b) {
    const uint32_t b0 = b.h[0], b1 = b.h[1], b2 = b.h[2], b3 = b.h[3], b4 = b.h[4];
    const uint32_t s1 = b1 * 5, s2 = b2 * 5, s3 = b3 * 5, s4 = b4 * 5;
    const uint64_t a0 = a.h[0], a1 = a.h[1], a2 = a.h[2], a3 = a.h[3], a4 = a.h[4];
    uint64_t d0 = a0 * b0 + a1 * s4 + a2 * s3 + a3 * s2 + a4 * s1;
    uint64_t d1 = a0 * b1 + a1 * b0 + a2 * s4 + a3 * s3 + a4 * s2;
    uint64_t d2 = a0 * b2 + a1 * b1 + a2 * b0 + a3 * s4 + a4 * s3;
    uint64_t d3 = a0 * b3 + a1 * b2 + a2 * b1 + a3 * b0 + a4 * s4;
    uint64_t d4 = a0 * b4 + a1 * b3 + a2 * b2 + a3 * b1 + a4 * b0;
    P130 r;
    uint32_t c = (uint32_t)(d0 >> 26);
    r.h[0] = (uint32_t)d0 & 0x3ffffff;
    d1 += c;
    c = (uint32_t)(d1 >> 26);
    r.h[1] = (uint32_t)d1 & 0x3ffffff;
    d2 += c;
    c = (uint32_t)(d2 >> 26);
    r.h[2] = (uint32_t)d2 & 0x3ffffff;
    d3 += c;
    c = (uint32_t)(d3 >> 26);
    r.h[3] = (uint32_t)d3 & 0x3ffffff;
    d4 += c;
    c = (uint32_t)(d4 >> 26);
    r.h[4] = (uint32_t)d4 & 0x3ffffff;
    r.h[0] += c * 5;
    c = r.h[0] >> 26;
    r.h[0] &= 0x3ffffff;
    r.h[1] += c;
    return r;
}

__device__ __forceinline__ P130 padd(const P130 &a, const P130 &b) {
    P130 r;
#pragma unroll
    for (int i = 0; i < 5; i++) r.h[i] = a.h[i] + b.h[i];
    return r;
}

// full carry: every limb < 2^26
__device__ __forceinline__ P130 pnorm(P130 a) {
    for (int pass = 0; pass < 2; pass++) {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            a.h[i] += c;
            c = a.h[i] >> 26;
            a.h[i] &= 0x3ffffff;
        }
        a.h[0] += c * 5;
    }
    return a;
}

__device__ __forceinline__ P130 pone() { return P130{{1u, 0u, 0u, 0u, 0u}}; }

__device__ P130 ppow(const P130 &r, uint32_t e) {
    P130 acc = pone(), p = r;
    while (e) {
        if (e & 1u) acc = pmul(acc, p);
        e >>= 1;
        if (e) p = pmul(p, p);
    }
    return acc;
}

// a 16-byte block (little-endian words) + 2^128 as limbs
__device__ __forceinline__ P130 pblock(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
    return P130{{w0 & 0x3ffffff, ((w0 >> 26) | (w1 << 6)) & 0x3ffffff, ((w1 >> 20) | (w2 << 12)) & 0x3ffffff,
                 ((w2 >> 14) | (w3 << 18)) & 0x3ffffff, (w3 >> 8) | (1u << 24)}};
}

__device__ __forceinline__ void chacha_block(const uint32_t k[8], uint32_t ctr, const uint32_t nw[3], uint32_t o[16]) {
    uint32_t x[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                      k[4],        k[5],        k[6],        k[7],        ctr,  nw[0], nw[1], nw[2]};
#define QR(a, b, c, d)                   \
    x[a] += x[b], x[d] ^= x[a], x[d] = rotl(x[d], 16); \
    x[c] += x[d], x[b] ^= x[c], x[b] = rotl(x[b], 12); \
    x[a] += x[b], x[d] ^= x[a], x[d] = rotl(x[d], 8);  \
    x[c] += x[d], x[b] ^= x[c], x[b] = rotl(x[b], 7)
#pragma unroll
    for (int r = 0; r < 10; r++) {
        QR(0, 4, 8, 12);
        QR(1, 5, 9, 13);
        QR(2, 6, 10, 14);
        QR(3, 7, 11, 15);
        QR(0, 5, 10, 15);
        QR(1, 6, 11, 12);
        QR(2, 7, 8, 13);
        QR(3, 4, 9, 14);
    }
#undef QR
    const uint32_t init[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                               k[4],        k[5],        k[6],        k[7],        ctr,  nw[0], nw[1], nw[2]};
#pragma unroll
    for (int i = 0; i < 16; i++) o[i] = x[i] + init[i];
}

__device__ __forceinline__ uint32_t ld_le32(const gc_u8 *p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

__global__ __launch_bounds__(LANES) void chacha_kernel(const jfs_aead_block *__restrict__ blocks, int nblk, int mode,
                                                        int32_t *__restrict__ ret, const int32_t *__restrict__ lens) {
    __shared__ uint32_t sh_limb[5][LANES];
    __shared__ int32_t sh_ok;
    const int b = blockIdx.x;
    const int t = threadIdx.x;
    if (b >= nblk) return;
    jfs_aead_block blk = ((JFS_GLOBAL const jfs_aead_block *)blocks)[b];
    if (lens) {
        const int32_t ln = lens[b];
        if (ln <= 0) {
            if (t == 0) ret[b] = JFS_CHAIN_FAILED;
            return;
        }
        blk.src_len = ln;
    }
    const gc_u8 *src = (const gc_u8 *)blk.src;
    g_u8 *dst = (g_u8 *)blk.dst;
    const int64_t n = mode == 0 ? (int64_t)blk.src_len : (int64_t)blk.src_len - 16;
    const int64_t need = mode == 0 ? n + 16 : n;
    if (blk.src_len < 0 || n < 0 || (int64_t)blk.dst_cap < need || blk.key == nullptr || blk.nonce == nullptr) {
        if (t == 0) ret[b] = -2;
        return;
    }
    const gc_u8 *key = (const gc_u8 *)blk.key, *nonce = (const gc_u8 *)blk.nonce;
    uint32_t k[8], nw[3];
#pragma unroll
    for (int i = 0; i < 8; i++) k[i] = ld_le32(key + 4 * i);
#pragma unroll
    for (int i = 0; i < 3; i++) nw[i] = ld_le32(nonce + 4 * i);
    // the one-time Poly1305 key: ChaCha20 block 0; r clamped
    uint32_t otk[16];
    chacha_block(k, 0u, nw, otk);
    const P130 r = P130{{otk[0] & 0x3ffffff, ((otk[0] >> 26) | (otk[1] << 6)) & 0x3ffff03,
                         ((otk[1] >> 20) | (otk[2] << 12)) & 0x3ffc0ff, ((otk[2] >> 14) | (otk[3] << 18)) & 0x3f03fff,
                         (otk[3] >> 8) & 0x00fffff}};
    const int64_t nb16 = (n + 15) >> 4;  // ciphertext blocks; the lengths block is block nb16
    const P130 rgap = ppow(r, 4 * (LANES - 1) + 1);
    const bool aligned = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15u) == 0;
    P130 A = {{0, 0, 0, 0, 0}};
    int64_t last = -1;
    for (int64_t c = t; 64 * c < n; c += LANES) {
        uint32_t ks[16];
        chacha_block(k, (uint32_t)(c + 1), nw, ks);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int64_t o = 64 * c + 16 * q;
            if (o >= n) break;
            const int len = n - o < 16 ? (int)(n - o) : 16;
            const uint4 in = gcm::load_part(src + o, len, aligned);
            const uint4 out = make_uint4(in.x ^ ks[4 * q], in.y ^ ks[4 * q + 1], in.z ^ ks[4 * q + 2], in.w ^ ks[4 * q + 3]);
            gcm::store_part(dst + o, out, len, aligned);
            uint4 ct = mode == 0 ? out : in;
            if (len < 16) {  // the ciphertext is zero-padded to 16 bytes
                uint32_t w[4] = {ct.x, ct.y, ct.z, ct.w};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int keep = len - 4 * j;
                    w[j] = keep >= 4 ? w[j] : keep <= 0 ? 0u : (w[j] & (0xFFFFFFFFu >> (8 * (4 - keep))));
                }
                ct = make_uint4(w[0], w[1], w[2], w[3]);
            }
            const P130 m = pblock(ct.x, ct.y, ct.z, ct.w);
            const int64_t bi = 4 * c + q;
            A = last < 0 ? m : padd(pmul(A, q == 0 ? rgap : r), m);
            last = bi;
        }
    }
    P130 v = {{0, 0, 0, 0, 0}};
    if (last >= 0) v = pmul(A, ppow(r, (uint32_t)(nb16 + 1 - last)));
    if (t == 0) {  // the lengths block: le64(len(aad) = 0) || le64(len(ciphertext)), times r
        const P130 L = pblock(0u, 0u, (uint32_t)n, (uint32_t)((uint64_t)n >> 32));
        v = padd(v, pmul(L, r));
    }
    v = pnorm(v);
#pragma unroll
    for (int i = 0; i < 5; i++) sh_limb[i][t] = v.h[i];
    __syncthreads();
    if (t == 0) {
        uint64_t d[5];
        for (int i = 0; i < 5; i++) {
            uint64_t a = 0;
            for (int j = 0; j < LANES; j++) a += sh_limb[i][j];
            d[i] = a;
        }
        // carry the 64-bit limb sums, fold 2^130 = 5, then poly1305-donna's finish
        uint64_t c = 0;
        for (int pass = 0; pass < 3; pass++) {
            for (int i = 0; i < 5; i++) {
                d[i] += c;
                c = d[i] >> 26;
                d[i] &= 0x3ffffff;
            }
            d[0] += c * 5;
            c = 0;
        }
        uint32_t h0 = (uint32_t)d[0], h1 = (uint32_t)d[1], h2 = (uint32_t)d[2], h3 = (uint32_t)d[3], h4 = (uint32_t)d[4];
        uint32_t cc2 = h0 >> 26;
        h0 &= 0x3ffffff;
        h1 += cc2;
        uint32_t g0 = h0 + 5;
        cc2 = g0 >> 26;
        g0 &= 0x3ffffff;
        uint32_t g1 = h1 + cc2;
        cc2 = g1 >> 26;
        g1 &= 0x3ffffff;
        uint32_t g2 = h2 + cc2;
        cc2 = g2 >> 26;
        g2 &= 0x3ffffff;
        uint32_t g3 = h3 + cc2;
        cc2 = g3 >> 26;
        g3 &= 0x3ffffff;
        const uint32_t g4 = h4 + cc2 - (1u << 26);
        const uint32_t mask = (g4 >> 31) - 1u;
        h0 = (h0 & ~mask) | (g0 & mask);
        h1 = (h1 & ~mask) | (g1 & mask);
        h2 = (h2 & ~mask) | (g2 & mask);
        h3 = (h3 & ~mask) | (g3 & mask);
        h4 = (h4 & ~mask) | (g4 & mask);
        const uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14),
                       w3 = (h3 >> 18) | (h4 << 8);
        uint64_t f = (uint64_t)w0 + otk[4];
        uint32_t tag[4];
        tag[0] = (uint32_t)f;
        f = (uint64_t)w1 + otk[5] + (f >> 32);
        tag[1] = (uint32_t)f;
        f = (uint64_t)w2 + otk[6] + (f >> 32);
        tag[2] = (uint32_t)f;
        f = (uint64_t)w3 + otk[7] + (f >> 32);
        tag[3] = (uint32_t)f;
        if (mode == 0) {
            for (int j = 0; j < 16; j++) dst[n + j] = (uint8_t)(tag[j >> 2] >> (8 * (j & 3)));
            ret[b] = (int32_t)(n + 16);
        } else {
            uint32_t diff = 0;
            for (int j = 0; j < 16; j++) diff |= (uint32_t)src[n + j] ^ ((tag[j >> 2] >> (8 * (j & 3))) & 255u);
            ret[b] = diff ? -1 : (int32_t)n;
            sh_ok = diff == 0;
        }
    }
    if (mode == 1) {  // x/crypto's Open clears its output when the tag does not verify
        __syncthreads();
        if (!sh_ok)
            for (int64_t i = t; i < nb16; i += LANES) {
                const int len = n - 16 * i < 16 ? (int)(n - 16 * i) : 16;
                gcm::store_part(dst + 16 * i, make_uint4(0, 0, 0, 0), len, aligned);
            }
    }
}

}  // namespace cc
}  // namespace jfs

// cipher: JFS_CIPHER_*; mode 0 = seal, 1 = open; lens: see gcm_kernel
extern "C" int jfs_launch_aead(int cipher, const jfs_aead_block *d_blocks, int nblk, int mode, int32_t *d_ret,
                               const int32_t *d_lens, hipStream_t stream) {
    if (nblk <= 0) return 0;
    if (cipher == JFS_CIPHER_AES256GCM)
        hipLaunchKernelGGL(jfs::gcm::gcm_kernel<JFS_CIPHER_AES256GCM>, dim3(nblk), dim3(jfs::gcm::LANES), 0, stream,
                           d_blocks, nblk, mode, d_ret, d_lens);
    else if (cipher == JFS_CIPHER_SM4GCM)
        hipLaunchKernelGGL(jfs::gcm::gcm_kernel<JFS_CIPHER_SM4GCM>, dim3(nblk), dim3(jfs::gcm::LANES), 0, stream,
                           d_blocks, nblk, mode, d_ret, d_lens);
    else if (cipher == JFS_CIPHER_CHACHA20POLY1305)
        hipLaunchKernelGGL(jfs::cc::chacha_kernel, dim3(nblk), dim3(jfs::cc::LANES), 0, stream, d_blocks, nblk, mode,
                           d_ret, d_lens);
    else
        return -1;
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jfs_launch_aes256gcm(const jfs_aead_block *d_blocks, int nblk, int mode, int32_t *d_ret,
                                    const int32_t *d_lens, hipStream_t stream) {
    return jfs_launch_aead(JFS_CIPHER_AES256GCM, d_blocks, nblk, mode, d_ret, d_lens, stream);
}
