// AES-256-GCM seal / open of device-resident blocks for gfx950 -- SURVEY.md
// section 8(f)3, the AEAD JuiceFS applies to every object right after
// compression (pkg/object/encrypt.go:178-189 aes.NewCipher + cipher.NewGCM;
// Encrypt :226-257 aead.Seal(p[:0], nonce, plaintext, nil), Decrypt :259-284
// aead.Open).  12-byte nonce, 16-byte tag, no additional data.  The per-object
// key wrap (RSA / SM2 of the random data key, :234-237) and the object header
// (:244-252) stay on the host: a few hundred bytes per object.
// CPU restatement (test infrastructure): oracle/aes_gcm_oracle.c.
//
// One workgroup of 256 lanes per block.  Lane t takes the 16-byte AES blocks
// t, t+256, t+512, ... (every row of 4 KiB is one coalesced read and write):
//   CTR:   C_i = P_i ^ AES_K(nonce || be32(i + 2)), T-tables in LDS;
//   GHASH: Y_m = sum_i C_i * H^(m+1-i) over GF(2^128).  Each lane folds its
//          blocks by Horner with the constant H^256 (multiply by a constant =
//          16 lookups in a 256-entry table of b*H^256 built per block), then
//          multiplies its sum by H^(m - i_last) and the lanes XOR-reduce;
//          tag = AES_K(J0) ^ (Y_m ^ L) * H,  L = bit lengths (0 || 8n).
// Elements of GF(2^128) are held as four big-endian words (GCM bit order:
// the first bit of the block is the x^0 coefficient = the MSB of word 0).
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

struct Tables {
    uint32_t te[4][256];  // T-tables: te[0][x] = (2s, s, s, 3s) as a big-endian word, te[k] = te[0] rotated right 8k
    uint32_t sb[256];     // S-box (a word per entry: no sub-dword LDS reads)
    uint32_t r8[256];     // GHASH: top 16 bits added when a byte d is shifted out by a multiply by x^8
};

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
    return T;
}

__constant__ Tables g_tab = make_tables();

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
__global__ __launch_bounds__(LANES) void gcm_kernel(const jfs_aead_block *__restrict__ blocks, int nblk, int mode,
                                                     int32_t *__restrict__ ret, const int32_t *__restrict__ lens) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    const int t = threadIdx.x, l = t & 63, wv = t >> 6;
    {
        const uint32_t *g = (const uint32_t *)&g_tab;
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
    if (t == 0) {  // AES-256 key expansion (FIPS-197 5.2, Nk = 8)
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
        aes_enc(s, h0, h1, h2, h3);
        G128 H = {{h0, h1, h2, h3}};
        s.H = H;
        uint32_t j0 = n0, j1 = n1, j2 = n2, j3 = 1;
        aes_enc(s, j0, j1, j2, j3);
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
        aes_enc(s, k0, k1, k2, k3);
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
}  // namespace jfs

extern "C" int jfs_launch_aes256gcm(const jfs_aead_block *d_blocks, int nblk, int mode, int32_t *d_ret,
                                    const int32_t *d_lens, hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::gcm::gcm_kernel, dim3(nblk), dim3(jfs::gcm::LANES), 0, stream, d_blocks, nblk, mode, d_ret,
                       d_lens);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
