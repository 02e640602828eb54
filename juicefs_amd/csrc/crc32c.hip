// CRC-32C (Castagnoli) of device-resident blocks for gfx950 -- SURVEY.md
// section 8(f)4, the checksums JuiceFS computes over the same buffers the codec
// touches:
//   pkg/object/checksum.go:30-45        object checksum = crc32.Update(0, crc32c, data)
//   pkg/chunk/disk_cache_file.go:139-152 disk-cache checksum(): crc32.Checksum of
//                                       every 32 KiB (csBlock) piece, big-endian
//                                       (utils.Buffer.Put32, buffer.go:42,102)
// CPU restatement (test infrastructure): oracle/crc32c_oracle.c.
//
// One workgroup of 256 lanes per block; the block is walked in segments of
// S = 4096 * rows bytes (32 KiB for the disk-cache layout).  Lane t owns the
// 16-byte chunks at 4096 r + 16 t of a segment (row r): every row is one fully
// coalesced 4 KiB read.  CRC is linear over GF(2): with raw(D) = the CRC of D
// from a zero register,
//     raw(A || B) = raw(A) * x^(8|B|) + raw(B)        (mod P, reflected)
// so lane t folds its rows by Horner (A <- A * x^(8*4096) + raw(chunk), the
// multiply by a constant done with four 256-entry tables), the segment is the
// XOR over lanes of A_t * x^(8*16*(255-t)), and the block is the Horner fold of
// its segments.  raw(chunk) uses slicing-by-8 tables; all tables (13 KiB) are
// compile-time constants copied to LDS.  A segment shorter than S (the block
// tail) is front-padded with zero bytes, which leaves raw() unchanged.
// Standard value: crc(D) = ~(raw(D) ^ (~0 * x^(8|D|))).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace crc {

constexpr uint32_t POLY = 0x82F63B78u;  // reflected Castagnoli
constexpr uint32_t ONE = 0x80000000u;   // x^0 in the reflected representation
constexpr int LANES = 256;
constexpr int ROW = LANES * 16;  // 4096 bytes per row

// a * b mod P (reflected; zlib's multmodp)
__host__ __device__ constexpr uint32_t mulp(uint32_t a, uint32_t b) {
    uint32_t p = 0;
    for (int i = 0; i < 32; i++) {
        if (a & (ONE >> i)) p ^= b;
        b = (b & 1u) ? (b >> 1) ^ POLY : b >> 1;
    }
    return p;
}

struct Tables {
    uint32_t slice[8][256];  // slicing-by-8: slice[k][b] = raw of byte b followed by k zero bytes
    uint32_t row[4][256];    // multiply by x^(8*ROW): row[j][b] = mulp(X_ROW, b << 8j)
    uint32_t lane[LANES];    // x^(8*16*(255-t))
    uint32_t x2k[64];        // x^(2^k)
};

constexpr Tables make_tables() {
    Tables T{};
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ POLY : c >> 1;
        T.slice[0][b] = c;
    }
    for (int k = 1; k < 8; k++)
        for (uint32_t b = 0; b < 256; b++)
            T.slice[k][b] = (T.slice[k - 1][b] >> 8) ^ T.slice[0][T.slice[k - 1][b] & 0xFFu];
    uint32_t x = ONE >> 1;  // x^1
    for (int k = 0; k < 64; k++) {
        T.x2k[k] = x;
        x = mulp(x, x);
    }
    // x^(8*ROW) = x^(2^15) (ROW = 4096 bytes = 2^15 bits)
    const uint32_t xrow = T.x2k[15];
    for (int j = 0; j < 4; j++)
        for (uint32_t b = 0; b < 256; b++) T.row[j][b] = mulp(xrow, b << (8 * j));
    // lane t: x^(8*16*(255-t)) = x^(128*(255-t))
    const uint32_t x128 = T.x2k[7];
    uint32_t v = ONE;
    for (int t = LANES - 1; t >= 0; t--) {
        T.lane[t] = v;
        v = mulp(v, x128);
    }
    return T;
}

__constant__ Tables g_tab = make_tables();

// x^(8n) mod P from the x^(2^k) table
__device__ __forceinline__ uint32_t xpow8(const Tables &T, uint64_t n) {
    uint32_t r = ONE;
    n <<= 3;
    for (int k = 0; n; k++, n >>= 1)
        if (n & 1) r = mulp(r, T.x2k[k]);
    return r;
}

// raw CRC of 16 bytes (four little-endian dwords) from a zero register
__device__ __forceinline__ uint32_t raw16(const Tables &T, uint4 w) {
    uint32_t c = T.slice[7][w.x & 0xFF] ^ T.slice[6][(w.x >> 8) & 0xFF] ^ T.slice[5][(w.x >> 16) & 0xFF] ^
                 T.slice[4][w.x >> 24] ^ T.slice[3][w.y & 0xFF] ^ T.slice[2][(w.y >> 8) & 0xFF] ^
                 T.slice[1][(w.y >> 16) & 0xFF] ^ T.slice[0][w.y >> 24];
    const uint32_t z = c ^ w.z;
    return T.slice[7][z & 0xFF] ^ T.slice[6][(z >> 8) & 0xFF] ^ T.slice[5][(z >> 16) & 0xFF] ^ T.slice[4][z >> 24] ^
           T.slice[3][w.w & 0xFF] ^ T.slice[2][(w.w >> 8) & 0xFF] ^ T.slice[1][(w.w >> 16) & 0xFF] ^
           T.slice[0][w.w >> 24];
}

__device__ __forceinline__ uint32_t mul_row(const Tables &T, uint32_t a) {
    return T.row[0][a & 0xFF] ^ T.row[1][(a >> 8) & 0xFF] ^ T.row[2][(a >> 16) & 0xFF] ^ T.row[3][a >> 24];
}

// 16 bytes [p, p+16) of which only [lo, hi) (absolute positions) are real;
// the rest read as zero.  Byte loads: used for the block's ragged edges and
// for sources that are not 16-byte aligned.
__device__ __forceinline__ uint4 load_masked(const gc_u8 *src, int64_t p, int64_t lo, int64_t hi) {
    uint32_t d[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const int64_t q = p + i;
        const uint32_t b = (q >= lo && q < hi) ? (uint32_t)src[q] : 0u;
        d[i >> 2] |= b << (8 * (i & 3));
    }
    return make_uint4(d[0], d[1], d[2], d[3]);
}

// Shared by the lanes of one workgroup: tables + the cross-wave reduction.
struct Smem {
    Tables T;
    uint32_t part[LANES / 64];
};

// lens (optional): per-block lengths produced on the device by the previous
// kernel (the codec's or the AEAD's result; <= 0 = it failed: crc 0);
// seeds (optional): crc32.Update(seed, crc32c, data) instead of seed 0.
__global__ __launch_bounds__(LANES) void crc32c_kernel(const jfs_dev_block *__restrict__ blocks, int nblk, int32_t rows,
                                                        int32_t emit_segments, uint32_t *__restrict__ crc_out,
                                                        int32_t *__restrict__ ret, const int32_t *__restrict__ lens,
                                                        const uint32_t *__restrict__ seeds) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    const int t = threadIdx.x, l = t & 63, w = t >> 6;
    {  // constant tables -> LDS
        const uint32_t *g = (const uint32_t *)&g_tab;
        uint32_t *d = (uint32_t *)&s.T;
        for (int i = t; i < (int)(sizeof(Tables) / 4); i += LANES) d[i] = g[i];
    }
    __syncthreads();
    if (b >= nblk) return;
    const Tables &T = s.T;
    const jfs_dev_block blk = ((const gc_blk *)blocks)[b];
    const gc_u8 *src = (const gc_u8 *)blk.src;
    g_u8 *out = (g_u8 *)blk.dst;
    const int64_t n = lens ? (int64_t)lens[b] : (int64_t)blk.src_len;
    const uint32_t seed = seeds ? seeds[b] : 0u;
    if (lens && (emit_segments ? n < 0 : n <= 0)) {  // the producing kernel failed (or, for a payload, wrote nothing)
        if (t == 0 && crc_out) crc_out[b] = 0;
        return;
    }
    const int64_t S = (int64_t)rows * ROW;
    const int64_t words = n > 0 ? (n - 1) / S + 1 : 1;  // Go's ((len-1)/csBlock+1), 1 word for len 0
    if (n < 0 || (emit_segments && (out == nullptr || (int64_t)blk.dst_cap < 4 * words))) {
        if (t == 0) {
            if (ret) ret[b] = -1;
            if (crc_out) crc_out[b] = 0;
        }
        return;
    }
    const bool aligned = (((uintptr_t)src) & 15u) == 0;
    const uint32_t xS = xpow8(T, (uint64_t)S);  // segment shift (same value in every lane)
    const uint32_t laneK = T.lane[t];
    uint32_t total = 0;  // raw CRC of the block so far (meaningful in lane 0)
    for (int64_t s0 = 0; s0 < n; s0 += S) {
        const int64_t e = s0 + S < n ? s0 + S : n;
        const int64_t len = e - s0;
        const int64_t v0 = e - S;  // virtual segment start: front-padded with zeros when len < S
        const bool fast = aligned && len == S;
        uint32_t A = 0;
        for (int r = 0; r < rows; r += 8) {
            const int nr = rows - r < 8 ? rows - r : 8;
            uint4 c[8];
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (k < nr) {
                    const int64_t p = v0 + (int64_t)(r + k) * ROW + 16 * t;
                    if (fast) c[k] = *(const gc_u4 *)(src + p);
                    else if (p + 16 <= s0) c[k] = make_uint4(0, 0, 0, 0);
                    else c[k] = load_masked(src, p, s0, e);
                }
            }
#pragma unroll
            for (int k = 0; k < 8; k++)
                if (k < nr) A = mul_row(T, A) ^ raw16(T, c[k]);
        }
        // segment raw CRC = XOR over lanes of A_t * x^(8*16*(255-t))
        uint32_t v = mulp(A, laneK);
        v ^= (uint32_t)__shfl_xor((int)v, 32, 64);
        v ^= (uint32_t)__shfl_xor((int)v, 16, 64);
        v ^= (uint32_t)__shfl_xor((int)v, 8, 64);
        v ^= (uint32_t)__shfl_xor((int)v, 4, 64);
        v ^= (uint32_t)__shfl_xor((int)v, 2, 64);
        v ^= (uint32_t)__shfl_xor((int)v, 1, 64);
        if (l == 0) s.part[w] = v;
        __syncthreads();
        if (t == 0) {
            uint32_t seg = 0;
            for (int i = 0; i < LANES / 64; i++) seg ^= s.part[i];
            const uint32_t xl = len == S ? xS : xpow8(T, (uint64_t)len);
            total = mulp(total, xl) ^ seg;
            if (emit_segments) {
                const uint32_t std_v = ~(seg ^ mulp(0xFFFFFFFFu, xl));
                const int64_t o = 4 * (s0 / S);
                out[o] = (uint8_t)(std_v >> 24);
                out[o + 1] = (uint8_t)(std_v >> 16);
                out[o + 2] = (uint8_t)(std_v >> 8);
                out[o + 3] = (uint8_t)std_v;
            }
        }
        __syncthreads();
    }
    if (t == 0) {
        if (n == 0 && emit_segments) out[0] = out[1] = out[2] = out[3] = 0;
        if (crc_out) crc_out[b] = n == 0 ? seed : ~(total ^ mulp(~seed, xpow8(T, (uint64_t)n)));
        if (ret) ret[b] = emit_segments ? (int32_t)(4 * words) : 0;
    }
}

}  // namespace crc
}  // namespace jfs

extern "C" int jfs_launch_crc32c(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes, uint32_t *d_crc,
                                 int32_t *d_ret, hipStream_t stream) {
    using namespace jfs::crc;
    if (nblk <= 0) return 0;
    const int emit = seg_bytes > 0;
    const int32_t S = emit ? seg_bytes : (32 << 10);
    if (S % ROW != 0 || S > (64 << 20)) return -1;
    hipLaunchKernelGGL(crc32c_kernel, dim3(nblk), dim3(LANES), 0, stream, d_blocks, nblk, S / ROW, emit, d_crc, d_ret,
                       (const int32_t *)nullptr, (const uint32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// whole-block CRC-32C of device blocks whose length the previous kernel wrote
// (lens), continuing from per-block seeds (the host path's PUT payloads)
extern "C" int jfs_launch_crc32c_lens(const jfs_dev_block *d_blocks, int nblk, const int32_t *d_lens,
                                      const uint32_t *d_seeds, uint32_t *d_crc, hipStream_t stream) {
    using namespace jfs::crc;
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(crc32c_kernel, dim3(nblk), dim3(LANES), 0, stream, d_blocks, nblk, (32 << 10) / ROW, 0, d_crc,
                       (int32_t *)nullptr, d_lens, d_seeds);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jfs_launch_crc32c_segs_lens(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes,
                                           const int32_t *d_lens, hipStream_t stream) {
    using namespace jfs::crc;
    if (nblk <= 0) return 0;
    if (seg_bytes <= 0 || seg_bytes % ROW != 0 || seg_bytes > (64 << 20)) return -1;
    hipLaunchKernelGGL(crc32c_kernel, dim3(nblk), dim3(LANES), 0, stream, d_blocks, nblk, seg_bytes / ROW, 1,
                       (uint32_t *)nullptr, (int32_t *)nullptr, d_lens, (const uint32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
