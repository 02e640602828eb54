// LZ4 block encoder for gfx950 -- byte-identical to LZ4_compress_default.
//
// Replaces LZ4_compress_default reached from pkg/compress/compress.go:115-117
// (LZ4.Compress -> lz4.CompressDefault(src, dst)).  The parse rules (hash
// tables, acceleration skip schedule, catch-up, immediate re-match) are the
// ones restated in oracle/lz4_oracle.c and SURVEY.md section 8a.
//
// The greedy parse is inherently serial (every table update depends on every
// earlier decision), so one wavefront owns one block and runs the parse with
// wave-uniform control flow; the 64 lanes do the byte-parallel parts: match
// extension (64 bytes per compare + ballot), backward catch-up, literal
// copies and table clears.  Throughput comes from running thousands of blocks
// at once (8 wavefronts per CU).  Output is staged in an LDS ring and written
// to HBM with wide stores; nothing is written at or beyond dst_cap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4e {

constexpr int64_t kMaxInput = 0x7E000000;
constexpr int OB = 4096;  // output staging ring
constexpr int OBMASK = OB - 1;
constexpr int OFLUSH = 2048;

struct Smem {
    alignas(16) uint32_t table[4096];  // byU32 view; byU16 view is the same 16 KiB
    alignas(16) uint8_t ob[OB];
};

struct Enc {
    const gc_u8 *src;
    g_u8 *dst;
    int64_t n, cap;
    int64_t op;  // output bytes produced
    int64_t F;   // flushed up to
    uint32_t dmis;
};

__device__ __forceinline__ uint32_t ld32u(const gc_u8 *p) {
    uintptr_t a = (uintptr_t)p;
    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)(a & 3);
    uint32_t w0 = w[0];
    if (sh == 0) return w0;
    uint32_t w1 = w[1];
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}

__device__ __forceinline__ uint64_t ld64u(const gc_u8 *p) {
    uintptr_t a = (uintptr_t)p;
    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
    uint32_t sh = (uint32_t)(a & 3);
    uint32_t w0 = w[0], w1 = w[1];
    if (sh == 0) return (uint64_t)w0 | ((uint64_t)w1 << 32);
    uint32_t w2 = w[2];
    uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
    uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

__device__ __forceinline__ uint32_t hpos(const gc_u8 *p, bool u16) {
    if (u16) return (ld32u(p) * 2654435761u) >> 19;
    return (uint32_t)(((ld64u(p) << 24) * 889523592379ull) >> 52);
}

__device__ __forceinline__ uint32_t tget(const Smem &s, uint32_t h, bool u16) {
    return u16 ? (uint32_t)((const uint16_t *)s.table)[h] : s.table[h];
}
__device__ __forceinline__ void tput(Smem &s, uint32_t h, uint32_t v, bool u16) {
    if (u16) ((uint16_t *)s.table)[h] = (uint16_t)v;
    else s.table[h] = v;
}

// staging slot of output position x (mirrors HBM 16-byte alignment)
__device__ __forceinline__ uint32_t obidx(const Enc &e, int64_t x) { return (uint32_t)((x + e.dmis) & OBMASK); }

__device__ __forceinline__ void oflush2(Smem &s, Enc &e, int64_t to) {
    const int l = lane_id();
    if (to > e.cap) to = e.cap;
    int64_t F = e.F;
    if (to <= F) return;
    int64_t a = F + (int64_t)((16u - ((e.dmis + (uint32_t)F) & 15u)) & 15u);
    if (a > to) a = to;
    if (l < a - F) e.dst[F + l] = s.ob[obidx(e, F + l)];
    int64_t b = a + ((to - a) & ~(int64_t)15);
    for (int64_t x = a + 16 * l; x < b; x += 1024) *(g_u4 *)(e.dst + x) = *(const uint4 *)(s.ob + obidx(e, x));
    if (l < to - b) e.dst[b + l] = s.ob[obidx(e, b + l)];
    e.F = to;
}

__device__ __forceinline__ void maybe_flush(Smem &s, Enc &e, int64_t keep_from) {
    // flush everything below min(op, keep_from) once enough is pending
    int64_t lim = e.op < keep_from ? e.op : keep_from;
    if (lim - e.F >= OFLUSH) {
        int64_t to = ((lim + e.dmis) & ~(int64_t)15) - e.dmis;
        oflush2(s, e, to);
    }
}

// one byte written by lane 0 (uniform position)
__device__ __forceinline__ void put1(Smem &s, Enc &e, uint32_t v) {
    if (lane_id() == 0) s.ob[obidx(e, e.op)] = (uint8_t)v;
    e.op++;
}

__device__ __forceinline__ void put_len(Smem &s, Enc &e, uint32_t len) {
    // 255-run then remainder; lanes write the run in parallel
    const int l = lane_id();
    uint32_t runs = len / 255;
    for (uint32_t k = 0; k < runs; k += 64) {
        if (k + l < runs) s.ob[obidx(e, e.op + l)] = 255;
        e.op += (runs - k < 64 ? runs - k : 64);
        maybe_flush(s, e, INT64_MAX);
    }
    put1(s, e, len % 255);
}

// copy literals src[from, from+len) into the output
__device__ __forceinline__ void put_lits(Smem &s, Enc &e, int64_t from, int64_t len, int64_t keep_from) {
    const int l = lane_id();
    for (int64_t k = 0; k < len; k += 64) {
        maybe_flush(s, e, keep_from);
        if (e.op + 64 - e.F > OB) {
            // token pending too far back: flush past it; the token is patched in HBM
            int64_t to = ((e.op + e.dmis) & ~(int64_t)15) - e.dmis;
            oflush2(s, e, to);
        }
        int64_t i = k + l;
        if (i < len) s.ob[obidx(e, e.op + l)] = e.src[from + i];
        e.op += (len - k < 64 ? len - k : 64);
    }
}

// set the token byte at output position tp
__device__ __forceinline__ void put_token(Smem &s, Enc &e, int64_t tp, uint32_t v) {
    if (lane_id() == 0) {
        if (tp >= e.F) s.ob[obidx(e, tp)] = (uint8_t)v;
        else if (tp < e.cap) e.dst[tp] = (uint8_t)v;
    }
}

__global__ __launch_bounds__(64) void lz4_encode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                       int32_t *__restrict__ ret) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    if (b >= nblk) return;
    const int l = lane_id();
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    Enc e;
    e.src = (const gc_u8 *)d.src;
    e.dst = (g_u8 *)d.dst;
    e.n = d.src_len;
    e.cap = d.dst_cap;
    e.op = 0;
    e.F = 0;
    e.dmis = (uint32_t)((uintptr_t)d.dst & 15u);
    const gc_u8 *src = e.src;
    const int64_t n = e.n;
    int32_t result;
    if (n < 0 || n > kMaxInput) {
        result = 0;
    } else if (n == 0) {
        if (e.cap <= 0) result = 0;
        else {
            if (l == 0) e.dst[0] = 0;
            result = 1;
        }
    } else {
        const bool u16 = n < 65536 + 12 - 1;
        for (int k = l; k < 4096; k += 64) s.table[k] = 0;
        __builtin_amdgcn_wave_barrier();
        const int64_t mflimitP1 = n - 12 + 1, matchlimit = n - 5;
        int64_t ip = 0, anchor = 0;
        if (n >= 13) {
            tput(s, hpos(src, u16), 0, u16);
            ip = 1;
            uint32_t fh = hpos(src + ip, u16);
            for (;;) {
                int64_t match;
                // ---- search (skip schedule: step = searchMatchNb++ >> 6)
                {
                    int64_t fip = ip;
                    int32_t step = 1, snb = 1 << 6;
                    bool last = false;
                    for (;;) {
                        uint32_t h = fh;
                        int64_t cur = fip;
                        uint32_t mi = tget(s, h, u16);
                        ip = fip;
                        fip += step;
                        step = snb++ >> 6;
                        if (fip > mflimitP1) { last = true; break; }
                        match = mi;
                        fh = hpos(src + fip, u16);
                        tput(s, h, (uint32_t)cur, u16);
                        if (!u16 && (int64_t)mi + 65535 < cur) continue;
                        if (ld32u(src + match) == ld32u(src + ip)) break;
                    }
                    if (last) break;
                }
                // ---- catch up (backwards, 64 bytes per step)
                {
                    int64_t lim = ip - anchor;
                    if (match < lim) lim = match;
                    int64_t back = 0;
                    while (back < lim) {
                        int64_t k = back + 1 + l;
                        bool eq = k <= lim && src[ip - k] == src[match - k];
                        uint64_t ne = ~__ballot(eq);
                        int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        back += run;
                        if (run < 64) break;
                    }
                    if (back > lim) back = lim;
                    ip -= back;
                    match -= back;
                }
                // ---- literals
                int64_t tp = e.op;
                uint32_t token;
                {
                    int64_t lit = ip - anchor;
                    e.op++;  // token slot
                    if (lit >= 15) { token = 15u << 4; put_len(s, e, (uint32_t)(lit - 15)); }
                    else token = (uint32_t)lit << 4;
                    put_lits(s, e, anchor, lit, tp);
                }
                for (;;) {  // next_match
                    uint32_t off = (uint32_t)(ip - match);
                    put1(s, e, off & 255);
                    put1(s, e, off >> 8);
                    // match length: count equal bytes from ip+4 / match+4 up to matchlimit
                    int64_t a0 = ip + 4, b0 = match + 4;
                    int64_t mc = 0;
                    for (;;) {
                        int64_t a = a0 + mc + l;
                        bool eq = a < matchlimit && src[a] == src[b0 + mc + l];
                        uint64_t ne = ~__ballot(eq);
                        int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        mc += run;
                        if (run < 64) break;
                    }
                    ip = a0 + mc;
                    if (mc >= 15) {
                        token += 15;
                        put_len(s, e, (uint32_t)(mc - 15));
                    } else {
                        token += (uint32_t)mc;
                    }
                    put_token(s, e, tp, token);
                    maybe_flush(s, e, INT64_MAX);
                    anchor = ip;
                    if (ip >= mflimitP1) break;
                    tput(s, hpos(src + ip - 2, u16), (uint32_t)(ip - 2), u16);
                    uint32_t h = hpos(src + ip, u16);
                    uint32_t mi = tget(s, h, u16);
                    tput(s, h, (uint32_t)ip, u16);
                    if ((u16 || (int64_t)mi + 65535 >= ip) && ld32u(src + mi) == ld32u(src + ip)) {
                        match = mi;
                        tp = e.op;
                        e.op++;
                        token = 0;
                        continue;
                    }
                    break;
                }
                if (anchor >= mflimitP1) break;
                ++ip;
                fh = hpos(src + ip, u16);
            }
        }
        // ---- last literals
        {
            int64_t lastrun = n - anchor;
            int64_t tp = e.op;
            e.op++;
            uint32_t token;
            if (lastrun >= 15) { token = 15u << 4; put_len(s, e, (uint32_t)(lastrun - 15)); }
            else token = (uint32_t)lastrun << 4;
            put_lits(s, e, anchor, lastrun, tp);
            put_token(s, e, tp, token);
        }
        if (e.op > e.cap) {
            result = 0;
        } else {
            oflush2(s, e, e.op);
            result = (int32_t)e.op;
        }
    }
    if (l == 0) ret[b] = result;
}

}  // namespace lz4e
}  // namespace jfs

extern "C" int jfs_launch_lz4_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4e::lz4_encode_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
