// Zstd level-1 frame encoder for gfx950, byte-identical to libzstd's
// ZSTD_compress(dst, cap, src, n, 1).
//
// Replaces ZStandard.Compress (pkg/compress/compress.go:82-91 ->
// zstd.CompressLevel(dst, src, 1) of github.com/DataDog/zstd).  The reference
// pins v1.5.6, which is not available offline; the frames here are pinned to
// libzstd 1.4.9 (the library of this image) through oracle/zstd_l1_oracle.c
// and the committed fixtures.  The rules restated are
// libzstd's: ZSTD_getCParams(1, n) + ZSTD_adjustCParams, ZSTD_compressBlock_fast
// (two positions per step, repeat offset at +2, skip step (d >> 7) + 2),
// ZSTD_compressBlock_internal (raw / RLE / compressed, repcode and entropy
// confirmation), ZSTD_compressLiterals + HUF_compress (table reuse), and
// ZSTD_entropyCompressSequences (FSE table choice, normalisation, bitstream).
//
// The kernels of a launch, the serial parts kept serial only where the format
// makes them so:
//   zl1_parse_kernel  one wave per FRAME: the greedy parse of every 128 KiB
//                     block in order (the hash table and repeat offsets carry
//                     across blocks); the hash table lives in LDS as 20-bit
//                     window-relative entries (40 KiB: four frames per CU);
//                     each search step tries the next 64 positions of the skip
//                     schedule at once (one per lane) and keeps exactly the
//                     serial loop's result.  Output: the blocks' sequences.
//   zl1_seq_kernel    one wave per BLOCK: gathers the block's literals (and
//                     their histograms per Huffman stream) and writes the
//                     complete sequences section (FSE tables + bitstream).
//   zl1_lithuf        one wave per BLOCK: the block's new Huffman table and
//                     its description;
//   zl1_litdec        one wave per FRAME, block after block: the literal
//                     section choice (table reuse decision, exact sizes), the
//                     raw / RLE / compressed choice and the block offsets;
//   zl1_litwrite      one wave per BLOCK: the block bytes written in place.
// Small batches (<= JFS_ZL1_SPEC_MAX blocks of multi-block frames) replace the
// frame-serial parse by zl1_spec_merge / zl1_spec_parse: every block parses at
// once from the prefix maxima of the other blocks' write sets, again until no
// block's inputs change -- the serial parse's result, by induction.
// A block that ends up raw or RLE does not pass its repeat offsets on
// (ZSTD_confirmRepcodesAndEntropyTables); the parse predicts that (RLE blocks
// are known exactly, others are assumed compressed) and the literal kernel
// checks the prediction: a frame whose wrong guess changed the offsets handed
// to the next block is parsed again with the now known outcomes (the host
// loop below; every pass settles at least one more block).
// ---------------------------------------------------------------------------
// Third-party notice.  Byte parity with libzstd forces its exact heuristics,
// so the following routines are transliterated from Zstandard (libzstd 1.4.9,
// https://github.com/facebook/zstd), Copyright (c) 2016-present, Yann Collet,
// Facebook, Inc.  All rights reserved.  Used under the BSD licence of that
// source tree:
//   FSE_normalizeCount and FSE_normalizeM2 (fse_compress.c), including its
//   rtbTable constants; FSE_writeNCount (fse_compress.c); HUF_setMaxHeight
//   and HUF_buildCTable_wksp (huf_compress.c).
// Redistribution and use in source and binary forms, with or without
// modification, are permitted provided that the following conditions are met:
//  * Redistributions of source code must retain the above copyright notice,
//    this list of conditions and the following disclaimer.
//  * Redistributions in binary form must reproduce the above copyright notice,
//    this list of conditions and the following disclaimer in the documentation
//    and/or other materials provided with the distribution.
//  * Neither the name Facebook nor the names of its contributors may be used to
//    endorse or promote products derived from this software without specific
//    prior written permission.
// THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS"
// AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
// IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE
// DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE
// FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL
// DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
// SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER
// CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY,
// OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE
// OF THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
// ---------------------------------------------------------------------------
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace zl1 {

constexpr int32_t BLK = 128 << 10;  // ZSTD_BLOCKSIZE_MAX
#ifndef JFS_ZL1_PB
#define JFS_ZL1_PB 64  // search iterations tried at once right after a match
#endif

// ---------------------------------------------------------------------------
// parameters: ZSTD_getCParams(1, n, 0) (level-1 row of the size tier, then
// ZSTD_adjustCParams_internal); strategy fast, targetLength 0 (step 2)
// ---------------------------------------------------------------------------
struct Params {
    uint32_t wlog, hlog, mls;
};
__host__ __device__ inline uint32_t hbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }
__host__ __device__ inline Params params_of(int64_t n) {
    Params p;
    if (n > (256 << 10)) { p.wlog = 19; p.hlog = 14; p.mls = 7; }
    else if (n > (128 << 10)) { p.wlog = 18; p.hlog = 14; p.mls = 6; }
    else if (n > (16 << 10)) { p.wlog = 17; p.hlog = 13; p.mls = 6; }
    else { p.wlog = 14; p.hlog = 15; p.mls = 5; }
    const uint32_t t = (uint32_t)n;
    const uint32_t srclog = t < 64 ? 6u : hbit(t - 1) + 1;
    if (p.wlog > srclog) p.wlog = srclog;
    if (p.hlog > p.wlog + 1) p.hlog = p.wlog + 1;
    if (p.wlog < 10) p.wlog = 10;
    return p;
}
__host__ __device__ inline int64_t zbound(int64_t n) { return n + (n >> 8) + (n < BLK ? (BLK - n) >> 11 : 0); }

// per frame / per block records (host-built, device-updated)
struct FInfo {
    const uint8_t *src;
    uint8_t *dst;
    int32_t n, cap;
    int32_t nb, b0;  // blocks, index of the first in the block array
    uint32_t wlog, hlog, mls;
    int32_t status;  // 0 done, 1 parse again (a confirmation guess was wrong), -2 dst too small
};
enum : int32_t { F_NOCOMP = 1, F_RLE = 2, F_ASSUMED = 4, F_LASTNC = 8 };
struct BInfo {
    int64_t seq_off;  // u64 records in the sequence scratch
    int64_t lit_off;  // bytes: literals (bsz), then the sequences section (bsz + 512)
    int32_t frame, bs, be;
    int32_t ns, nl;                    // sequences, literals
    uint32_t rin0, rin1, rout0, rout1;  // repeat offsets in / out (offset_1, offset_2)
    int32_t flags;
    int32_t conf;   // outcome known from an earlier pass: 0 unknown, 1 confirmed, 2 not
    int32_t secsz;  // sequences section bytes, -1 = larger than the block
};
constexpr int64_t SEC_EXTRA = 512;
__host__ __device__ inline int64_t seq_cap(int32_t bsz) { return bsz / 4 + 4; }

// sequence record: ll | mlb << 17 | Offset_Value << 34
__device__ __forceinline__ uint64_t seq_pack(uint32_t ll, uint32_t mlb, uint32_t ofv) {
    return (uint64_t)ll | ((uint64_t)mlb << 17) | ((uint64_t)ofv << 34);
}

// ---------------------------------------------------------------------------
// source access through a buffer resource: the descriptor covers exactly the
// dwords that hold input bytes, so every load is range-checked by the
// hardware (out-of-range dwords read 0, nothing past the input is touched)
// and needs only a 32-bit offset -- no per-load guards or 64-bit address math
// ---------------------------------------------------------------------------
struct Src {
    __amdgpu_buffer_rsrc_t r;
    int32_t sh;  // input byte 0 sits at byte sh of the first dword
};
__device__ __forceinline__ Src make_src(const uint8_t *p, int32_t n) {
    Src s;
    const uintptr_t a = (uintptr_t)p;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)(a & ~(uintptr_t)3));
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    s.sh = (int32_t)__builtin_amdgcn_readfirstlane((uint32_t)(a & 3u));
    const int32_t nb = n > 0 ? (int32_t)((n + s.sh + 3) & ~3) : 0;
    s.r = __builtin_amdgcn_make_buffer_rsrc((void *)(((uintptr_t)hi << 32) | lo), 0,
                                            (int)__builtin_amdgcn_readfirstlane((uint32_t)nb), 0x00020000);
    return s;
}
__device__ __forceinline__ uint32_t ldw(const Src &S, int32_t byteoff) {
    return __builtin_amdgcn_raw_buffer_load_b32(S.r, (uint32_t)byteoff, 0, 0);
}
// byte at position p
__device__ __forceinline__ uint32_t ldb(const Src &S, int32_t p) {
    return __builtin_amdgcn_raw_buffer_load_b8(S.r, (uint32_t)(p + S.sh), 0, 0);
}
// 16 bytes at position p (p >= -3; bytes before the input read 0).  A
// negative offset must never reach a buffer instruction: the compiler merges
// the five loads into wider ones and the whole merged load would read 0.
__device__ __forceinline__ uint4 ld128(const Src &S, int32_t p) {
    const int32_t b = p + S.sh;
    const int32_t o = b & ~3;
    const uint32_t s = (uint32_t)b & 3u;
    const bool neg = o < 0;
    const int32_t oc = neg ? 0 : o;
    uint32_t w0 = ldw(S, oc), w1 = ldw(S, oc + 4), w2 = ldw(S, oc + 8), w3 = ldw(S, oc + 12), w4 = ldw(S, oc + 16);
    if (neg) {  // o == -4: the words are one dword later than loaded
        w4 = w3;
        w3 = w2;
        w2 = w1;
        w1 = w0;
        w0 = 0;
    }
    uint4 r;
    r.x = __builtin_amdgcn_alignbyte(w1, w0, s);
    r.y = __builtin_amdgcn_alignbyte(w2, w1, s);
    r.z = __builtin_amdgcn_alignbyte(w3, w2, s);
    r.w = __builtin_amdgcn_alignbyte(w4, w3, s);
    return r;
}

#ifdef JFS_PROF
// diagnostic build only: per-phase s_memtime sums of the parse waves
// (0 positions + windows + hashes, 1 after-match inserts + repeat loop, 2 table
// reads + bucket tags, 3 candidate loads + decision, 4 table writes, 5 match
// extension, 6 block setup (RLE scan, window refresh); 8 sequences, 9 search
// steps, 10 extension round trips, 11 blocks)
__device__ unsigned long long g_zpprof[12];
#define ZP_DECL uint64_t zp_t = __builtin_amdgcn_s_memtime(), zp_acc[12] = {0};
#define ZP(k) do { const uint64_t x_ = __builtin_amdgcn_s_memtime(); zp_acc[k] += x_ - zp_t; zp_t = x_; } while (0)
#define ZPC(k) (zp_acc[k] += 1)
#define ZP_FLUSH() do { if (lane_id() == 0) for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_zpprof[i_], (unsigned long long)zp_acc[i_]); } while (0)
#else
#define ZP_DECL
#define ZP(k) do { } while (0)
#define ZPC(k) do { } while (0)
#define ZP_FLUSH() do { } while (0)
#endif

// ZSTD_hashPtr for minMatch 5 / 6 / 7 of the 8 little-endian bytes at a position
__device__ __forceinline__ uint32_t zhash(uint64_t v, uint32_t hlog, uint32_t mls) {
    const uint64_t prime = mls == 5 ? 889523592379ull : mls == 6 ? 227718039650203ull : 58295818150454627ull;
    return (uint32_t)(((v << (64 - 8 * mls)) * prime) >> (64 - hlog));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __ballot(p); }
__device__ __forceinline__ int ctz64(uint64_t m) { return m ? __builtin_ctzll(m) : 64; }

// ---------------------------------------------------------------------------
// hash table in LDS.  Entries hold index = position + 1 (0 = empty).  WIDE
// tables keep 20 bits (16 in lo[], 4 in a nibble array) and decode relative to
// the block end R: the entry is the unique index = e (mod 2^20) in
// (R - 2^20, R].  Entries that fall out of the 2^wlog window are rewritten as
// the window's lowest index at each block start, so every live entry is
// within 640 KiB of R and decodes exactly.  Narrow tables (frames < 64 KiB)
// keep the whole index in 16 bits.
// ---------------------------------------------------------------------------
template <bool WIDE>
struct Tab {
    uint16_t *lo;
    uint32_t *hi;
    __device__ __forceinline__ uint32_t raw(uint32_t h) const {
        return WIDE ? (uint32_t)lo[h] | (((hi[h >> 3] >> ((h & 7) * 4)) & 15u) << 16) : (uint32_t)lo[h];
    }
    __device__ __forceinline__ uint32_t get(uint32_t h, uint32_t R) const {
        const uint32_t e = raw(h);
        return WIDE ? R - ((R - e) & 0xFFFFFu) : e;
    }
    // fire-and-forget: a u16 store and two LDS atomics (clear, set) on the
    // nibble's dword, no read round trip; lanes sharing the dword touch
    // disjoint nibbles
    __device__ __forceinline__ void put(uint32_t h, uint32_t idx) {
        lo[h] = (uint16_t)idx;
        if (WIDE) {
            const uint32_t sh = (h & 7) * 4;
            (void)__hip_atomic_fetch_and(&hi[h >> 3], ~(15u << sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            (void)__hip_atomic_fetch_or(&hi[h >> 3], ((idx >> 16) & 15u) << sh, __ATOMIC_RELAXED,
                                        __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
};

// ---------------------------------------------------------------------------
// byte compares (wave-parallel)
// ---------------------------------------------------------------------------
// count of i in [0, lim) with s[a + i] == s[b + i] before the first mismatch
__device__ int32_t fwd_count(const Src &S, int32_t a, int32_t b, int32_t lim) {
    const int l = lane_id();
    if (lim <= 0) return 0;
    {
        bool eq = false;
        if (l < lim) eq = ldb(S, a + l) == ldb(S, b + l);
        const int r = ctz64(~ballot(eq));
        if (r < 64) return r;
    }
    int32_t m = 64;
    for (int guard = 0; guard < 256 && m < lim; guard++) {
        const int32_t o = m + 16 * l;
        uint32_t d = 16;  // first differing byte of this lane's 16 (16: none)
        if (o < lim) {
            const uint4 x = ld128(S, a + o), y = ld128(S, b + o);
            const uint32_t e0 = x.x ^ y.x, e1 = x.y ^ y.y, e2 = x.z ^ y.z, e3 = x.w ^ y.w;
            d = e0 ? (uint32_t)__builtin_ctz(e0) >> 3
                   : e1 ? 4 + ((uint32_t)__builtin_ctz(e1) >> 3)
                        : e2 ? 8 + ((uint32_t)__builtin_ctz(e2) >> 3) : e3 ? 12 + ((uint32_t)__builtin_ctz(e3) >> 3) : 16u;
            if ((int32_t)d > lim - o) d = (uint32_t)(lim - o);
        } else {
            d = 0;
        }
        const int f = ctz64(~ballot(d == 16));
        if (f < 64) return m + 16 * f + (int32_t)readlane(d, f);
        m += 1024;
    }
    return lim < m ? lim : m;
}
// count of i in [0, lim) with s[a - 1 - i] == s[b - 1 - i] before the first mismatch
__device__ int32_t back_count(const Src &S, int32_t a, int32_t b, int32_t lim) {
    const int l = lane_id();
    int32_t m = 0;
    for (int guard = 0; guard < 4096 && m < lim; guard++) {
        const int32_t k = m + l;
        bool eq = false;
        if (k < lim) eq = ldb(S, a - 1 - k) == ldb(S, b - 1 - k);
        const int r = ctz64(~ballot(eq));
        if (r < 64) return m + r;
        m += 64;
    }
    return lim < m ? lim : m;
}

// remaining forward / backward equal-byte counts of a match; the first
// 64-byte steps of both directions are loaded in one round trip
__device__ void ext_counts(const Src &S, int32_t fa, int32_t fb, int32_t flim, int32_t ba, int32_t bb, int32_t blim,
                           int32_t &fwd, int32_t &bk) {
    const int l = lane_id();
    uint32_t x0 = 0, x1 = 1, y0 = 0, y1 = 1;
    if (l < flim) {
        x0 = ldb(S, fa + l);
        x1 = ldb(S, fb + l);
    }
    if (l < blim) {
        y0 = ldb(S, ba - 1 - l);
        y1 = ldb(S, bb - 1 - l);
    }
    const int rf = ctz64(~ballot(l < flim && x0 == x1)), rb = ctz64(~ballot(l < blim && y0 == y1));
    fwd = rf < 64 ? rf : 64 + fwd_count(S, fa + 64, fb + 64, flim - 64);
    bk = rb < 64 ? rb : 64 + back_count(S, ba - 64, bb - 64, blim - 64);
}

// bit i set when byte i of a equals byte i of b
__device__ __forceinline__ uint32_t eqmask16(uint4 a, uint4 b) {
    const uint32_t x[4] = {a.x ^ b.x, a.y ^ b.y, a.z ^ b.z, a.w ^ b.w};
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 4; d++)
#pragma unroll
        for (int k = 0; k < 4; k++) m |= (((x[d] >> (8 * k)) & 0xFFu) == 0u ? 1u : 0u) << (4 * d + k);
    return m;
}
// index, counted from byte k, of the first nonzero byte of x at or after k (16 - k: none)
__device__ __forceinline__ uint32_t first_diff(uint4 x, int k) {
    uint64_t lo = (uint64_t)x.x | ((uint64_t)x.y << 32), hi = (uint64_t)x.z | ((uint64_t)x.w << 32);
    if (k >= 8) {
        lo = hi >> (8 * (k - 8));
        hi = 0;
    } else if (k > 0) {
        lo = (lo >> (8 * k)) | (hi << (64 - 8 * k));
        hi >>= 8 * k;
    }
    if (lo) return (uint32_t)__builtin_ctzll(lo) >> 3;
    if (hi) return 8 + ((uint32_t)__builtin_ctzll(hi) >> 3);
    return (uint32_t)(16 - k);
}
__device__ __forceinline__ uint4 readlane4(uint4 v, int j) {
    return make_uint4(readlane(v.x, j), readlane(v.y, j), readlane(v.z, j), readlane(v.w, j));
}

// compiler-only ordering point: the LDS executes one wave's DS instructions in
// issue order, so a one-wave workgroup needs neither s_barrier nor an lgkmcnt
// drain between its own LDS writes and reads -- only that the compiler keeps
// their order
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// step-schedule position of search iteration l from ip0 (ZSTD_compressBlock_fast:
// ip += ((ip - anchor) >> 7) + 2 on a miss)
__device__ __forceinline__ int32_t sched_pos(int32_t ip0, int32_t anchor, uint32_t l) {
    uint32_t d = (uint32_t)(ip0 - anchor), r = l;
    for (int guard = 0; guard < 80 && ballot(r > 0); guard++) {
        if (r > 0) {
            const uint32_t k = d >> 7, st = k + 2, rem = ((k + 1) << 7) - d;
            uint32_t c = 1;
            if (st < rem) {
                c = (uint32_t)((float)rem * __builtin_amdgcn_rcpf((float)st));
                c += (c * st < rem);
                c += (c * st < rem);
                c -= (c > 1 && (c - 1) * st >= rem);
            }
            const uint32_t t = r < c ? r : c;
            d += t * st;
            r -= t;
        }
    }
    return anchor + (int32_t)d;
}

// all bytes of [a, b) equal (ZSTD_isRLE)
__device__ bool all_equal(const Src &S, int32_t a, int32_t b) {
    const int l = lane_id();
    const uint32_t c = ldb(S, a);
    const uint32_t c4 = c * 0x01010101u;
    for (int32_t p0 = a; p0 < b; p0 += 1024) {
        const int32_t p = p0 + 16 * l;
        bool bad = false;
        if (p < b) {
            const uint4 x = ld128(S, p);
            const int32_t k = b - p;  // valid bytes of the 16
            const uint32_t v[4] = {x.x ^ c4, x.y ^ c4, x.z ^ c4, x.w ^ c4};
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int32_t vb = k - 4 * i;
                const uint32_t m = vb >= 4 ? 0xFFFFFFFFu : vb <= 0 ? 0u : (0xFFFFFFFFu >> (32 - 8 * vb));
                bad |= (v[i] & m) != 0;
            }
        }
        if (ballot(bad)) return false;
    }
    return true;
}

// ---------------------------------------------------------------------------
// kernel 1: the parse (one wave per frame)
// ---------------------------------------------------------------------------
// the serial loop's state between two segments of a block
struct SegSt {
    int32_t ip0, anchor;
    uint32_t o1, o2, saved;
};

// One block of ZSTD_compressBlock_fast_generic (+ the block decisions the
// parse must predict), on the wave's LDS table T; off1 / off2 = the repeat
// offsets handed in (updated as the serial loop passes them on).
// Segments (the speculative parse): the loop's iterations whose search step
// starts at ip0 < se, entered from the state *sin (nullptr: the block start)
// and left in sout at the first search step at or past se (a match and its
// inserts / repeat loop belong to the iteration that found it).  A segment's
// sequences go to index (anchor in - bs) / 4 of the block's area: every
// sequence covers >= 4 bytes, so the segments' ranges never overlap; ns / nl
// count the segment's own.  The block fields are written by the first
// segment (rin) and the last (se >= be: rout, flags, ns / nl of the segment).
template <bool WIDE>
__device__ __forceinline__ void parse_block(const FInfo &F, BInfo &B, int32_t k, Tab<WIDE> &T, const Src &S,
                            uint64_t *__restrict__ seqs, uint32_t &off1, uint32_t &off2, const SegSt *sin,
                            int32_t se, SegSt &sout, int32_t &ons, int32_t &onl) {
    const int l = lane_id();
    const uint32_t hlog = F.hlog, mls = F.mls, tsize = 1u << hlog;
    const int32_t maxDist = 1 << F.wlog;
    ZP_DECL
    const int32_t bs = B.bs, be = B.be;
    const uint32_t rin0 = off1, rin1 = off2;
    ons = 0;
    onl = 0;
    if (be - bs < 7) {  // ZSTD_buildSeqStore: too small to compress, match state untouched
        if (l == 0) {
            B.ns = 0;
            B.nl = be - bs;
            B.rin0 = rin0; B.rin1 = rin1; B.rout0 = rin0; B.rout1 = rin1;
            B.flags = F_NOCOMP;
        }
        onl = be - bs;
        return;
    }
    const int32_t prefixPos = be > maxDist ? be - maxDist : 0;
    const uint32_t prefixIdx = (uint32_t)prefixPos + 1, R = (uint32_t)be;
    if (WIDE && prefixPos > 0) {  // entries that left the window: the window's lowest index
        __syncthreads();
        for (uint32_t h = l; h < tsize; h += 64)
            if (T.get(h, R) <= prefixIdx) T.put(h, prefixIdx);
        __syncthreads();
    }
    ZP(6);
    ZPC(11);
    // ---- ZSTD_compressBlock_fast_generic
    const int32_t ilimit = be - 8;
    int32_t ip0 = bs, anchor = bs, ns = 0, nl = 0;
    uint32_t o1 = off1, o2 = off2, saved = 0;
    if (!sin) {
        if (ip0 == prefixPos) ip0++;
        const uint32_t maxRep = (uint32_t)(ip0 > maxDist ? maxDist : ip0);
        if (o2 > maxRep) { saved = o2; o2 = 0; }
        if (o1 > maxRep) { saved = o1; o1 = 0; }
        if (l == 0) { B.rin0 = rin0; B.rin1 = rin1; }
    } else {
        ip0 = sin->ip0;
        anchor = sin->anchor;
        o1 = sin->o1;
        o2 = sin->o2;
        saved = sin->saved;
    }
    uint64_t *sq = seqs + B.seq_off + (anchor - bs) / 4;
    // sequence records collect in a VGPR (lane i: record 64 g + i) and are
    // stored 64 at a time: no store per sequence for later vmcnt waits to drain
    uint64_t sbuf = 0;
    auto emit = [&](uint32_t ll, uint32_t mlb, uint32_t ofv) {
        const uint64_t r = seq_pack(ll, mlb, ofv);
        if (l == (ns & 63)) sbuf = r;
        if ((ns & 63) == 63) sq[ns - 63 + l] = sbuf;
        ns++;
    };
    int pend = 0;  // 1: after a search match (insert ip0-2, then the repeat loop); 2: after a repeat-loop match
    // windows of the last step whose positions were bp + 2 l (lanes [0, bvalid) valid)
    uint4 Ap = make_uint4(0, 0, 0, 0);
    int32_t bp = -1, bvalid = 0;
    for (int guard = 0; guard < 4 * BLK; guard++) {
        const bool pb = pend != 0;
        const int32_t ipb = ip0;
        // positions of this search step (after a match: ip0 + 2 l)
        const int32_t q = pb ? ip0 + 2 * l : sched_pos(ip0, anchor, (uint32_t)l);
        // windows A = bytes [q - 2, q + 14).  After a match they come from
        // the previous step's lanes when those hold them (a cross-lane
        // permute instead of a memory round trip); lanes without a source
        // sit this step out
        uint4 A = make_uint4(0, 0, 0, 0);
        const bool use_sh = pb && bp >= 0 && ip0 - bp <= 2 * (bvalid - 2);
        bool have = true;
        if (use_sh) {
            const int32_t e = (ip0 - bp) + 2 * l;
            const int s0 = e >> 1;
            const uint32_t dl = (uint32_t)e & 1u;
            const int sa = s0 < 63 ? s0 : 63, sb = s0 + 1 < 63 ? s0 + 1 : 63;
            const uint32_t x0 = (uint32_t)__shfl((int)Ap.x, sa, 64), x1 = (uint32_t)__shfl((int)Ap.y, sa, 64),
                           x2 = (uint32_t)__shfl((int)Ap.z, sa, 64), x3 = (uint32_t)__shfl((int)Ap.w, sa, 64),
                           y3 = (uint32_t)__shfl((int)Ap.w, sb, 64);
            A = dl ? make_uint4(__builtin_amdgcn_alignbyte(x1, x0, 1), __builtin_amdgcn_alignbyte(x2, x1, 1),
                                __builtin_amdgcn_alignbyte(x3, x2, 1), __builtin_amdgcn_alignbyte(y3 >> 16, x3, 1))
                   : make_uint4(x0, x1, x2, x3);
            have = s0 + (int)dl < bvalid;
        }
        const bool on = q + 1 < ilimit && (!pb || l < JFS_ZL1_PB) && have;
        // (after a match every lane loads its window, on or not: the next
        // step's windows then come from these)
        const bool ld = !use_sh && (pb || on);
        // AR = the same bytes o1 back (repeat check + its first extension
        // bytes), R2 = (lane 0, after a match) 16 bytes at ip0 - 2 - o2 (the
        // repeat loop): both awaited only where used
        uint4 AR = make_uint4(0, 0, 0, 0), R2 = make_uint4(0, 0, 0, 0);
        if (ld) A = ld128(S, q - 2);
        if (on) AR = ld128(S, q - 2 - (int32_t)o1);
        if (pb && l == 0) R2 = ld128(S, ip0 - 2 - (int32_t)o2);
        const int32_t vcount = pb ? (int32_t)__builtin_popcountll(ballot(use_sh ? have : ld)) : 0;
        const uint64_t v0 = (uint64_t)__builtin_amdgcn_alignbyte(A.y, A.x, 2) | ((uint64_t)__builtin_amdgcn_alignbyte(A.z, A.y, 2) << 32);
        const uint64_t v1 = (uint64_t)__builtin_amdgcn_alignbyte(A.y, A.x, 3) | ((uint64_t)__builtin_amdgcn_alignbyte(A.z, A.y, 3) << 32);
        const uint32_t val0 = (uint32_t)v0, val1 = (uint32_t)v1;
        const uint32_t h0 = zhash(v0, hlog, mls), h1 = zhash(v1, hlog, mls);
        ZP(0);
        ZPC(9);
        if (pend == 1) {  // hashTable[hash(ip0 - 2)] = ip0 - 2
            const uint64_t vm2 = (uint64_t)A.x | ((uint64_t)A.y << 32);
            const uint32_t hm2 = readlane(zhash(vm2, hlog, mls), 0);
            if (l == 0) T.put(hm2, (uint32_t)(ip0 - 2 + 1));
            lds_order();
        }
        // the repeat loop's check waits for R2: the search step's table
        // reads and bucket tags go first (undone if the repeat loop fires)
        const bool rchk = pb && o2 > 0 && ip0 <= ilimit;
        pend = 0;
        const uint64_t onm = ballot(on);
        if (!onm && !rchk) break;  // ip1 >= ilimit: no more positions in this block
        const int non = onm ? 64 - __builtin_clzll(onm) : 0;  // lanes [0, non) are on
        // table reads (before any write of this step), then tags to find
        // lanes sharing a bucket
        uint32_t olo0 = 0, olo1 = 0, i0 = 0, i1 = 0;
        if (on) {
            olo0 = T.lo[h0];
            olo1 = T.lo[h1];
            i0 = T.get(h0, R);
            i1 = T.get(h1, R);
        }
        lds_order();
        if (on) {
            T.lo[h0] = (uint16_t)l;
            T.lo[h1] = (uint16_t)l;
        }
        lds_order();
        uint32_t cm = 64;
        if (on) {
            const uint32_t t0 = T.lo[h0], t1 = T.lo[h1];
            if (t0 != (uint32_t)l) cm = umin32((uint32_t)l, t0);
            if (t1 != (uint32_t)l) cm = umin32(cm, umin32((uint32_t)l, t1));
        }
        const int cut = (int)dwave_min(cm) + 1;
        const int nbt = cut < non ? cut : non;  // lanes [0, nbt) read exactly what the serial loop reads
        const bool dec = l < nbt;
        const bool c0 = dec && i0 > prefixIdx, c1 = dec && i1 > prefixIdx;
        // candidates: bytes [cand - 2, cand + 14) (check + first extension bytes)
        uint4 X0 = make_uint4(0, 0, 0, 0), X1 = make_uint4(0, 0, 0, 0);
        if (c0) X0 = ld128(S, (int32_t)i0 - 3);
        if (c1) X1 = ld128(S, (int32_t)i1 - 3);
        ZP(2);
        if (rchk) {
            const uint4 a0 = readlane4(A, 0), r0 = readlane4(R2, 0);
            const uint4 X = make_uint4(a0.x ^ r0.x, a0.y ^ r0.y, a0.z ^ r0.z, a0.w ^ r0.w);
            if (first_diff(X, 2) >= 4) {  // MEM_read32(ip0) == MEM_read32(ip0 - offset_2)
                if (on) {  // the search step did not happen: its tags come off
                    T.lo[h0] = (uint16_t)olo0;
                    T.lo[h1] = (uint16_t)olo1;
                }
                lds_order();
                // repeat-offset match at ip0 (offset_2), then swap
                const int32_t flim = be - (ip0 + 4);
                int32_t rl = (int32_t)umin32(first_diff(X, 6), (uint32_t)flim);
                if (rl == 10 && rl < flim) {
                    int32_t f2 = 0, b2 = 0;
                    ext_counts(S, ip0 + 4 + rl, ip0 + 4 + rl - (int32_t)o2, flim - rl, 0, 0, 0, f2, b2);
                    rl += f2;
                }
                rl += 4;
                const uint32_t t = o2;
                o2 = o1;
                o1 = t;
                if (l == 0) T.put(readlane(h0, 0), (uint32_t)(ip0 + 1));
                lds_order();
                emit(0, (uint32_t)(rl - 3), 1);
                Ap = A;
                bp = ipb;
                bvalid = vcount;
                ip0 += rl;
                anchor = ip0;
                if (ip0 <= ilimit) pend = 2;
                ZP(1);
                continue;
            }
        }
        ZP(1);
        if (ip0 >= se) {  // the next segment's first search step: its tags come off
            if (on) {
                T.lo[h0] = (uint16_t)olo0;
                T.lo[h1] = (uint16_t)olo1;
            }
            lds_order();
            break;
        }
        if (!onm) break;
        const bool rep = dec && o1 > 0 && AR.y == A.y;  // MEM_read32(ip2 - offset_1) == MEM_read32(ip2)
        const bool k0 = c0 && __builtin_amdgcn_alignbyte(X0.y, X0.x, 2) == val0;
        const bool k1 = c1 && __builtin_amdgcn_alignbyte(X1.y, X1.x, 2) == val1;
        const int j = ctz64(ballot(rep || k0 || k1));
        ZP(3);
        // lanes after the first hit (and past the cut) put their buckets
        // back; then the lanes up to the hit insert ip0 and ip1
        lds_order();
        if (on && (l >= nbt || l > j)) {
            T.lo[h0] = (uint16_t)olo0;
            T.lo[h1] = (uint16_t)olo1;
        }
        lds_order();
        if (on && l < nbt && l <= j) {
            T.put(h0, (uint32_t)q + 1);
            T.put(h1, (uint32_t)q + 2);
        }
        lds_order();
        ZP(4);
        if (j >= 64) {
            const int32_t ql = (int32_t)readlane((uint32_t)q, nbt - 1);
            ip0 = ql + ((ql - anchor) >> 7) + 2;
            bp = -1;
            continue;
        }
        Ap = A;
        bp = pb ? ipb : -1;
        bvalid = vcount;
        // ---- a match at iteration j.  Every lane works out, in VGPRs, the
        // match its own iteration would give (start, source, the cheap
        // part of the extension from the windows already loaded); lane j's
        // values are then read once (few SGPRs live: no SGPR spills)
        uint32_t mstart = 0, msrc = 0, mlen0 = 4, fch = 0, bch = 0, mflags = 0;
        {
            const int ty = rep ? 0 : k0 ? 1 : 2;
            uint4 Aa = A;
            if (ty == 2)  // the match starts at q + 1: shift the window by a byte
                Aa = make_uint4(__builtin_amdgcn_alignbyte(A.y, A.x, 1), __builtin_amdgcn_alignbyte(A.z, A.y, 1),
                                __builtin_amdgcn_alignbyte(A.w, A.z, 1), A.w >> 8);
            const uint4 Bb = ty == 0 ? AR : ty == 1 ? X0 : X1;
            const uint4 X = make_uint4(Aa.x ^ Bb.x, Aa.y ^ Bb.y, Aa.z ^ Bb.z, Aa.w ^ Bb.w);
            if (ty == 0) {
                const uint32_t ml0 = (X.x >> 24) == 0u ? 1u : 0u;  // ip2[-1] == repMatch[-1]
                mstart = (uint32_t)q + 2 - ml0;
                msrc = mstart - o1;
                mlen0 = 4 + ml0;
                fch = first_diff(X, 8);  // bytes q+6 .. q+13
                mflags = fch == 8 ? 1u : 0u;
            } else {
                mstart = ty == 1 ? (uint32_t)q : (uint32_t)q + 1;
                msrc = (ty == 1 ? i0 : i1) - 1;
                const uint32_t favail = ty == 1 ? 10 : 9;  // bytes start+4 .. (window end)
                fch = umin32(first_diff(X, 6), favail);
                bch = ((X.x >> 8) & 0xFFu) ? 0u : ((X.x & 0xFFu) ? 1u : 2u);
                mflags = (fch == favail ? 1u : 0u) | (bch == 2 ? 2u : 0u) | 4u;
            }
        }
        const uint32_t h2 = zhash((uint64_t)A.y | ((uint64_t)A.z << 32), hlog, mls);  // hash at q + 2
        const int32_t qj = (int32_t)readlane((uint32_t)q, j);
        const uint32_t jh2 = readlane(h2, j);
        int32_t start = (int32_t)readlane(mstart, j), mst = (int32_t)readlane(msrc, j);
        int32_t mlen = (int32_t)readlane(mlen0, j), fcheap = (int32_t)readlane(fch, j), bcheap = (int32_t)readlane(bch, j);
        const uint32_t fl = readlane(mflags, j);
        const bool fex = fl & 1u, bex = (fl & 2u) != 0, regular = (fl & 4u) != 0;
        uint32_t ofv = 1;
        if (regular) {
            o2 = o1;
            o1 = (uint32_t)(start - mst);
            ofv = o1 + 3;
        }
        const int32_t flim = be - (start + mlen);
        const int32_t blim = !regular ? 0 : (int32_t)umin32((uint32_t)(start - anchor), (uint32_t)(mst - prefixPos));
        if (fcheap > flim) fcheap = flim;
        if (bcheap > blim) bcheap = blim;
        const bool nf = fex && fcheap < flim, nbk = bex && bcheap < blim;
        if (nf || nbk) {
            ZPC(10);
            int32_t f2 = 0, b2 = 0;
            ext_counts(S, start + mlen + fcheap, mst + mlen + fcheap, nf ? flim - fcheap : 0, start - bcheap,
                       mst - bcheap, nbk ? blim - bcheap : 0, f2, b2);
            fcheap += f2;
            bcheap += b2;
        }
        start -= bcheap;
        mst -= bcheap;
        mlen += bcheap + fcheap;
        emit((uint32_t)(start - anchor), (uint32_t)(mlen - 3), ofv);
        ZPC(8);
        nl += start - anchor;
        ip0 = start + mlen;
        anchor = ip0;
        if (ip0 <= ilimit) {
            if (l == 0) T.put(jh2, (uint32_t)(qj + 2 + 1));  // hashTable[hash(current0 + 2)]
            lds_order();
            pend = 1;
        }
        ZP(5);
    }
    if (ns & 63) {  // the last partial group
        const int32_t g0 = ns & ~63;
        if (g0 + l < ns) sq[g0 + l] = sbuf;
    }
    ons = ns;
    if (se < be) {  // a segment before the block's last: hand the loop's state on
        onl = nl;
        sout.ip0 = ip0;
        sout.anchor = anchor;
        sout.o1 = o1;
        sout.o2 = o2;
        sout.saved = saved;
        ZP_FLUSH();
        return;
    }
    nl += be - anchor;
    onl = nl;
    const bool rle = k > 0 && all_equal(S, bs, be);
    const uint32_t ro0 = o1 ? o1 : saved, ro1 = o2 ? o2 : saved;
    const bool assumed = B.conf ? B.conf == 1 : !rle;
    if (l == 0) {
        B.ns = ns;
        B.nl = nl;
        B.rout0 = ro0; B.rout1 = ro1;
        B.flags = (rle ? F_RLE : 0) | (assumed ? F_ASSUMED : 0);
    }
    if (assumed) {
        off1 = ro0;
        off2 = ro1;
    }
    ZP_FLUSH();
}

template <bool WIDE>
__global__ __launch_bounds__(64) void zl1_parse_kernel(const FInfo *__restrict__ fi, const int32_t *__restrict__ flist,
                                                       BInfo *__restrict__ bi, uint64_t *__restrict__ seqs) {
    extern __shared__ uint32_t smem[];
    const int l = lane_id();
    const FInfo F = fi[flist[blockIdx.x]];
    if (F.status < 0) return;
    const uint32_t tsize = 1u << F.hlog;
    Tab<WIDE> T;
    T.lo = (uint16_t *)smem;
    T.hi = smem + (tsize >> 1);
    for (uint32_t k = l; k < (tsize >> 1); k += 64) smem[k] = 0;
    if (WIDE)
        for (uint32_t k = l; k < (tsize >> 3); k += 64) T.hi[k] = 0;
    __syncthreads();
    const Src S = make_src(F.src, F.n);
    uint32_t off1 = 1, off2 = 4;  // repStartValue
    SegSt so;
    int32_t a, b;
    for (int32_t k = 0; k < F.nb; k++)
        parse_block<WIDE>(F, bi[F.b0 + k], k, T, S, seqs, off1, off2, nullptr, 0x7FFFFFFF, so, a, b);
}

// ---------------------------------------------------------------------------
// small batches: block-parallel speculative parse (exact)
// ---------------------------------------------------------------------------
// The frame-serial parse runs one wave per frame: a lone 4 MiB frame is 32
// block parses in a row (~0.7 s).  A block's parse depends on the frame only
// through its starting hash table and repeat offsets, and the table at the
// start of block k holds, for every bucket, the last index any earlier block
// wrote there -- the maximum over those blocks' WRITE SETS (indices grow with
// the block).  So every block parses at once from inputs built out of the
// other blocks' latest results (zl1_spec_merge: prefix maxima of the write
// sets, the repeat offsets passed on in block order), and again whenever its
// inputs changed; when a round changes no block's inputs, each block's inputs
// are what its predecessors' parses produce, and by induction from block 0
// (whose inputs are the empty table and repStartValue) every block's parse is
// the serial one.  Text settles in 7-8 rounds, random and zero data in 3 (CPU
// simulation on the fixture inputs); at most nb + 1 rounds in any case.
// Segments: a block splits into segsz-byte segments (the loop's iterations
// whose search step starts inside, parse_block) when the batch has few blocks,
// so a round is a fraction of a block parse; the same fixed point holds with
// the loop's state (position, anchor, repeat offsets) handed from segment to
// segment like the table.  A CPU simulation of the bench frame
// (scripts/sim/spec_sim.cc) settles in 7 rounds of 128 KiB, 11 of 32 KiB,
// 15 of 16 KiB: 7, 2.75 and 1.9 block parses of wall time.
struct SpecB {
    int32_t chg;          // run this round
    uint32_t rin0, rin1;  // first segment of a block: repeat offsets handed in
    int32_t blk, q;       // block (index into bi) and segment of the block
    SegSt in, out;        // later segments: the loop's state handed in / out
    int32_t ns, nl;       // sequences and literals of the segment
};
constexpr uint32_t SPEC_TSZ = 1u << 14;  // table slots per segment (wide frames: hashLog <= 14)
constexpr int SPEC_MAXSEG = 4096;        // segments per frame (the merge's flags)

// grid (frame, 64-bucket chunk): chunk 0 hands every segment its inputs
// (repeat offsets, the loop's state: a thread per segment); every thread
// takes one bucket through the frame's segments (prefix maxima of the write
// sets).  Flags only ever rise (zl1_spec_parse clears its own).
// any[r]: round r changed something.  The host looks every few rounds; a
// round after a settled one exits at once (and would change nothing anyway).
__global__ __launch_bounds__(64) void zl1_spec_merge(const FInfo *__restrict__ fi, const int32_t *__restrict__ sflist,
                                                      const int32_t *__restrict__ sslot, const int32_t *__restrict__ snseg,
                                                      const BInfo *__restrict__ bi, const uint32_t *__restrict__ W,
                                                      uint32_t *__restrict__ I, SpecB *__restrict__ sp,
                                                      int32_t *__restrict__ any, int r) {
    __shared__ uint32_t mark[SPEC_MAXSEG / 32];
    __shared__ int32_t anyc;
    const int first = r == 0;
    if (r >= 2 && !any[r - 1]) return;
    const FInfo F = fi[sflist[blockIdx.x]];
    const int32_t s0 = sslot[blockIdx.x], nseg = snseg[blockIdx.x];
    const uint32_t tsize = 1u << F.hlog;
    const int t = threadIdx.x;
    for (int i = t; i < SPEC_MAXSEG / 32; i += 64) mark[i] = 0;
    if (t == 0) anyc = 0;
    __syncthreads();
    if (blockIdx.y == 0) {
        // a segment after a block's first takes its predecessor's state; a
        // block's first takes the repeat offsets of the nearest earlier block
        // that passes them on (compressed-assumed, >= 7 bytes), else
        // repStartValue -- independent per segment, one thread each
        for (int32_t s = t; s < nseg; s += 64) {
            SpecB &x = sp[s0 + s];
            bool c = first != 0;
            if (x.q == 0) {
                uint32_t r0 = 1, r1 = 4;
                for (int32_t j = x.blk - 1; j >= F.b0; j--) {
                    const BInfo &Bj = bi[j];
                    if (Bj.be - Bj.bs >= 7 && (Bj.flags & F_ASSUMED)) {
                        r0 = Bj.rout0;
                        r1 = Bj.rout1;
                        break;
                    }
                }
                c |= x.rin0 != r0 || x.rin1 != r1;
                x.rin0 = r0;
                x.rin1 = r1;
            } else if (!first) {  // (round 0 keeps the host's guess)
                const SegSt p = sp[s0 + s - 1].out;
                c |= x.in.ip0 != p.ip0 || x.in.anchor != p.anchor || x.in.o1 != p.o1 || x.in.o2 != p.o2 ||
                     x.in.saved != p.saved;
                x.in = p;
            }
            if (c) {
                atomicOr(&mark[s >> 5], 1u << (s & 31));
                anyc = 1;
            }
        }
    }
    const uint32_t h = blockIdx.y * 64 + t;
    if (h < tsize) {
        uint32_t run = 0;
        for (int32_t s1 = 0; s1 < nseg; s1 += 16) {  // sixteen segments' loads in flight
            uint32_t iv[16], wv[16];
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const size_t o = (size_t)(s0 + s1 + u) * SPEC_TSZ + h;
                iv[u] = s1 + u < nseg ? I[o] : 0u;
                wv[u] = s1 + u < nseg ? W[o] : 0u;
            }
#pragma unroll
            for (int u = 0; u < 16; u++) {
                const int32_t s = s1 + u;
                if (s < nseg && iv[u] != run) {
                    I[(size_t)(s0 + s) * SPEC_TSZ + h] = run;
                    atomicOr(&mark[s >> 5], 1u << (s & 31));
                    anyc = 1;
                }
                run = umax32(run, wv[u]);
            }
        }
    }
    __syncthreads();
    for (int32_t s = t; s < nseg; s += 64)
        if ((mark[s >> 5] >> (s & 31)) & 1u) sp[s0 + s].chg = 1;
    if (t == 0 && anyc) atomicOr(&any[r], 1);
}

// one wave per segment whose inputs changed
template <bool WIDE>
__global__ __launch_bounds__(64) void zl1_spec_parse(const FInfo *__restrict__ fi, BInfo *__restrict__ bi,
                                                     uint64_t *__restrict__ seqs, const uint32_t *__restrict__ I,
                                                     uint32_t *__restrict__ W, SpecB *__restrict__ sp, int32_t segsz) {
    extern __shared__ uint32_t smem[];
    const int g = blockIdx.x;
    const SpecB x = sp[g];
    if (!x.chg) return;
    const int l = lane_id();
    BInfo &B = bi[x.blk];
    const FInfo F = fi[B.frame];
    const int32_t k = x.blk - F.b0;
    const uint32_t tsize = 1u << F.hlog;
    const int32_t maxDist = 1 << F.wlog;
    const int32_t ss = B.bs + x.q * segsz, se = B.be - ss > segsz ? ss + segsz : 0x7FFFFFFF;
    Tab<WIDE> T;
    T.lo = (uint16_t *)smem;
    T.hi = smem + (tsize >> 1);
    // the input table: entries at or below the window's lowest index act as
    // "no candidate" (and must not alias into the 20-bit window)
    const uint32_t prefixIdx = (uint32_t)(B.be > maxDist ? B.be - maxDist : 0) + 1;
    const uint32_t *Ik = I + (size_t)g * SPEC_TSZ;
    for (uint32_t h8 = l; h8 < (tsize >> 3); h8 += 64) {
        uint32_t nib = 0;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t v = umax32(Ik[8 * h8 + q], prefixIdx);
            T.lo[8 * h8 + q] = (uint16_t)v;
            nib |= ((v >> 16) & 15u) << (4 * q);
        }
        if (WIDE) T.hi[h8] = nib;
    }
    __syncthreads();
    const Src S = make_src(F.src, F.n);
    uint32_t off1 = x.rin0, off2 = x.rin1;
    SegSt out = x.in;
    int32_t ns = 0, nl = 0;
    parse_block<WIDE>(F, B, k, T, S, seqs, off1, off2, x.q ? &x.in : nullptr, se, out, ns, nl);
    __syncthreads();
    // the segment's write set: the entries now at indices of this segment
    // (entries of earlier segments past ss are in its input already: the
    // merge's maxima do not change)
    uint32_t *Wk = W + (size_t)g * SPEC_TSZ;
    const uint32_t R = (uint32_t)B.be;
    for (uint32_t h = l; h < tsize; h += 64) {
        const uint32_t e = T.get(h, R);
        Wk[h] = e > (uint32_t)ss ? e : 0u;
    }
    if (l == 0) {
        SpecB &y = sp[g];
        y.chg = 0;
        y.out = out;
        y.ns = ns;
        y.nl = nl;
    }
}

// one wave per block of the speculative frames, after the last round: the
// segments' sequences moved together (forward: a record never moves up),
// the block's counts
__global__ __launch_bounds__(64) void zl1_spec_compact(const int32_t *__restrict__ bfirst, BInfo *__restrict__ bi,
                                                       uint64_t *__restrict__ seqs, const SpecB *__restrict__ sp) {
    const int l = lane_id();
    const int32_t g0 = bfirst[blockIdx.x], g1 = bfirst[blockIdx.x + 1];
    BInfo &B = bi[sp[g0].blk];
    if (B.flags & F_NOCOMP) return;  // (set whole by the parse)
    uint64_t *sq = seqs + B.seq_off;
    int32_t ns = 0, nl = 0;
    for (int32_t g = g0; g < g1; g++) {
        const SpecB x = sp[g];
        const int32_t base = x.q ? (x.in.anchor - B.bs) / 4 : 0;
        if (base != ns)
            for (int32_t i = 0; i < x.ns; i += 64) {
                const uint64_t v = i + l < x.ns ? sq[base + i + l] : 0;
                __builtin_amdgcn_wave_barrier();
                if (i + l < x.ns) sq[ns + i + l] = v;
            }
        ns += x.ns;
        nl += x.nl;
    }
    if (l == 0) {
        B.ns = ns;
        B.nl = nl;
    }
}

// ---------------------------------------------------------------------------
// FSE / Huffman tables (FSE_buildCTable_wksp, FSE_normalizeCount,
// FSE_writeNCount, HUF_buildCTable_wksp, HUF_writeCTable) -- serial, lane 0
// ---------------------------------------------------------------------------
__constant__ uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint8_t LL_CODE[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                    16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21,
                                    22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                                    24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
__constant__ uint8_t ML_CODE[128] = {
    0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23, 24, 25,
    26, 27, 28, 29, 30, 31, 32, 32, 33, 33, 34, 34, 35, 35, 36, 36, 36, 36, 37, 37, 37, 37, 38, 38, 38, 38,
    38, 38, 38, 38, 39, 39, 39, 39, 39, 39, 39, 39, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40,
    40, 40, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 42, 42, 42, 42, 42, 42, 42, 42,
    42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42};
__constant__ int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

__device__ __forceinline__ uint32_t ll_code(uint32_t ll) { return ll > 63 ? hbit(ll) + 19 : LL_CODE[ll]; }
__device__ __forceinline__ uint32_t ml_code(uint32_t mlb) { return mlb > 127 ? hbit(mlb) + 36 : ML_CODE[mlb]; }

// FSE encoding table; N = state capacity
template <int N, int NS>
struct CTab {
    uint16_t st[N];
    int32_t dnb[NS];
    int16_t dfs[NS];
    int32_t tlog;
};

__device__ uint32_t fse_min_tlog(uint32_t src, uint32_t maxsv) {
    const uint32_t a = hbit(src) + 1, b = hbit(maxsv) + 2;
    return a < b ? a : b;
}
__device__ uint32_t fse_opt_tlog(uint32_t maxtl, uint32_t src, uint32_t maxsv, uint32_t minus) {
    const uint32_t maxBitsSrc = hbit(src - 1) - minus;
    uint32_t tl = maxtl;
    const uint32_t minBits = fse_min_tlog(src, maxsv);
    if (maxBitsSrc < tl) tl = maxBitsSrc;
    if (minBits > tl) tl = minBits;
    if (tl < 5) tl = 5;
    if (tl > 12) tl = 12;
    return tl;
}

__device__ int fse_norm_m2(int16_t *norm, uint32_t tlog, const uint32_t *count, uint32_t total, uint32_t maxsv,
                           int16_t lowProb) {
    const int16_t NYA = -2;
    uint32_t s, distributed = 0, toDist;
    const uint32_t lowThreshold = total >> tlog;
    uint32_t lowOne = (uint32_t)(((uint64_t)total * 3) >> (tlog + 1));
    for (s = 0; s <= maxsv; s++) {
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) { norm[s] = lowProb; distributed++; total -= count[s]; continue; }
        if (count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
        norm[s] = NYA;
    }
    toDist = (1u << tlog) - distributed;
    if (toDist == 0) return 0;
    if ((total / toDist) > lowOne) {
        lowOne = (uint32_t)(((uint64_t)total * 3) / (toDist * 2));
        for (s = 0; s <= maxsv; s++)
            if (norm[s] == NYA && count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; }
        toDist = (1u << tlog) - distributed;
    }
    if (distributed == maxsv + 1) {
        uint32_t maxV = 0, maxC = 0;
        for (s = 0; s <= maxsv; s++)
            if (count[s] > maxC) { maxV = s; maxC = count[s]; }
        norm[maxV] = (int16_t)(norm[maxV] + (int16_t)toDist);
        return 0;
    }
    if (total == 0) {
        for (s = 0; toDist > 0; s = (s + 1) % (maxsv + 1))
            if (norm[s] > 0) { toDist--; norm[s]++; }
        return 0;
    }
    {
        const uint64_t vStepLog = 62 - tlog;
        const uint64_t mid = (1ull << (vStepLog - 1)) - 1;
        const uint64_t rStep = ((((uint64_t)1 << vStepLog) * toDist) + mid) / total;
        uint64_t tmpTotal = mid;
        for (s = 0; s <= maxsv; s++) {
            if (norm[s] == NYA) {
                const uint64_t end = tmpTotal + (count[s] * rStep);
                const uint32_t sStart = (uint32_t)(tmpTotal >> vStepLog), sEnd = (uint32_t)(end >> vStepLog);
                const uint32_t weight = sEnd - sStart;
                if (weight < 1) return -1;
                norm[s] = (int16_t)weight;
                tmpTotal = end;
            }
        }
    }
    return 0;
}

__device__ int fse_normalize(int16_t *norm, uint32_t tlog, const uint32_t *count, uint32_t total, uint32_t maxsv,
                             bool lowprob) {
    const uint32_t rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    const int16_t lowProbCount = lowprob ? -1 : 1;
    const uint64_t scale = 62 - tlog;
    const uint64_t step = ((uint64_t)1 << 62) / total;
    const uint64_t vStep = 1ull << (scale - 20);
    int still = 1 << tlog;
    uint32_t s, largest = 0;
    int16_t largestP = 0;
    const uint32_t lowThreshold = total >> tlog;
    for (s = 0; s <= maxsv; s++) {
        if (count[s] == total) return 0;
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) {
            norm[s] = lowProbCount;
            still--;
        } else {
            int16_t proba = (int16_t)((count[s] * step) >> scale);
            if (proba < 8) {
                const uint64_t restToBeat = vStep * rtb[proba];
                proba += (count[s] * step) - ((uint64_t)proba << scale) > restToBeat;
            }
            if (proba > largestP) { largestP = proba; largest = s; }
            norm[s] = proba;
            still -= proba;
        }
    }
    if (-still >= (norm[largest] >> 1)) {
        if (fse_norm_m2(norm, tlog, count, total, maxsv, lowProbCount) < 0) return -1;
    } else {
        norm[largest] = (int16_t)(norm[largest] + still);
    }
    return (int)tlog;
}

// FSE_writeNCount layout into out (LDS), returns bytes
__device__ int write_ncount(uint8_t *out, const int16_t *norm, uint32_t maxsv, uint32_t tlog) {
    int o = 0;
    const int tsize = 1 << tlog;
    int remaining = tsize + 1, threshold = tsize, nbits = (int)tlog + 1;
    uint32_t bs = tlog - 5;
    int bc = 4;
    uint32_t sym = 0;
    const uint32_t alpha = maxsv + 1;
    int prev0 = 0;
    while (sym < alpha && remaining > 1) {
        if (prev0) {
            uint32_t start = sym;
            while (sym < alpha && !norm[sym]) sym++;
            if (sym == alpha) break;
            while (sym >= start + 24) {
                start += 24;
                bs += 0xFFFFu << bc;
                out[o] = (uint8_t)bs;
                out[o + 1] = (uint8_t)(bs >> 8);
                o += 2;
                bs >>= 16;
            }
            while (sym >= start + 3) {
                start += 3;
                bs += 3u << bc;
                bc += 2;
            }
            bs += (sym - start) << bc;
            bc += 2;
            if (bc > 16) {
                out[o] = (uint8_t)bs;
                out[o + 1] = (uint8_t)(bs >> 8);
                o += 2;
                bs >>= 16;
                bc -= 16;
            }
        }
        int count = norm[sym++];
        const int max = (2 * threshold - 1) - remaining;
        remaining -= count < 0 ? -count : count;
        count++;
        if (count >= threshold) count += max;
        bs += (uint32_t)count << bc;
        bc += nbits;
        bc -= count < max ? 1 : 0;
        prev0 = count == 1;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
        if (bc > 16) {
            out[o] = (uint8_t)bs;
            out[o + 1] = (uint8_t)(bs >> 8);
            o += 2;
            bs >>= 16;
            bc -= 16;
        }
    }
    out[o] = (uint8_t)bs;
    out[o + 1] = (uint8_t)(bs >> 8);
    o += (bc + 7) / 8;
    return o;
}

template <int N, int NS>
__device__ void build_ctab(uint8_t *tsym, CTab<N, NS> &t, const int16_t *norm, uint32_t maxsv, uint32_t tlog) {
    const uint32_t size = 1u << tlog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t high = size - 1;
    uint32_t cumul[NS + 1];
    t.tlog = (int32_t)tlog;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= maxsv + 1; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            tsym[high--] = (uint8_t)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
        }
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxsv; s++) {
        for (int k = 0; k < norm[s]; k++) {
            tsym[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    }
    for (uint32_t u = 0; u < size; u++) t.st[cumul[tsym[u]]++] = (uint16_t)(size + u);
    uint32_t total = 0;
    for (uint32_t s = 0; s <= maxsv; s++) {
        const int nc = norm[s];
        if (nc == 0) {
            t.dnb[s] = (int32_t)(((tlog + 1) << 16) - size);
            t.dfs[s] = 0;
        } else if (nc == -1 || nc == 1) {
            t.dnb[s] = (int32_t)((tlog << 16) - size);
            t.dfs[s] = (int16_t)((int32_t)total - 1);
            total += 1;
        } else {
            const uint32_t mbo = tlog - hbit((uint32_t)nc - 1);
            t.dnb[s] = (int32_t)((mbo << 16) - ((uint32_t)nc << mbo));
            t.dfs[s] = (int16_t)((int32_t)total - nc);
            total += (uint32_t)nc;
        }
    }
}
template <int N, int NS>
__device__ void build_rle(CTab<N, NS> &t, uint32_t sym) {
    t.tlog = 0;
    t.st[0] = 0;
    t.st[1] = 0;
    t.dnb[sym] = 0;
    t.dfs[sym] = 0;
}

// ---------------------------------------------------------------------------
// backward bitstream into global memory (BIT_CStream bit order)
// ---------------------------------------------------------------------------
struct BitW {
    g_u8 *dst;
    int64_t wp, lim;
    uint64_t bc;
    int bp;
    bool ovf;
};
__device__ __forceinline__ void bw_add(BitW &w, uint32_t v, int nb) {
    w.bc |= ((uint64_t)v & ((1ull << nb) - 1ull)) << w.bp;
    w.bp += nb;
}
__device__ __forceinline__ void bw_flush(BitW &w) {
    const int nbytes = w.bp >> 3;
    const int l = lane_id();
    if (w.wp + nbytes > w.lim) w.ovf = true;
    if (!w.ovf && l < nbytes) w.dst[w.wp + l] = (uint8_t)(w.bc >> (8 * l));
    w.wp += nbytes;
    w.bc = nbytes >= 8 ? 0ull : (w.bc >> (8 * nbytes));
    w.bp &= 7;
}

// ---------------------------------------------------------------------------
// kernel 2: literals + sequences section of one block (one wave per block)
// ---------------------------------------------------------------------------
struct SeqSmem {
    uint32_t h4[4][256];  // literal histograms per Huffman stream segment
    uint32_t cnt[3][64];  // LL / OF / ML code histograms
    int16_t norm[64];
    uint8_t tsym[512];
    CTab<512, 36> tLL;
    CTab<256, 32> tOF;
    CTab<512, 53> tML;
    uint8_t hdr[3][128];
    int32_t hsz[3], type[3];
    uint32_t lastc[3];
    uint32_t ring[256];  // sequence bitstream staging (8,192 bits)
};

// A wave's bit writer through an LDS ring of 256 dwords: bit 0 of the ring is
// bit 0 of the dword holding the stream's first byte (dst + o); complete
// dwords are stored as they fill, the bytes of that first dword before the
// stream are kept, nothing is written at or past byte `lim` of dst (a stream
// that does not fit only reports it).
struct RingW {
    uint32_t *ring;
    g_u8 *base;          // dword-aligned
    int64_t first_byte;  // bytes of dword 0 before the stream
    int64_t limb;        // byte limit, from base
    uint64_t bitpos;     // next bit, from base
    uint64_t flushed;    // dwords stored
};
__device__ __forceinline__ void rw_init(RingW &w, uint32_t *ring, g_u8 *dst, int64_t o, int64_t lim) {
    w.ring = ring;
    w.base = (g_u8 *)((uintptr_t)(dst + o) & ~(uintptr_t)3);
    w.first_byte = (int64_t)((uintptr_t)(dst + o) & 3u);
    w.limb = w.first_byte + (lim - o);
    w.bitpos = (uint64_t)w.first_byte * 8;
    w.flushed = 0;
    for (int k = lane_id(); k < 256; k += 64) ring[k] = 0;
    __syncthreads();
}
// OR n (<= 32) bits of v in at bit p (lanes at once; p from base)
__device__ __forceinline__ void rw_or(RingW &w, uint64_t p, uint32_t v, uint32_t n) {
    if (!n) return;
    v &= (uint32_t)((1ull << n) - 1ull);
    const uint32_t d = (uint32_t)(p >> 5) & 255u, sh = (uint32_t)(p & 31u);
    atomicOr(&w.ring[d], v << sh);
    if (sh + n > 32) atomicOr(&w.ring[(d + 1) & 255u], v >> (32 - sh));
}
// store the dwords below bitpos that are complete
__device__ __forceinline__ void rw_flush(RingW &w) {
    const int l = lane_id();
    __syncthreads();
    const uint64_t full = w.bitpos >> 5;
    for (uint64_t dw = w.flushed + l; dw < full; dw += 64) {
        const uint32_t v = w.ring[dw & 255u];
        if (dw == 0 && w.first_byte > 0) {
            for (int k = (int)w.first_byte; k < 4; k++)
                if (k < w.limb) w.base[k] = (uint8_t)(v >> (8 * k));
        } else if ((int64_t)dw * 4 + 4 <= w.limb) {
            ((g_u32 *)w.base)[dw] = v;
        }
        w.ring[dw & 255u] = 0;
    }
    __syncthreads();
    w.flushed = full;
}
// the last partial dword; returns the stream's end (bytes from dst + o)
__device__ __forceinline__ int64_t rw_close(RingW &w) {
    const int l = lane_id();
    rw_flush(w);
    const uint64_t endbyte = (w.bitpos + 7) >> 3;
    const uint64_t lastdw = (endbyte + 3) >> 2;
    for (uint64_t dw = w.flushed + l; dw < lastdw; dw += 64) {
        const uint32_t v = w.ring[dw & 255u];
        for (int k = 0; k < 4; k++) {
            const int64_t by = (int64_t)dw * 4 + k;
            if (by >= w.first_byte && by < (int64_t)endbyte && by < w.limb) w.base[by] = (uint8_t)(v >> (8 * k));
        }
    }
    __syncthreads();
    return (int64_t)endbyte - w.first_byte;
}

__global__ __launch_bounds__(64) void zl1_seq_kernel(const FInfo *__restrict__ fi, const int32_t *__restrict__ blist,
                                                     BInfo *__restrict__ bi, const uint64_t *__restrict__ seqs,
                                                     uint8_t *__restrict__ bytes, uint32_t *__restrict__ hist) {
    __shared__ SeqSmem s;
    const int l = lane_id();
    const int bid = blist[blockIdx.x];
    BInfo &B = bi[bid];
    const FInfo F = fi[B.frame];
    if (F.status < 0) return;
    const int32_t flags = B.flags;
    if (flags & F_NOCOMP) {
        if (l == 0) B.secsz = 0;
        return;
    }
    const Src S = make_src(F.src, F.n);
    const int32_t ns = B.ns, nl = B.nl, bs = B.bs, be = B.be, bsz = be - bs;
    const uint64_t *sq = seqs + B.seq_off;
    g_u8 *lit = (g_u8 *)(bytes + B.lit_off);
    g_u8 *sec = (g_u8 *)(bytes + B.lit_off + bsz);
    // ---- 1. literals: runs in sequence order (+ the last literals), gathered
    // into lit[], histograms per stream segment
    for (int k = l; k < 4 * 256; k += 64) (&s.h4[0][0])[k] = 0;
    __syncthreads();
    const uint32_t seg = (uint32_t)(nl + 3) / 4;
    {
        int32_t lbase = 0, sbase = 0;  // literal / source offsets at the chunk start
        for (int32_t c0 = 0; c0 <= ns; c0 += 64) {
            const int32_t i = c0 + l;
            uint32_t ll = 0, ml = 0;
            if (i < ns) {
                const uint64_t r = sq[i];
                ll = (uint32_t)(r & 0x1FFFFu);
                ml = (uint32_t)((r >> 17) & 0x1FFFFu) + 3;
            }
            uint32_t tl = 0, ts = 0;
            const uint32_t lp = wave_scan_excl(ll, &tl);
            const uint32_t sp = wave_scan_excl(ll + ml, &ts);
            if (i == ns) ll = (uint32_t)(nl - lbase) - lp;  // the last literals: what the runs leave
            const uint32_t Lc = (ns < c0 + 64) ? tl + readlane(ll, ns - c0) : tl;
            // byte t of this chunk's literals -> its run (binary search over
            // the lanes' run starts; runs past the last one excluded)
            for (uint32_t t0 = 0; t0 < Lc; t0 += 256) {
                uint32_t bv[4];
                int32_t xs[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint32_t t = t0 + 64 * u + l;
                    const uint32_t te = t < Lc ? t : Lc - 1;
                    int lo = 0;
#pragma unroll
                    for (int st = 32; st >= 1; st >>= 1) {
                        const int c = lo + st;
                        const uint32_t lpc = (uint32_t)__shfl((int)lp, c < 64 ? c : 63, 64);
                        if (c < 64 && c0 + c <= ns && lpc <= te) lo = c;
                    }
                    const uint32_t lpr = (uint32_t)__shfl((int)lp, lo, 64), spr = (uint32_t)__shfl((int)sp, lo, 64);
                    const int32_t pos = bs + sbase + (int32_t)spr + (int32_t)(te - lpr);
                    xs[u] = t < Lc ? lbase + (int32_t)t : -1;
                    bv[u] = ldb(S, pos);
                    if (t >= Lc) bv[u] = 0u;
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (xs[u] >= 0) {
                        lit[xs[u]] = (uint8_t)bv[u];
                        const uint32_t sg = seg ? umin32((uint32_t)xs[u] / seg, 3u) : 0u;
                        atomicAdd(&s.h4[sg][bv[u]], 1u);
                    }
                }
            }
            lbase += (int32_t)Lc;
            sbase += (int32_t)ts;
        }
    }
    __syncthreads();
    for (int k = l; k < 4 * 256; k += 64) hist[(int64_t)bid * 1024 + k] = (&s.h4[0][0])[k];
    // ---- 2. sequences section (ZSTD_entropyCompressSequences_internal after the literals)
    const int64_t cap = bsz + SEC_EXTRA;
    int64_t o = 0;
    if (ns < 128) {
        if (l == 0) sec[0] = (uint8_t)ns;
        o = 1;
    } else if (ns < 0x7F00) {
        if (l == 0) sec[0] = (uint8_t)((ns >> 8) + 0x80);
        if (l == 1) sec[1] = (uint8_t)ns;
        o = 2;
    } else {
        if (l == 0) sec[0] = 0xFF;
        if (l == 1) sec[1] = (uint8_t)(ns - 0x7F00);
        if (l == 2) sec[2] = (uint8_t)((ns - 0x7F00) >> 8);
        o = 3;
    }
    if (ns == 0) {
        if (l == 0) {
            B.secsz = (int32_t)o;
            B.flags = flags & ~F_LASTNC;
        }
        return;
    }
    for (int k = l; k < 3 * 64; k += 64) (&s.cnt[0][0])[k] = 0;
    __syncthreads();
    for (int32_t i = l; i < ns; i += 64) {
        const uint64_t r = sq[i];
        const uint32_t ll = (uint32_t)(r & 0x1FFFFu), mlb = (uint32_t)((r >> 17) & 0x1FFFFu), ofv = (uint32_t)(r >> 34);
        const uint32_t lc = ll_code(ll), oc = hbit(ofv), mc = ml_code(mlb);
        atomicAdd(&s.cnt[0][lc], 1u);
        atomicAdd(&s.cnt[1][oc], 1u);
        atomicAdd(&s.cnt[2][mc], 1u);
        if (i == ns - 1) {
            s.lastc[0] = lc;
            s.lastc[1] = oc;
            s.lastc[2] = mc;
        }
    }
    __syncthreads();
    if (l == 0) {
        // ZSTD_selectEncodingType (strategy fast) + ZSTD_buildCTable, LL, OF, ML
        const uint32_t maxs[3] = {35, 31, 52}, flog[3] = {9, 8, 9}, dlog[3] = {6, 5, 6};
        for (int t = 0; t < 3; t++) {
            uint32_t *cnt = s.cnt[t];
            uint32_t max = maxs[t];
            while (!cnt[max]) max--;
            uint32_t mf = 0;
            for (uint32_t v = 0; v <= max; v++) mf = cnt[v] > mf ? cnt[v] : mf;
            const bool defOK = t != 1 || max <= 28;
            int type;
            if (mf == (uint32_t)ns) {
                type = (defOK && ns <= 2) ? 0 : 1;
            } else {
                type = 2;
                if (defOK) {
                    const uint32_t dynMin = ((1u << dlog[t]) * 9u) >> 3;
                    if ((uint32_t)ns < dynMin || mf < ((uint32_t)ns >> (dlog[t] - 1))) type = 0;
                }
            }
            s.type[t] = type;
            s.hsz[t] = 0;
            if (type == 1) {  // set_rle
                s.hdr[t][0] = (uint8_t)max;
                s.hsz[t] = 1;
                if (t == 0) build_rle(s.tLL, max);
                else if (t == 1) build_rle(s.tOF, max);
                else build_rle(s.tML, max);
            } else if (type == 0) {  // set_basic
                if (t == 0) build_ctab(s.tsym, s.tLL, LL_DEF, 35, 6);
                else if (t == 1) build_ctab(s.tsym, s.tOF, OF_DEF, 28, 5);
                else build_ctab(s.tsym, s.tML, ML_DEF, 52, 6);
            } else {  // set_compressed
                uint32_t nb1 = (uint32_t)ns;
                const uint32_t tlog = fse_opt_tlog(flog[t], (uint32_t)ns, max, 2);
                if (cnt[s.lastc[t]] > 1) {
                    cnt[s.lastc[t]]--;
                    nb1--;
                }
                fse_normalize(s.norm, tlog, cnt, nb1, max, nb1 >= 2048);
                s.hsz[t] = write_ncount(s.hdr[t], s.norm, max, tlog);
                if (t == 0) build_ctab(s.tsym, s.tLL, s.norm, max, tlog);
                else if (t == 1) build_ctab(s.tsym, s.tOF, s.norm, max, tlog);
                else build_ctab(s.tsym, s.tML, s.norm, max, tlog);
            }
        }
    }
    __syncthreads();
    // header: Symbol_Compression_Modes, then LL, OF, ML table descriptions
    if (l == 0) sec[o] = (uint8_t)((s.type[0] << 6) + (s.type[1] << 4) + (s.type[2] << 2));
    o += 1;
    int64_t lastnc = -1;
    for (int t = 0; t < 3; t++) {
        if (s.type[t] == 2) lastnc = o;
        for (int k = l; k < s.hsz[t]; k += 64) sec[o + k] = s.hdr[t][k];
        o += s.hsz[t];
    }
    // ZSTD_encodeSequences: last sequence first, 64 at a time.  A scalar
    // state pass steps the three states and leaves each sequence's state bits
    // (OF, ML, LL) in its lane; then every lane ORs its sequence's bits --
    // state bits, LL, ML and OF extra bits -- into the LDS bit ring at a
    // prefix-summed position (the serial writer's bits in its order).
    RingW w;
    rw_init(w, s.ring, sec, o, cap);
    uint32_t sML = 0, sOF = 0, sLL = 0;
    for (int64_t c0 = ns - 1; c0 >= 0; c0 -= 64) {
        const int64_t i = c0 - l;
        uint32_t ll = 0, mlb = 0, ofv = 1;
        if (i >= 0) {
            const uint64_t r = sq[i];
            ll = (uint32_t)(r & 0x1FFFFu);
            mlb = (uint32_t)((r >> 17) & 0x1FFFFu);
            ofv = (uint32_t)(r >> 34);
        }
        const uint32_t lc = ll_code(ll), mc = ml_code(mlb), oc = hbit(ofv);
        const int32_t dO = s.tOF.dnb[oc], dM = s.tML.dnb[mc], dL = s.tLL.dnb[lc];
        const int32_t fO = s.tOF.dfs[oc], fM = s.tML.dfs[mc], fL = s.tLL.dfs[lc];
        const int nj = c0 + 1 < 64 ? (int)(c0 + 1) : 64;
        uint32_t stv = 0, stn = 0;  // lane jj: sequence c0 - jj's state bits and their count
        for (int jj = 0; jj < nj; ++jj) {
            const int32_t jdO = (int32_t)readlane((uint32_t)dO, jj), jdM = (int32_t)readlane((uint32_t)dM, jj),
                          jdL = (int32_t)readlane((uint32_t)dL, jj);
            const int32_t jfO = (int32_t)readlane((uint32_t)fO, jj), jfM = (int32_t)readlane((uint32_t)fM, jj),
                          jfL = (int32_t)readlane((uint32_t)fL, jj);
            if (c0 == ns - 1 && jj == 0) {  // FSE_initCState2 with the last sequence
                const uint32_t nM = (uint32_t)((jdM + (1 << 15)) >> 16), nO = (uint32_t)((jdO + (1 << 15)) >> 16),
                               nL = (uint32_t)((jdL + (1 << 15)) >> 16);
                sML = s.tML.st[(((nM << 16) - (uint32_t)jdM) >> nM) + (uint32_t)jfM];
                sOF = s.tOF.st[(((nO << 16) - (uint32_t)jdO) >> nO) + (uint32_t)jfO];
                sLL = s.tLL.st[(((nL << 16) - (uint32_t)jdL) >> nL) + (uint32_t)jfL];
            } else {
                const uint32_t nO = (uint32_t)(((int32_t)sOF + jdO) >> 16), nM = (uint32_t)(((int32_t)sML + jdM) >> 16),
                               nL = (uint32_t)(((int32_t)sLL + jdL) >> 16);
                const uint32_t v = (sOF & ((1u << nO) - 1u)) | ((sML & ((1u << nM) - 1u)) << nO) |
                                   ((sLL & ((1u << nL) - 1u)) << (nO + nM));
                if (l == jj) {
                    stv = v;
                    stn = nO + nM + nL;
                }
                const uint32_t tO = s.tOF.st[(sOF >> nO) + (uint32_t)jfO], tM = s.tML.st[(sML >> nM) + (uint32_t)jfM],
                               tL = s.tLL.st[(sLL >> nL) + (uint32_t)jfL];
                sOF = tO;
                sML = tM;
                sLL = tL;
            }
        }
        // the lanes' bits: state bits, then LL, ML, OF extra bits
        const uint32_t nll = l < nj ? (uint32_t)LL_BITS[lc] : 0u, nml = l < nj ? (uint32_t)ML_BITS[mc] : 0u,
                       nof = l < nj ? oc : 0u;
        const uint32_t tot = stn + nll + nml + nof;
        uint32_t sum = 0;
        const uint32_t ex = wave_scan_excl(tot, &sum);
        uint64_t p = w.bitpos + ex;
        rw_or(w, p, stv, stn);
        p += stn;
        rw_or(w, p, ll, nll);
        p += nll;
        rw_or(w, p, mlb, nml);
        p += nml;
        rw_or(w, p, ofv, nof);
        w.bitpos += sum;
        rw_flush(w);
    }
    if (l == 0) {  // the final states (ML, OF, LL) and the end mark
        uint64_t p = w.bitpos;
        rw_or(w, p, sML, (uint32_t)s.tML.tlog);
        p += (uint32_t)s.tML.tlog;
        rw_or(w, p, sOF, (uint32_t)s.tOF.tlog);
        p += (uint32_t)s.tOF.tlog;
        rw_or(w, p, sLL, (uint32_t)s.tLL.tlog);
        p += (uint32_t)s.tLL.tlog;
        rw_or(w, p, 1u, 1u);
    }
    w.bitpos += (uint64_t)(s.tML.tlog + s.tOF.tlog + s.tLL.tlog + 1);
    const int64_t wp = o + rw_close(w);
    if (l == 0) {
        B.secsz = wp > cap ? -1 : (int32_t)wp;
        // zstd <= 1.3.4 decoder workaround: a last FSE_Compressed table
        // description closer than 4 bytes to the end -> raw block
        B.flags = (lastnc >= 0 && wp - lastnc < 4) ? (flags | F_LASTNC) : (flags & ~F_LASTNC);
    }
}

// ---------------------------------------------------------------------------
// kernel 3: literal sections, block decisions and the frame bytes (one wave
// per frame, blocks in order)
// ---------------------------------------------------------------------------
struct HNode {
    uint32_t count;
    uint16_t parent;
    uint8_t byte, nbBits;
};
struct LitSmem {
    uint8_t pnb[256];   // previous (confirmed) Huffman table: code lengths
    uint16_t pval[256]; //                                      codes
    uint8_t nnb[256];   // this block's new table
    uint16_t nval[256];
    uint32_t cnt[4][256];
    uint32_t tot[256];
    HNode node[2 * 256 + 2];
    uint8_t hdr[160];
    uint8_t wt[256];
    int16_t wnorm[16];
    uint32_t wcnt[16];
    uint8_t wtsym[64];
    CTab<64, 16> wct;
    uint32_t ring[256];  // Huffman stream staging (8,192 bits)
    int32_t hs, maxbits;
};

// HUF_setMaxHeight
__device__ uint32_t huf_set_max_height(HNode *huffNode, uint32_t lastNonNull, uint32_t maxNbBits) {
    const uint32_t largestBits = huffNode[lastNonNull].nbBits;
    if (largestBits <= maxNbBits) return largestBits;
    int totalCost = 0;
    const uint32_t baseCost = 1u << (largestBits - maxNbBits);
    int n = (int)lastNonNull;
    while (huffNode[n].nbBits > maxNbBits) {
        totalCost += (int)(baseCost - (1u << (largestBits - huffNode[n].nbBits)));
        huffNode[n].nbBits = (uint8_t)maxNbBits;
        n--;
    }
    while (huffNode[n].nbBits == maxNbBits) n--;
    totalCost >>= (largestBits - maxNbBits);
    const uint32_t noSymbol = 0xF0F0F0F0u;
    uint32_t rankLast[14];
    for (int i = 0; i < 14; i++) rankLast[i] = noSymbol;
    {
        uint32_t currentNbBits = maxNbBits;
        for (int pos = n; pos >= 0; pos--) {
            if (huffNode[pos].nbBits >= currentNbBits) continue;
            currentNbBits = huffNode[pos].nbBits;
            rankLast[maxNbBits - currentNbBits] = (uint32_t)pos;
        }
    }
    for (int guard = 0; totalCost > 0 && guard < 100000; guard++) {
        uint32_t nBitsToDecrease = hbit((uint32_t)totalCost) + 1;
        for (; nBitsToDecrease > 1; nBitsToDecrease--) {
            const uint32_t highPos = rankLast[nBitsToDecrease], lowPos = rankLast[nBitsToDecrease - 1];
            if (highPos == noSymbol) continue;
            if (lowPos == noSymbol) break;
            const uint32_t highTotal = huffNode[highPos].count, lowTotal = 2 * huffNode[lowPos].count;
            if (highTotal <= lowTotal) break;
        }
        while (nBitsToDecrease <= 12 && rankLast[nBitsToDecrease] == noSymbol) nBitsToDecrease++;
        totalCost -= 1 << (nBitsToDecrease - 1);
        if (rankLast[nBitsToDecrease - 1] == noSymbol) rankLast[nBitsToDecrease - 1] = rankLast[nBitsToDecrease];
        huffNode[rankLast[nBitsToDecrease]].nbBits++;
        if (rankLast[nBitsToDecrease] == 0)
            rankLast[nBitsToDecrease] = noSymbol;
        else {
            rankLast[nBitsToDecrease]--;
            if (huffNode[rankLast[nBitsToDecrease]].nbBits != maxNbBits - nBitsToDecrease)
                rankLast[nBitsToDecrease] = noSymbol;
        }
    }
    for (int guard = 0; totalCost < 0 && guard < 100000; guard++) {
        if (rankLast[1] == noSymbol) {
            while (huffNode[n].nbBits == maxNbBits) n--;
            huffNode[n + 1].nbBits--;
            rankLast[1] = (uint32_t)(n + 1);
            totalCost++;
            continue;
        }
        huffNode[rankLast[1] + 1].nbBits--;
        rankLast[1]++;
        totalCost++;
    }
    return maxNbBits;
}

// HUF_buildCTable_wksp's node reset and its stable sort of the symbols by
// decreasing count (the insertion sort's order: ties keep symbol order), as a
// rank per symbol -- all lanes
__device__ void huf_sort(LitSmem &s, uint32_t maxsv) {
    const int l = lane_id();
    for (int i = l; i < 2 * 256 + 2; i += 64) {
        s.node[i].count = 0;
        s.node[i].parent = 0;
        s.node[i].byte = 0;
        s.node[i].nbBits = 0;
    }
    __syncthreads();
    HNode *const huffNode = s.node + 1;
    for (uint32_t i = (uint32_t)l; i <= maxsv; i += 64) {
        const uint32_t c = s.tot[i];
        uint32_t r = 0;
        for (uint32_t j = 0; j <= maxsv; j++) {
            const uint32_t cj = s.tot[j];
            r += (cj > c || (cj == c && j < i)) ? 1u : 0u;
        }
        huffNode[r].count = c;
        huffNode[r].byte = (uint8_t)i;
    }
    __syncthreads();
}

// HUF_buildCTable_wksp into (nnb, nval) after huf_sort; lane 0; returns the
// max code length
__device__ uint32_t huf_build(LitSmem &s, uint32_t maxsv, uint32_t maxNbBits) {
    HNode *const huffNode = s.node + 1;
    const int STARTNODE = 256;
    int nonNullRank = (int)maxsv;
    while (huffNode[nonNullRank].count == 0) nonNullRank--;
    int lowS = nonNullRank, nodeNb = STARTNODE;
    const int nodeRoot = nodeNb + lowS - 1;
    int lowN = nodeNb;
    huffNode[nodeNb].count = huffNode[lowS].count + huffNode[lowS - 1].count;
    huffNode[lowS].parent = huffNode[lowS - 1].parent = (uint16_t)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int n = nodeNb; n <= nodeRoot; n++) huffNode[n].count = 1u << 30;
    s.node[0].count = 1u << 31;
    while (nodeNb <= nodeRoot) {
        const int n1 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        const int n2 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        huffNode[nodeNb].count = huffNode[n1].count + huffNode[n2].count;
        huffNode[n1].parent = huffNode[n2].parent = (uint16_t)nodeNb;
        nodeNb++;
    }
    huffNode[nodeRoot].nbBits = 0;
    for (int n = nodeRoot - 1; n >= STARTNODE; n--) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    for (int n = 0; n <= nonNullRank; n++) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    maxNbBits = huf_set_max_height(huffNode, (uint32_t)nonNullRank, maxNbBits);
    uint16_t nbPerRank[13], valPerRank[13];
    for (int i = 0; i < 13; i++) nbPerRank[i] = valPerRank[i] = 0;
    for (int n = 0; n <= nonNullRank; n++) nbPerRank[huffNode[n].nbBits]++;
    {
        uint16_t mn = 0;
        for (int n = (int)maxNbBits; n > 0; n--) {
            valPerRank[n] = mn;
            mn += nbPerRank[n];
            mn >>= 1;
        }
    }
    for (int i = 0; i < 256; i++) {
        s.nnb[i] = 0;
        s.nval[i] = 0;
    }
    for (int n = 0; n <= (int)maxsv; n++) s.nnb[huffNode[n].byte] = huffNode[n].nbBits;
    for (int n = 0; n <= (int)maxsv; n++) s.nval[n] = valPerRank[s.nnb[n]]++;
    return maxNbBits;
}

// HUF_writeCTable (weights FSE-compressed when that is smaller) into s.hdr; lane 0; 0 = impossible
__device__ int huf_write_ctable(LitSmem &s, uint32_t maxsv, uint32_t huffLog) {
    uint8_t b2w[13];
    b2w[0] = 0;
    for (uint32_t n = 1; n < huffLog + 1; n++) b2w[n] = (uint8_t)(huffLog + 1 - n);
    for (uint32_t n = 0; n < maxsv; n++) s.wt[n] = b2w[s.nnb[n]];
    // HUF_compressWeights
    const uint32_t wtSize = maxsv;
    int hsz = 0;
    if (wtSize > 1) {
        for (int i = 0; i < 16; i++) s.wcnt[i] = 0;
        for (uint32_t i = 0; i < wtSize; i++) s.wcnt[s.wt[i]]++;
        uint32_t wmax = 12;
        while (!s.wcnt[wmax]) wmax--;
        uint32_t maxc = 0;
        for (uint32_t i = 0; i <= wmax; i++) maxc = s.wcnt[i] > maxc ? s.wcnt[i] : maxc;
        if (maxc == wtSize) {
            hsz = 1;
        } else if (maxc == 1) {
            hsz = 0;
        } else {
            const uint32_t tlog = fse_opt_tlog(6, wtSize, wmax, 2);
            if (fse_normalize(s.wnorm, tlog, s.wcnt, wtSize, wmax, false) >= 0) {
                int o = 1 + write_ncount(s.hdr + 1, s.wnorm, wmax, tlog);
                build_ctab(s.wtsym, s.wct, s.wnorm, wmax, tlog);
                // FSE_compress_usingCTable: two states, last symbols first
                uint64_t bc = 0;
                int bp = 0;
                const int lim = 159;
                auto flush = [&]() {
                    while (bp >= 8) {
                        if (o < lim) s.hdr[o] = (uint8_t)bc;
                        o++;
                        bc >>= 8;
                        bp -= 8;
                    }
                };
                auto add = [&](uint32_t v, int nb) {
                    bc |= ((uint64_t)v & ((1ull << nb) - 1ull)) << bp;
                    bp += nb;
                };
                auto init = [&](uint32_t sym) -> uint32_t {
                    const int32_t dnb = s.wct.dnb[sym];
                    const uint32_t nbo = (uint32_t)((dnb + (1 << 15)) >> 16);
                    return s.wct.st[(((nbo << 16) - (uint32_t)dnb) >> nbo) + (uint32_t)s.wct.dfs[sym]];
                };
                auto enc = [&](uint32_t &st, uint32_t sym) {
                    const uint32_t nbo = (uint32_t)(((int32_t)st + s.wct.dnb[sym]) >> 16);
                    add(st, (int)nbo);
                    st = s.wct.st[(st >> nbo) + (uint32_t)s.wct.dfs[sym]];
                };
                int ip = (int)wtSize;
                uint32_t s1, s2;
                if (wtSize > 2) {
                    if (wtSize & 1) {
                        s1 = init(s.wt[--ip]);
                        s2 = init(s.wt[--ip]);
                        enc(s1, s.wt[--ip]);
                        flush();
                    } else {
                        s2 = init(s.wt[--ip]);
                        s1 = init(s.wt[--ip]);
                    }
                    if ((wtSize - 2) & 2) {
                        enc(s2, s.wt[--ip]);
                        enc(s1, s.wt[--ip]);
                        flush();
                    }
                    while (ip > 0) {
                        enc(s2, s.wt[--ip]);
                        enc(s1, s.wt[--ip]);
                        enc(s2, s.wt[--ip]);
                        enc(s1, s.wt[--ip]);
                        flush();
                    }
                    add(s2, (int)tlog);
                    flush();
                    add(s1, (int)tlog);
                    flush();
                    add(1, 1);
                    flush();
                    if (bp > 0) {
                        if (o < lim) s.hdr[o] = (uint8_t)bc;
                        o++;
                    }
                    hsz = o - 1;
                } else {
                    hsz = 0;
                }
            }
        }
    }
    if (hsz > 1 && hsz < (int)(maxsv / 2)) {
        s.hdr[0] = (uint8_t)hsz;
        return hsz + 1;
    }
    if (maxsv > 128) return 0;
    s.hdr[0] = (uint8_t)(128 + (maxsv - 1));
    s.wt[maxsv] = 0;
    for (uint32_t n = 0; n < maxsv; n += 2) s.hdr[n / 2 + 1] = (uint8_t)((s.wt[n] << 4) + s.wt[n + 1]);
    return (int)((maxsv + 1) / 2 + 1);
}

// wave copy dst[0, len) <- src[0, len): 16-byte aligned stores, dword loads
// of the source that never touch a dword without a source byte
__device__ void wave_copy(g_u8 *dst, const uint8_t *srcp, int64_t len) {
    const int l = lane_id();
    if (len <= 0) return;
    const int64_t h16 = (int64_t)((16u - (uint32_t)((uintptr_t)dst & 15u)) & 15u);
    const int64_t head = len < h16 ? len : h16;
    const gc_u8 *sb = (const gc_u8 *)srcp;
    if (l < head) dst[l] = sb[l];
    const Src S = make_src(srcp, (int32_t)(len < 0x7FFFFFFF ? len : 0x7FFFFFFF));
    int64_t x = head;
    for (; x + 16 <= len; x += 1024) {
        const int64_t y = x + 16 * l;
        if (y + 16 <= len) *(g_u4 *)(dst + y) = ld128(S, (int32_t)y);
    }
    const int64_t xe = head + ((len - head) & ~(int64_t)15);
    if (xe + l < len) dst[xe + l] = sb[xe + l];
}

__device__ __forceinline__ void put_bytes(g_u8 *dst, int64_t o, uint64_t v, int n) {
    const int l = lane_id();
    if (l < n) dst[o + l] = (uint8_t)(v >> (8 * l));
}

// encode literals lit[a, b) with table (nb, val), last symbol first, into dst
// at byte o; returns the stream bytes (end mark included)
__device__ int64_t huf_stream(uint32_t *ring, const uint8_t *tnb, const uint16_t *tval, const gc_u8 *lit, int32_t a,
                              int32_t b, g_u8 *dst, int64_t o) {
    const int l = lane_id();
    // ring bit 0 = bit 0 of the dword at (dst + o) & ~3
    const uint32_t boff = (uint32_t)((uintptr_t)(dst + o) & 3u) * 8u;
    g_u8 *base = (g_u8 *)((uintptr_t)(dst + o) & ~(uintptr_t)3);
    g_u32 *wbase = (g_u32 *)base;
    const int64_t first_byte = (int64_t)(boff >> 3);  // bytes of dword 0 before the stream: keep
    for (int k = l; k < 256; k += 64) ring[k] = 0;
    __syncthreads();
    uint64_t bitpos = boff;  // absolute bit position from base
    uint64_t flushed = 0;    // dwords stored
    for (int32_t c0 = b - 1; c0 >= a; c0 -= 64) {
        const int32_t i = c0 - l;
        uint32_t len = 0, code = 0;
        if (i >= a) {
            const uint32_t sym = lit[i];
            len = tnb[sym];
            code = tval[sym];
        }
        uint32_t tot = 0;
        const uint32_t ex = wave_scan_excl(len, &tot);
        if (len) {
            const uint64_t p = bitpos + ex;
            const uint32_t d = (uint32_t)(p >> 5) & 255u, sh = (uint32_t)(p & 31u);
            atomicOr(&ring[d], code << sh);
            if (sh + len > 32) atomicOr(&ring[(d + 1) & 255u], code >> (32 - sh));
        }
        __syncthreads();
        bitpos += tot;
        // store the complete dwords
        const uint64_t full = bitpos >> 5;
        for (uint64_t dw = flushed + l; dw < full; dw += 64) {
            const uint32_t v = ring[dw & 255u];
            if (dw == 0 && first_byte > 0) {
                for (int k = (int)first_byte; k < 4; k++) base[k] = (uint8_t)(v >> (8 * k));
            } else {
                wbase[dw] = v;
            }
            ring[dw & 255u] = 0;
        }
        __syncthreads();
        flushed = full;
    }
    // end mark, last partial dword (bytes up to the end only)
    if (l == 0) {
        const uint32_t d = (uint32_t)(bitpos >> 5) & 255u, sh = (uint32_t)(bitpos & 31u);
        ring[d] |= 1u << sh;
    }
    __syncthreads();
    bitpos += 1;
    const uint64_t endbyte = (bitpos + 7) >> 3;  // bytes from base
    const uint64_t lastdw = (endbyte + 3) >> 2;
    for (uint64_t dw = flushed + l; dw < lastdw; dw += 64) {
        const uint32_t v = ring[dw & 255u];
        const int64_t b0 = (int64_t)dw * 4;
        for (int k = 0; k < 4; k++) {
            const int64_t by = b0 + k;
            if (by >= first_byte && by < (int64_t)endbyte) base[by] = (uint8_t)(v >> (8 * k));
        }
    }
    __syncthreads();
    return (int64_t)endbyte - first_byte;
}

// The literal sections and the block bytes, in three launches (the Huffman
// reuse decision is serial per frame, the heavy work is per block):
//   zl1_lithuf    one wave per block: histogram totals, and the block's new
//                 Huffman table + its description (HUF_buildCTable,
//                 HUF_writeCTable) whenever the block may need one;
//   zl1_litdec    one wave per frame, block after block: the frame header,
//                 HUF_compress_internal's choices (repeat check, size
//                 estimates, exact stream sizes from the segment histograms),
//                 the raw / RLE / compressed choice and every block's offset;
//                 a wrong confirmation guess sends the frame back to the parse;
//   zl1_litwrite  one wave per block: the block written in place.
struct LitTab {
    uint8_t nnb[256];   // the block's new table (zl1_lithuf)
    uint16_t nval[256];
    uint8_t hdr[160];
    int32_t hs;         // description bytes (0: impossible), -1: not built
    int32_t lkind;      // 0 raw, 1 RLE, 2 Huffman new table, 3 Huffman previous table (zl1_litdec)
    int64_t op;         // block header offset in dst
    int64_t cS;         // 0 raw block, 1 RLE block, else the compressed block size
    int64_t clit;       // Huffman streams + description bytes
    int32_t tsrc;       // block whose new table the streams use
    int32_t single;     // one stream
};

__global__ __launch_bounds__(64) void zl1_lithuf_kernel(const FInfo *__restrict__ fi, const int32_t *__restrict__ blist,
                                                        const BInfo *__restrict__ bi, const uint32_t *__restrict__ hist,
                                                        LitTab *__restrict__ lt) {
    __shared__ LitSmem s;
    const int l = lane_id();
    const int32_t g = blist[blockIdx.x];
    const BInfo B = bi[g];
    if (fi[B.frame].status < 0) return;
    LitTab &T = lt[g];
    int32_t hs = -1;
    const int32_t L = B.nl;
    if (!(B.flags & F_NOCOMP) && L > 63) {
        for (int i = l; i < 256; i += 64)
            s.tot[i] = hist[(int64_t)g * 1024 + i] + hist[(int64_t)g * 1024 + 256 + i] +
                       hist[(int64_t)g * 1024 + 512 + i] + hist[(int64_t)g * 1024 + 768 + i];
        __syncthreads();
        uint32_t mx = 0, largest = 0;
        for (int i = l; i < 256; i += 64) {
            if (s.tot[i]) mx = umax32(mx, (uint32_t)i);
            largest = umax32(largest, s.tot[i]);
        }
        const uint32_t maxsv = dwave_max(mx);
        largest = dwave_max(largest);
        if (largest != (uint32_t)L && largest > (uint32_t)(L >> 7) + 4) {  // (else RLE or raw: no table)
            const uint32_t hlog0 = fse_opt_tlog(11, (uint32_t)L, maxsv, 1);
            huf_sort(s, maxsv);
            if (l == 0) {
                s.maxbits = (int32_t)huf_build(s, maxsv, hlog0);
                s.hs = huf_write_ctable(s, maxsv, (uint32_t)s.maxbits);
            }
            __syncthreads();
            hs = s.hs;
            for (int i = l; i < 256; i += 64) {
                T.nnb[i] = s.nnb[i];
                T.nval[i] = s.nval[i];
            }
            for (int i = l; i < hs && i < 160; i += 64) T.hdr[i] = s.hdr[i];
        }
    }
    if (l == 0) T.hs = hs;
}

struct LitDecSmem {
    uint8_t pnb[256];  // previous (confirmed) Huffman table: code lengths
    uint8_t nnb[256];  // this block's new table
    uint32_t cnt[4][256];
    uint32_t tot[256];
};

__global__ __launch_bounds__(64) void zl1_litdec_kernel(FInfo *__restrict__ fi, const int32_t *__restrict__ flist,
                                                        BInfo *__restrict__ bi, const uint32_t *__restrict__ hist,
                                                        LitTab *__restrict__ lt, int32_t *__restrict__ ret) {
    __shared__ LitDecSmem s;
    const int l = lane_id();
    const int fidx = flist[blockIdx.x];
    FInfo &FR = fi[fidx];
    const FInfo F = FR;
    if (F.status < 0) return;
    g_u8 *dst = (g_u8 *)F.dst;
    // frame header (ZSTD_writeFrameHeader: no checksum, no dictionary, FCS)
    const uint32_t n = (uint32_t)F.n;
    const bool single1 = (1u << F.wlog) >= n;
    const uint32_t fcs = (n >= 256) + (n >= 65536 + 256);
    int64_t op = 0;
    {
        uint64_t hv = 0xFD2FB528ull | ((uint64_t)((single1 ? 0x20 : 0) | (fcs << 6)) << 32);
        int hn = 5;
        if (!single1) {
            hv |= (uint64_t)((F.wlog - 10) << 3) << 40;
            hn = 6;
        }
        put_bytes(dst, 0, hv, hn);
        op = hn;
        if (fcs == 0) {
            if (single1) {
                put_bytes(dst, op, n, 1);
                op += 1;
            }
        } else if (fcs == 1) {
            put_bytes(dst, op, n - 256, 2);
            op += 2;
        } else {
            put_bytes(dst, op, n, 4);
            op += 4;
        }
    }
    if (F.nb == 0) {  // empty input: one last empty raw block
        put_bytes(dst, op, 1, 3);
        op += 3;
    }
    for (int k = l; k < 256; k += 64) s.pnb[k] = 0;
    int prep = 0;          // HUF repeat mode of the previous confirmed table: 0 none, 1 check
    int32_t ptab = -1;     // the block whose new table that is
    __syncthreads();
    for (int32_t k = 0; k < F.nb; k++) {
        const int32_t g = F.b0 + k;
        BInfo &B = bi[g];
        LitTab &T = lt[g];
        const int32_t bs = B.bs, be = B.be, bsz = be - bs, flags = B.flags;
        const bool last = k == F.nb - 1;
        int64_t cS = 0;
        int lkind = 0;  // literal section: 0 raw, 1 RLE, 2 Huffman new table, 3 Huffman previous table
        int64_t litsz = 0, clit = 0;
        bool single = false;
        int32_t L = 0;
        if (!(flags & F_NOCOMP)) {
            L = B.nl;
            for (int i = l; i < 1024; i += 64) (&s.cnt[0][0])[i] = hist[(int64_t)g * 1024 + i];
            __syncthreads();
            for (int i = l; i < 256; i += 64) s.tot[i] = s.cnt[0][i] + s.cnt[1][i] + s.cnt[2][i] + s.cnt[3][i];
            __syncthreads();
            // ---- ZSTD_compressLiterals + HUF_compress_internal
            const int64_t fl = 1 + (L > 31) + (L > 4095);
            const int32_t minGain = (L >> 6) + 2;
            const int lh = 3 + (L >= 1024) + (L >= 16384);
            single = L < 256;
            lkind = 0;
            if (L > 63) {
                uint32_t largest = 0;
                for (int i = l; i < 256; i += 64) largest = umax32(largest, s.tot[i]);
                largest = dwave_max(largest);
                int repeat = prep;
                const bool prefer = L <= 1024;
                if (largest == (uint32_t)L) {
                    clit = 1;
                } else if (largest <= (uint32_t)(L >> 7) + 4) {
                    clit = 0;
                } else {
                    if (repeat == 1) {
                        bool bad = false;
                        for (int i = l; i < 256; i += 64) bad |= (s.tot[i] != 0) && (s.pnb[i] == 0);
                        if (ballot(bad)) repeat = 0;
                    }
                    // exact stream sizes of a table: sum of code bits per segment
                    auto streams = [&](const uint8_t *tnb) -> int64_t {
                        uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0;
                        for (int i = l; i < 256; i += 64) {
                            b0 += s.cnt[0][i] * tnb[i];
                            b1 += s.cnt[1][i] * tnb[i];
                            b2 += s.cnt[2][i] * tnb[i];
                            b3 += s.cnt[3][i] * tnb[i];
                        }
                        b0 = dwave_sum(b0); b1 = dwave_sum(b1); b2 = dwave_sum(b2); b3 = dwave_sum(b3);
                        if (single) return (int64_t)((b0 + b1 + b2 + b3 + 1 + 7) >> 3);
                        return 6 + (int64_t)((b0 + 8) >> 3) + ((b1 + 8) >> 3) + ((b2 + 8) >> 3) + ((b3 + 8) >> 3);
                    };
                    auto estimate = [&](const uint8_t *tnb) -> int64_t {
                        uint32_t a = 0;
                        for (int i = l; i < 256; i += 64) a += s.tot[i] * tnb[i];
                        return (int64_t)(dwave_sum(a) >> 3);
                    };
                    auto ct_internal = [&](const uint8_t *tnb, int64_t hs) -> int64_t {
                        const int64_t t = hs + streams(tnb);
                        return t >= L - 1 ? 0 : t;
                    };
                    if (prefer && repeat != 0) {
                        clit = ct_internal(s.pnb, 0);
                        lkind = 3;
                    } else {
                        // the new table zl1_lithuf built for exactly this case
                        for (int i = l; i < 256; i += 64) s.nnb[i] = T.nnb[i];
                        __syncthreads();
                        const int64_t hs = T.hs;
                        bool decided = false;
                        if (hs == 0) {
                            clit = 0;
                            decided = true;
                        } else if (repeat != 0) {
                            const int64_t oldSize = estimate(s.pnb), newSize = estimate(s.nnb);
                            if (oldSize <= hs + newSize || hs + 12 >= L) {
                                clit = ct_internal(s.pnb, 0);
                                lkind = 3;
                                decided = true;
                            }
                        }
                        if (!decided) {
                            if (hs + 12 >= L) {
                                clit = 0;
                            } else {
                                clit = ct_internal(s.nnb, hs);
                                lkind = 2;
                            }
                        }
                    }
                }
                if (clit == 0 || clit >= L - minGain) {
                    lkind = 0;
                } else if (clit == 1) {
                    lkind = 1;
                }
            }
            litsz = lkind == 0 ? fl + L : lkind == 1 ? fl + 1 : lh + clit;
            // ---- the block: ZSTD_entropyCompressSequences + ZSTD_compressBlock_internal
            const int32_t secsz = B.secsz;
            if (secsz < 0 || (flags & F_LASTNC)) {
                cS = 0;
            } else {
                const int64_t c = litsz + secsz;
                cS = c >= (int64_t)bsz - ((bsz >> 6) + 2) ? 0 : c;
            }
            if (k > 0 && cS < 25 && (flags & F_RLE)) cS = 1;
        }
        const bool confirmed = cS > 1;
        const bool assumed = (flags & F_ASSUMED) != 0;
        if (confirmed != assumed && !last && (B.rout0 != B.rin0 || B.rout1 != B.rin1)) {
            // the parse handed the wrong offsets to block k + 1: parse again
            // with this block's outcome known
            for (int32_t i = l; i <= k; i += 64) {
                BInfo &Bi = bi[F.b0 + i];
                if (i < k) Bi.conf = (Bi.flags & F_ASSUMED) ? 1 : 2;
            }
            if (l == 0) {
                B.conf = confirmed ? 1 : 2;
                FR.status = 1;
            }
            return;
        }
        if (l == 0) {
            T.op = op;
            T.cS = cS;
            T.lkind = lkind;
            T.clit = clit;
            T.tsrc = lkind == 3 ? ptab : g;
            T.single = single;
        }
        op += cS == 0 ? 3 + bsz : cS == 1 ? 4 : 3 + cS;
        if (confirmed && lkind == 2) {  // this block's new table becomes the previous table
            for (int i = l; i < 256; i += 64) s.pnb[i] = s.nnb[i];
            prep = 1;
            ptab = g;
        }
        __syncthreads();
    }
    if (l == 0) {
        ret[fidx] = op <= F.cap ? (int32_t)op : -2;
        FR.status = 0;
    }
}

struct LitWSmem {
    uint8_t tnb[256];
    uint16_t tval[256];
    uint32_t ring[256];  // Huffman stream staging (8,192 bits)
};

__global__ __launch_bounds__(64) void zl1_litwrite_kernel(const FInfo *__restrict__ fi, const int32_t *__restrict__ blist,
                                                          const BInfo *__restrict__ bi, const uint8_t *__restrict__ bytes,
                                                          const LitTab *__restrict__ lt) {
    __shared__ LitWSmem s;
    const int l = lane_id();
    const int32_t g = blist[blockIdx.x];
    const BInfo B = bi[g];
    const FInfo F = fi[B.frame];
    if (F.status != 0) return;  // (zl1_litdec sent the frame back to the parse)
    const LitTab &T = lt[g];
    const int64_t op = T.op, cS = T.cS;
    const int lkind = T.lkind;
    const int64_t clit = T.clit;
    const bool single = T.single != 0;
    g_u8 *dst = (g_u8 *)F.dst;
    const Src S = make_src(F.src, F.n);
    const int32_t bs = B.bs, bsz = B.be - B.bs;
    const bool last = g - F.b0 == F.nb - 1;
    const uint8_t *lit8 = bytes + B.lit_off;
    const gc_u8 *lit = (const gc_u8 *)lit8;
    if (cS == 0) {
        put_bytes(dst, op, (uint32_t)(last ? 1 : 0) | ((uint32_t)bsz << 3), 3);
        wave_copy(dst + op + 3, F.src + bs, bsz);
        return;
    }
    if (cS == 1) {
        put_bytes(dst, op, (uint32_t)(last ? 1 : 0) | (1u << 1) | ((uint32_t)bsz << 3), 3);
        const uint32_t rb = ldb(S, bs);
        if (l == 0) dst[op + 3] = (uint8_t)rb;
        return;
    }
    put_bytes(dst, op, (uint32_t)(last ? 1 : 0) | (2u << 1) | ((uint32_t)cS << 3), 3);
    int64_t o = op + 3;
    const int32_t L = B.nl;
    const int64_t fl = 1 + (L > 31) + (L > 4095);
    if (lkind == 0 || lkind == 1) {
        const uint32_t t = lkind;
        const uint64_t hv = fl == 1 ? (t | ((uint64_t)L << 3))
                                    : fl == 2 ? (t | (1u << 2) | ((uint64_t)L << 4)) : (t | (3u << 2) | ((uint64_t)L << 4));
        put_bytes(dst, o, hv, (int)fl);
        o += fl;
        if (lkind == 0) {
            wave_copy(dst + o, lit8, L);
            o += L;
        } else {
            if (l == 0) dst[o] = lit[0];
            o += 1;
        }
    } else {
        const int lh = 3 + (L >= 1024) + (L >= 16384);
        const uint64_t ht = lkind == 2 ? 2 : 3;
        uint64_t hv;
        if (lh == 3) hv = ht | ((uint64_t)(single ? 0 : 1) << 2) | ((uint64_t)L << 4) | ((uint64_t)clit << 14);
        else if (lh == 4) hv = ht | (2ull << 2) | ((uint64_t)L << 4) | ((uint64_t)clit << 18);
        else hv = ht | (3ull << 2) | ((uint64_t)L << 4) | ((uint64_t)clit << 22);
        put_bytes(dst, o, hv, lh);
        o += lh;
        const LitTab &U = lt[T.tsrc];
        for (int i = l; i < 256; i += 64) {
            s.tnb[i] = U.nnb[i];
            s.tval[i] = U.nval[i];
        }
        if (lkind == 2) {
            for (int i = l; i < T.hs; i += 64) dst[o + i] = T.hdr[i];
            o += T.hs;
        }
        __syncthreads();
        if (single) {
            o += huf_stream(s.ring, s.tnb, s.tval, lit, 0, L, dst, o);
        } else {
            const int32_t sg = (L + 3) / 4;
            const int64_t jt = o;
            o += 6;
            int64_t sz[4];
            for (int q = 0; q < 4; q++) {
                const int32_t a = q * sg, b = q < 3 ? a + sg : L;
                sz[q] = huf_stream(s.ring, s.tnb, s.tval, lit, a, b, dst, o);
                o += sz[q];
            }
            put_bytes(dst, jt, (uint64_t)sz[0] | ((uint64_t)sz[1] << 16) | ((uint64_t)sz[2] << 32), 6);
        }
    }
    // the sequences section
    wave_copy(dst + o, bytes + B.lit_off + bsz, B.secsz);
}

}  // namespace zl1
}  // namespace jfs

// ---------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------
namespace {
using namespace jfs::zl1;
struct ZL1Scratch {
    std::mutex mu;
    uint8_t *d = nullptr;
    size_t cap = 0;
    bool grow(size_t need) {
        if (cap >= need) return true;
        if (d) (void)hipFree(d);  // hipFree waits for work still using it
        d = nullptr;
        cap = 0;
        size_t want = (size_t)64 << 20;
        while (want < need) want <<= 1;
        if (hipMalloc((void **)&d, want) != hipSuccess) return false;
        cap = want;
        return true;
    }
};
// two per device: the coalescer's two lanes encode at once
ZL1Scratch g_zl1[16][2];
inline size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }
}  // namespace

#ifdef JFS_PROF
extern "C" int jfs_zpprof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::zl1::g_zpprof), sizeof(unsigned long long) * 12) == hipSuccess ? 0 : -1;
}
extern "C" int jfs_zpprof_reset() {
    unsigned long long z[12] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::zl1::g_zpprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

// Small batches take the block-parallel speculative parse (zl1_spec_*) for
// their multi-block frames: at most JFS_ZL1_SPEC_MAX blocks in all (default
// 2,048; 0 = never).  Larger batches fill the GPU with frame-serial parses.
// segments per block of the speculative parse at most (1, 2, 4, 8, 16;
// default 16: a lone 4 MiB frame 37.5 ms one-call vs 40.8 at 8, 68 at 4)
int spec_segs() {  // (read per launch: the tests sweep it)
    const char *e = getenv("JFS_ZL1_SEGS");
    const int p = e ? atoi(e) : 16;
    int q = 1;
    while (q * 2 <= p && q < 16) q *= 2;
    return q;
}

// slots (segments) a small batch may take at most (JFS_ZL1_SLOTS; default
// 4,096: 20 concurrent 4 MiB frames take 4 segments per block, 187 ms a burst
// vs 198 with whole blocks and 228 with 2 -- the late rounds, with few
// changed segments, are the cheap ones; 128 KiB of scratch per slot)
int spec_slots() {
    const char *e = getenv("JFS_ZL1_SLOTS");
    return e ? std::max(1, atoi(e)) : 4096;
}

int spec_max_blocks() {
    static int v = [] {
        const char *e = getenv("JFS_ZL1_SPEC_MAX");
        return e ? std::max(0, atoi(e)) : 2048;
    }();
    return v;
}

extern "C" int jfs_launch_zstd_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    if (nblk <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
    // a free scratch of this device (blocking on the first only if both are taken)
    ZL1Scratch *zp = nullptr;
    std::unique_lock<std::mutex> lk;
    for (int i = 0; i < 2 && !zp; i++) {
        std::unique_lock<std::mutex> t(g_zl1[dev][i].mu, std::try_to_lock);
        if (t.owns_lock()) {
            lk = std::move(t);
            zp = &g_zl1[dev][i];
        }
    }
    if (!zp) {
        lk = std::unique_lock<std::mutex>(g_zl1[dev][0].mu);
        zp = &g_zl1[dev][0];
    }
    ZL1Scratch &z = *zp;
    // the descriptors may have been written on this stream: read them after it drains
    std::vector<jfs_dev_block> h(nblk);
    if (hipMemcpyAsync(h.data(), d_blocks, sizeof(jfs_dev_block) * nblk, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    std::vector<FInfo> fi(nblk);
    std::vector<BInfo> bi;
    std::vector<int32_t> hret(nblk, -2);
    int64_t seq_total = 0, byte_total = 0;
    for (int f = 0; f < nblk; f++) {
        FInfo &F = fi[f];
        const int64_t n = h[f].src_len, cap = h[f].dst_cap;
        F.src = (const uint8_t *)h[f].src;
        F.dst = (uint8_t *)h[f].dst;
        F.n = (int32_t)std::max<int64_t>(0, std::min<int64_t>(n, 0x7FFFFFFF));
        F.cap = (int32_t)std::max<int64_t>(0, std::min<int64_t>(cap, 0x7FFFFFFF));
        const Params p = params_of(F.n);
        F.wlog = p.wlog;
        F.hlog = p.hlog;
        F.mls = p.mls;
        F.b0 = (int32_t)bi.size();
        F.nb = 0;
        // compress.go:86-89: cap(dst) < CompressBound -> "buffer too short"
        F.status = (n < 0 || n > 0x7FFFFF00ll || cap < zbound(n)) ? -2 : 0;
        if (F.status < 0) continue;
        for (int64_t bs = 0; bs < n; bs += BLK) {
            BInfo B;
            memset(&B, 0, sizeof(B));
            B.frame = f;
            B.bs = (int32_t)bs;
            B.be = (int32_t)std::min<int64_t>(n, bs + BLK);
            const int32_t bsz = B.be - B.bs;
            B.seq_off = seq_total;
            B.lit_off = byte_total;
            seq_total += seq_cap(bsz);
            byte_total += (int64_t)a256((size_t)(2 * (int64_t)bsz + SEC_EXTRA));
            bi.push_back(B);
            F.nb++;
        }
    }
    const int nbk = (int)bi.size();
    // speculative parse: the multi-block (wide) frames of a small batch, their
    // blocks in slots grouped by hashLog
    // frames, their blocks in slots grouped by hashLog; a block takes
    // segsz-byte segments (one slot each) when the batch has few blocks: the
    // most segments per block (<= JFS_ZL1_SEGS, default 16) that keep the slots
    // within the ~1,024 waves the GPU holds at once (four per CU by LDS)
    std::vector<int32_t> sf, sslot, snseg, bfirst;
    std::vector<SpecB> slots;
    std::vector<std::pair<uint32_t, std::pair<int, int>>> sgrp;  // hashLog -> (first slot, slots)
    int32_t segsz = BLK;
    {
        int64_t cand = 0, fmax = 0;
        for (int f = 0; f < nblk; f++)
            if (fi[f].status == 0 && fi[f].nb >= 2 && fi[f].n >= 65536) {
                cand += fi[f].nb;
                fmax = std::max<int64_t>(fmax, fi[f].nb);
            }
        if (cand > 0 && cand <= spec_max_blocks()) {
            int P = spec_segs();
            while (P > 1 && (cand * P > spec_slots() || fmax * P > SPEC_MAXSEG)) P >>= 1;
            segsz = BLK / P;
            for (uint32_t hl = 6; hl <= 14; hl++) {
                const int g0 = (int)slots.size();
                for (int f = 0; f < nblk; f++) {
                    const FInfo &F = fi[f];
                    if (F.status != 0 || F.nb < 2 || F.n < 65536 || F.hlog != hl) continue;
                    sf.push_back(f);
                    sslot.push_back((int32_t)slots.size());
                    for (int k = 0; k < F.nb; k++) {
                        const BInfo &B = bi[F.b0 + k];
                        bfirst.push_back((int32_t)slots.size());
                        for (int32_t q = 0; q == 0 || B.bs + q * segsz < B.be; q++) {
                            SpecB x;
                            memset(&x, 0, sizeof(x));
                            x.blk = F.b0 + k;
                            x.q = q;
                            // round 0's guess of the state handed in: the loop
                            // at the segment start (any valid state will do)
                            x.in.ip0 = x.in.anchor = B.bs + q * segsz;
                            x.in.o1 = 1;
                            x.in.o2 = 4;
                            slots.push_back(x);
                        }
                    }
                    snseg.push_back((int32_t)slots.size() - sslot.back());
                }
                if ((int)slots.size() > g0) sgrp.push_back({hl, {g0, (int)slots.size() - g0}});
            }
            bfirst.push_back((int32_t)slots.size());
        }
    }
    const int nsf = (int)sf.size(), nsb = (int)slots.size(), nspb = bfirst.empty() ? 0 : (int)bfirst.size() - 1;
    int maxseg = 0;
    for (int32_t c : snseg) maxseg = std::max(maxseg, c);
    if (maxseg > SPEC_MAXSEG) return -1;  // (cannot happen: P keeps every frame within it)
    const size_t fb = a256(sizeof(FInfo) * nblk), bb = a256(sizeof(BInfo) * std::max(nbk, 1)),
                 lb = a256(sizeof(int32_t) * (2 * (size_t)nblk + (size_t)nbk + 16)), sb = a256(sizeof(uint64_t) * (size_t)std::max<int64_t>(seq_total, 1)),
                 yb = a256((size_t)std::max<int64_t>(byte_total, 1)), hb = a256(sizeof(uint32_t) * 1024 * (size_t)std::max(nbk, 1)),
                 tb = a256(sizeof(LitTab) * (size_t)std::max(nbk, 1));
    const size_t spb = nsb ? a256(sizeof(int32_t) * (3 * (size_t)nsf + nspb + 16)) + a256(sizeof(SpecB) * nsb) +
                                 2 * a256(sizeof(uint32_t) * SPEC_TSZ * (size_t)nsb) + a256(sizeof(int32_t) * (maxseg + 3))
                           : 0;
    if (!z.grow(fb + bb + lb + sb + yb + hb + tb + spb)) return -1;
    uint8_t *p = z.d;
    FInfo *d_fi = (FInfo *)p;
    p += fb;
    BInfo *d_bi = (BInfo *)p;
    p += bb;
    int32_t *d_list = (int32_t *)p;
    p += lb;
    uint64_t *d_seq = (uint64_t *)p;
    p += sb;
    uint8_t *d_bytes = p;
    p += yb;
    uint32_t *d_hist = (uint32_t *)p;
    p += hb;
    LitTab *d_lt = (LitTab *)p;
    p += tb;
    int32_t *d_slists = nullptr, *d_any = nullptr;
    SpecB *d_sp = nullptr;
    uint32_t *d_W = nullptr, *d_I = nullptr;
    if (nsb) {
        d_slists = (int32_t *)p;
        p += a256(sizeof(int32_t) * (3 * (size_t)nsf + nspb + 16));
        d_sp = (SpecB *)p;
        p += a256(sizeof(SpecB) * nsb);
        d_W = (uint32_t *)p;
        p += a256(sizeof(uint32_t) * SPEC_TSZ * (size_t)nsb);
        d_I = (uint32_t *)p;
        p += a256(sizeof(uint32_t) * SPEC_TSZ * (size_t)nsb);
        d_any = (int32_t *)p;
    }
    if (hipMemcpyAsync(d_fi, fi.data(), sizeof(FInfo) * nblk, hipMemcpyHostToDevice, stream) != hipSuccess) return -1;
    if (nbk > 0 && hipMemcpyAsync(d_bi, bi.data(), sizeof(BInfo) * nbk, hipMemcpyHostToDevice, stream) != hipSuccess)
        return -1;
    std::vector<int32_t> todo;
    for (int f = 0; f < nblk; f++)
        if (fi[f].status == 0) todo.push_back(f);
    // frames that cannot be encoded report -2 now; the others are written by zl1_litdec / zl1_litwrite
    for (int f = 0; f < nblk; f++)
        if (fi[f].status < 0) hret[f] = -2;
    if (hipMemcpyAsync(d_ret, hret.data(), sizeof(int32_t) * nblk, hipMemcpyHostToDevice, stream) != hipSuccess) return -1;
    std::vector<char> spec_f(nblk, 0);
    for (int f : sf) spec_f[f] = 1;
    for (int pass = 0; pass <= nbk + 1 && !todo.empty(); pass++) {
        // pass 0: the speculative block-parallel parse of the small batch's
        // multi-block frames (a frame whose confirmation guess turns out wrong
        // is parsed again frame-serially in the next pass)
        if (pass == 0 && nsb) {
            std::vector<int32_t> sl(sf);
            sl.insert(sl.end(), sslot.begin(), sslot.end());
            sl.insert(sl.end(), snseg.begin(), snseg.end());
            sl.insert(sl.end(), bfirst.begin(), bfirst.end());
            if (hipMemcpyAsync(d_slists, sl.data(), sizeof(int32_t) * sl.size(), hipMemcpyHostToDevice, stream) !=
                    hipSuccess ||
                hipMemcpyAsync(d_sp, slots.data(), sizeof(SpecB) * nsb, hipMemcpyHostToDevice, stream) != hipSuccess ||
                hipMemsetAsync(d_W, 0, sizeof(uint32_t) * SPEC_TSZ * (size_t)nsb, stream) != hipSuccess)
                return -1;
            const int32_t *d_sf = d_slists, *d_ss = d_slists + nsf, *d_sn = d_slists + 2 * nsf,
                          *d_bf = d_slists + 3 * nsf;
            bool settled = false;
            const int rmax = maxseg + 2;  // (segments + 1 rounds settle any frame)
            if (hipMemsetAsync(d_any, 0, sizeof(int32_t) * (rmax + 1), stream) != hipSuccess) return -1;
            for (int r = 0; r <= rmax; r++) {
                hipLaunchKernelGGL(zl1_spec_merge, dim3(nsf, SPEC_TSZ / 64), dim3(64), 0, stream, d_fi, d_sf, d_ss,
                                   d_sn, d_bi, d_W, d_I, d_sp, d_any, r);
                if (hipGetLastError() != hipSuccess) return -1;
                if (r > 0 && (r % 4 == 0 || r == rmax)) {  // a look every four rounds
                    int32_t h_any = 1;
                    if (hipMemcpyAsync(&h_any, d_any + r, sizeof(int32_t), hipMemcpyDeviceToHost, stream) != hipSuccess ||
                        hipStreamSynchronize(stream) != hipSuccess)
                        return -1;
                    if (!h_any) { settled = true; break; }
                }
                for (const auto &g : sgrp) {
                    const size_t tsz = (size_t)1 << g.first;
                    const int g0 = g.second.first, cnt = g.second.second;
                    hipLaunchKernelGGL(zl1_spec_parse<true>, dim3(cnt), dim3(64), tsz * 2 + tsz / 2, stream, d_fi,
                                       d_bi, d_seq, d_I + (size_t)g0 * SPEC_TSZ, d_W + (size_t)g0 * SPEC_TSZ, d_sp + g0,
                                       segsz);
                    if (hipGetLastError() != hipSuccess) return -1;
                }
            }
            if (!settled) return -1;  // (cannot happen: segments + 1 rounds settle any frame)
            hipLaunchKernelGGL(zl1_spec_compact, dim3(nspb), dim3(64), 0, stream, d_bf, d_bi, d_seq, (const SpecB *)d_sp);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        // parse launches: one per (table width, hashLog) so each gets exactly its LDS
        std::vector<int32_t> lists, blist;
        struct Grp { bool wide; uint32_t hlog; int off, cnt; };
        std::vector<Grp> grps;
        for (int wide = 0; wide < 2; wide++)
            for (uint32_t hl = 6; hl <= 15; hl++) {
                Grp g{wide != 0, hl, (int)lists.size(), 0};
                for (int f : todo) {
                    const bool w = fi[f].n >= 65536;
                    if (pass == 0 && spec_f[f]) continue;  // parsed above
                    if (w == (wide != 0) && fi[f].hlog == hl && fi[f].nb > 0) {
                        lists.push_back(f);
                        g.cnt++;
                    }
                }
                if (g.cnt) grps.push_back(g);
            }
        // Longest chain first: a launch lasts its longest frame's serial parse,
        // and workgroups start in index order (a 4 MiB frame queued behind
        // 1,000 small ones starts late), so each group lists its frames by
        // decreasing size and the groups launch largest frame first.
        for (const Grp &g : grps)
            std::stable_sort(lists.begin() + g.off, lists.begin() + g.off + g.cnt,
                             [&](int32_t a, int32_t b) { return fi[a].n > fi[b].n; });
        std::stable_sort(grps.begin(), grps.end(),
                         [&](const Grp &a, const Grp &b) { return fi[lists[a.off]].n > fi[lists[b.off]].n; });
        const int flist_off = (int)lists.size();
        for (int f : todo) lists.push_back(f);
        for (int f : todo)
            for (int k = 0; k < fi[f].nb; k++) blist.push_back(fi[f].b0 + k);
        const int blist_off = (int)lists.size();
        lists.insert(lists.end(), blist.begin(), blist.end());
        if ((size_t)lists.size() * sizeof(int32_t) > lb) {
            // (cannot happen: a pass lists each frame twice at most and each block once)
            return -1;
        }
        if (hipMemcpyAsync(d_list, lists.data(), sizeof(int32_t) * lists.size(), hipMemcpyHostToDevice, stream) !=
            hipSuccess)
            return -1;
        for (const Grp &g : grps) {
            const size_t tsz = (size_t)1 << g.hlog;
            if (g.wide) {
                hipLaunchKernelGGL(zl1_parse_kernel<true>, dim3(g.cnt), dim3(64), tsz * 2 + tsz / 2, stream, d_fi,
                                   d_list + g.off, d_bi, d_seq);
            } else {
                hipLaunchKernelGGL(zl1_parse_kernel<false>, dim3(g.cnt), dim3(64), tsz * 2, stream, d_fi,
                                   d_list + g.off, d_bi, d_seq);
            }
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (!blist.empty()) {
            hipLaunchKernelGGL(zl1_seq_kernel, dim3((unsigned)blist.size()), dim3(64), 0, stream, d_fi,
                               d_list + blist_off, d_bi, d_seq, d_bytes, d_hist);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (!blist.empty())
            hipLaunchKernelGGL(zl1_lithuf_kernel, dim3((unsigned)blist.size()), dim3(64), 0, stream, d_fi,
                               d_list + blist_off, d_bi, d_hist, d_lt);
        hipLaunchKernelGGL(zl1_litdec_kernel, dim3((unsigned)todo.size()), dim3(64), 0, stream, d_fi, d_list + flist_off,
                           d_bi, d_hist, d_lt, d_ret);
        if (!blist.empty())
            hipLaunchKernelGGL(zl1_litwrite_kernel, dim3((unsigned)blist.size()), dim3(64), 0, stream, d_fi,
                               d_list + blist_off, d_bi, d_bytes, d_lt);
        if (hipGetLastError() != hipSuccess) return -1;
        // frames whose confirmation guess was wrong go again
        std::vector<FInfo> chk(nblk);
        if (hipMemcpyAsync(chk.data(), d_fi, sizeof(FInfo) * nblk, hipMemcpyDeviceToHost, stream) != hipSuccess ||
            hipStreamSynchronize(stream) != hipSuccess)
            return -1;
        std::vector<int32_t> again;
        for (int f : todo)
            if (chk[f].status == 1) again.push_back(f);
        todo.swap(again);
    }
    if (!todo.empty()) return -1;
    return hipStreamSynchronize(stream) == hipSuccess ? 0 : -1;
}
