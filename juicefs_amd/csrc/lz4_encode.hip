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
// at once.  What keeps the serial parse off HBM latency:
//   * the bytes ahead of the parse position live in a 2 KiB LDS window that
//     slides in 1 KiB steps; the next step is prefetched into registers one
//     step early, so hashing and the parse-side compare read LDS only;
//   * every hash-table entry (byU32 table) carries check bits -- a hash of the
//     4 bytes at its position -- next to the position.  A candidate whose
//     check bits differ from those of the current 4 bytes cannot match, so the
//     HBM read of the candidate's bytes is made only when a match is likely.
//     The decision is still the exact 4-byte compare, so the parse (and every
//     output byte) is unchanged.
// Output is staged in an LDS ring and written to HBM with wide stores; nothing
// is written at or beyond dst_cap.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4e {

#ifdef JFS_PROF
// diagnostic build only: per-phase s_memtime sums of the encoder wave
__device__ unsigned long long g_eprof[12];
#define EP_DECL uint64_t ep_t = __builtin_amdgcn_s_memtime(), ep_acc[12] = {0};
#define EP(k) do { const uint64_t x_ = __builtin_amdgcn_s_memtime(); ep_acc[k] += x_ - ep_t; ep_t = x_; } while (0)
#define EPC(k) (ep_acc[k] += 1)
#define EP_FLUSH() do { if (lane_id() == 0) for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_eprof[i_], (unsigned long long)ep_acc[i_]); } while (0)
#else
#define EP_DECL
#define EP(k) do { } while (0)
#define EPC(k) do { } while (0)
#define EP_FLUSH() do { } while (0)
#endif
#ifndef JFS_LZ4E_PSEARCH
#define JFS_LZ4E_PSEARCH 1  // lane-parallel search over the skip schedule (serial loop on shared hashes)
#endif
constexpr int64_t kMaxInput = 0x7E000000;
constexpr int OB = 2048;  // output staging ring (the put_* paths assume OB >= 2 * OFLUSH + slack)
constexpr int OBMASK = OB - 1;
constexpr int OFLUSH = 1024;
constexpr int SW = 2048;  // source window (LDS), slides in SW/2 steps
constexpr int SWMASK = SW - 1;
constexpr int SWSTEP = SW / 2;  // = 64 lanes x 16 bytes

struct Smem {
    alignas(16) uint32_t table[4096];  // byU32 view; byU16 view is the same 16 KiB
    alignas(16) uint8_t ob[OB];
    alignas(16) uint8_t sw[SW];
};

struct Enc {
    const gc_u8 *src;
    g_u8 *dst;
    int64_t n, cap;
    int64_t op;  // output bytes produced
    int64_t F;   // flushed up to
    uint32_t dmis;
    // source window: covers "aligned offsets" q in [wq, wq + SW), q = p + smis
    // for source position p; pf = this lane's 16 bytes of [wq + SW, wq + SW + SWSTEP)
    const gc_u4 *sa;  // src rounded down to 16 bytes
    int64_t smis, wq, nq;
    uint4 pf;
    int pb;        // position bits of a byU32 table entry (check bits above)
    uint32_t pmask;
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

// ---- source window ---------------------------------------------------------
__device__ __forceinline__ uint4 sw_chunk(const Enc &e, int64_t q) {  // 16 bytes at aligned offset q
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < e.nq) v = e.sa[q >> 4];
    return v;
}
__device__ __forceinline__ void sw_put(Smem &s, int64_t q, const uint4 &v) {
    *(uint4 *)(s.sw + (uint32_t)(q & SWMASK)) = v;
}
// (re)fill the window to start at aligned offset wq (multiple of SWSTEP)
__device__ __forceinline__ void sw_fill(Smem &s, Enc &e, int64_t wq) {
    const int l = lane_id();
    const uint4 a = sw_chunk(e, wq + 16 * l), b = sw_chunk(e, wq + SWSTEP + 16 * l);
    e.pf = sw_chunk(e, wq + SW + 16 * l);
    sw_put(s, wq + 16 * l, a);
    sw_put(s, wq + SWSTEP + 16 * l, b);
    e.wq = wq;
    __builtin_amdgcn_wave_barrier();
}
// make source bytes [p, p + len) readable from the window (len <= 16)
__device__ __forceinline__ void sw_need(Smem &s, Enc &e, int64_t p, int len) {
    const int64_t q = p + e.smis;
    if (q + len <= e.wq + SW) return;
    if (q + len <= e.wq + SW + SWSTEP && q >= e.wq + SWSTEP) {
        // slide by one step: the prefetched chunk replaces the oldest half
        const int l = lane_id();
        sw_put(s, e.wq + SW + 16 * l, e.pf);
        e.wq += SWSTEP;
        e.pf = sw_chunk(e, e.wq + SW + 16 * l);
        __builtin_amdgcn_wave_barrier();
        return;
    }
    sw_fill(s, e, (q & ~(int64_t)(SWSTEP - 1)) - SWSTEP > 0 ? (q & ~(int64_t)(SWSTEP - 1)) - SWSTEP : 0);
}
__device__ __forceinline__ bool sw_has(const Enc &e, int64_t p, int len) {
    const int64_t q = p + e.smis;
    return q >= e.wq && q + len <= e.wq + SW;
}
__device__ __forceinline__ uint32_t sw_rd32(const Smem &s, const Enc &e, int64_t p) {
    const uint32_t q = (uint32_t)(p + e.smis);
    const uint32_t a = q & ~3u, sh = q & 3u;
    const uint32_t w0 = *(const uint32_t *)(s.sw + (a & SWMASK)), w1 = *(const uint32_t *)(s.sw + ((a + 4) & SWMASK));
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}
__device__ __forceinline__ uint64_t sw_rd64(const Smem &s, const Enc &e, int64_t p) {
    const uint32_t q = (uint32_t)(p + e.smis);
    const uint32_t a = q & ~3u, sh = q & 3u;
    const uint32_t w0 = *(const uint32_t *)(s.sw + (a & SWMASK)), w1 = *(const uint32_t *)(s.sw + ((a + 4) & SWMASK)),
                   w2 = *(const uint32_t *)(s.sw + ((a + 8) & SWMASK));
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}
// 8 bytes at p through the window (slides it forward as needed)
__device__ __forceinline__ uint64_t src64(Smem &s, Enc &e, int64_t p) {
    sw_need(s, e, p, 8);
    if (sw_has(e, p, 8)) return sw_rd64(s, e, p);
    const uint32_t lo = ld32u(e.src + p), hi = ld32u(e.src + p + 4);  // (window just reset below p)
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// 4 bytes at an arbitrary earlier position (window if present, else HBM)
__device__ __forceinline__ uint32_t src32(const Smem &s, const Enc &e, int64_t p) {
    if (sw_has(e, p, 4)) return sw_rd32(s, e, p);
    return ld32u(e.src + p);
}

__device__ __forceinline__ uint32_t hash_of(uint64_t v, bool u16) {
    if (u16) return ((uint32_t)v * 2654435761u) >> 19;
    return (uint32_t)(((v << 24) * 889523592379ull) >> 52);
}
// check bits of the 4 bytes v (independent of the table hash)
__device__ __forceinline__ uint32_t check_of(const Enc &e, uint32_t v) {
    return ((v * 0x9E3779B1u) >> e.pb) << e.pb;  // top (32 - pb) bits
}

__device__ __forceinline__ uint32_t tget(const Smem &s, uint32_t h, bool u16) {
    return u16 ? (uint32_t)((const uint16_t *)s.table)[h] : s.table[h];
}
// insert position pos whose first 4 bytes are v
__device__ __forceinline__ void tput(Smem &s, const Enc &e, uint32_t h, uint32_t pos, uint32_t v, bool u16) {
    if (u16) ((uint16_t *)s.table)[h] = (uint16_t)pos;
    else s.table[h] = pos | check_of(e, v);
}
// can the entry (found for 4 bytes v) be a match?  (byU16: always ask HBM)
__device__ __forceinline__ bool may_match(const Enc &e, uint32_t ent, uint32_t v, bool u16) {
    return u16 || (ent & ~e.pmask) == check_of(e, v);
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
__device__ __forceinline__ void put_lits(Smem &s, Enc &e, int64_t from, int64_t len, int64_t keep_from,
                                         int32_t pre = -1) {
    const int l = lane_id();
    for (int64_t k = 0; k < len; k += 64) {
        maybe_flush(s, e, keep_from);
        if (e.op + 64 + 16 - e.F > OB) {
            // token pending too far back: flush past it (the token is patched in
            // HBM); the 16 bytes of slack hold the offset bytes that follow the
            // run before the next flush, so the ring never wraps onto unflushed bytes
            int64_t to = ((e.op + e.dmis) & ~(int64_t)15) - e.dmis;
            oflush2(s, e, to);
        }
        int64_t i = k + l;
        if (i < len) s.ob[obidx(e, e.op + l)] = (k == 0 && pre >= 0) ? (uint8_t)pre : e.src[from + i];
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

// Residency: 20 KiB of LDS per block -> 8 blocks (waves) per CU.
__global__ __launch_bounds__(64) void lz4_encode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                       int32_t *__restrict__ ret) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    if (b >= nblk) return;
    const int l = lane_id();
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    EP_DECL
    Enc e;
    e.src = (const gc_u8 *)d.src;
    e.dst = (g_u8 *)d.dst;
    e.n = d.src_len;
    e.cap = d.dst_cap;
    e.op = 0;
    e.F = 0;
    e.dmis = (uint32_t)((uintptr_t)d.dst & 15u);
    e.sa = (const gc_u4 *)((uintptr_t)d.src & ~(uintptr_t)15);
    e.smis = (int64_t)((uintptr_t)d.src & 15u);
    e.nq = e.n + e.smis;
    e.wq = 0;
    e.pf = make_uint4(0, 0, 0, 0);
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
        // byU32 entries: position in the low pb bits, check bits above
        e.pb = 32 - __builtin_clz((uint32_t)n);
        if (e.pb < 16) e.pb = 16;
        e.pmask = e.pb >= 32 ? 0xFFFFFFFFu : ((1u << e.pb) - 1u);
        sw_fill(s, e, 0);
        // empty table: every entry is position 0 (LZ4's zeroed table), with its check bits
        const uint32_t init = u16 ? 0u : (n >= 4 ? check_of(e, sw_rd32(s, e, 0)) : 0u);
        for (int k = l; k < 4096; k += 64) s.table[k] = init;
        __builtin_amdgcn_wave_barrier();
        const int64_t mflimitP1 = n - 12 + 1, matchlimit = n - 5;
        int64_t ip = 0, anchor = 0;
        if (n >= 13) {
            uint64_t v0 = src64(s, e, 0);
            tput(s, e, hash_of(v0, u16), 0, (uint32_t)v0, u16);
            ip = 1;
            uint64_t fv = src64(s, e, ip);  // 8 bytes at the next search position
            uint32_t fh = hash_of(fv, u16);
            for (;;) {
                int64_t match;
                // ---- search (skip schedule: step = searchMatchNb++ >> 6)
                bool last = false;
                // bytes for the match's catch-up / literals / extension, loaded
                // together with the candidate checks for the first lane whose
                // check bits pass (nearly always the match): one round trip less
                bool pre_ok = false;
                int64_t pre_ip = -1, pre_m = -1;
                uint32_t p_ca = 0, p_cb = 1, p_xa = 0, p_xb = 1;
                int32_t p_lit = -1;
#if JFS_LZ4E_PSEARCH
                // Lane-parallel: lane j takes the j-th next position of the
                // schedule; every lane reads its table entry before any insert
                // of the batch, which is the serial order exactly when no two
                // positions of the batch share a hash (checked by a tagged
                // write + read-back).  The first lane whose candidate matches
                // ends the search; positions up to it are inserted, the others'
                // entries are restored.
                int32_t k0 = 0;  // schedule index of lane 0
                int64_t pk = ip;
                for (;;) {
                    const int32_t k = k0 + l;
                    const int32_t sk = k == 0 ? 1 : (63 + k) >> 6;
                    const uint32_t inc = dpp_scan_add((uint32_t)sk);
                    const int64_t P = pk + (int64_t)(inc - (uint32_t)sk), Pn = pk + (int64_t)inc;
                    const bool span = P - pk <= 512;
                    const uint64_t endm = __ballot(span && Pn > mflimitP1), spm = __ballot(span);
                    const int jend = endm ? (int)__builtin_ctzll(endm) : 64;
                    const int jspan = ~spm ? (int)__builtin_ctzll(~spm) : 64;
                    const int nl = jend < jspan ? jend : jspan;  // lanes [0, nl) are looked up
                    const bool on = l < nl;
                    if (nl > 0) sw_need(s, e, pk + (int64_t)readlane(inc - (uint32_t)sk, nl - 1), 8);
                    uint32_t cv = 0, h = 0, E = 0;
                    if (on) {
                        const uint64_t v = sw_rd64(s, e, P);
                        cv = (uint32_t)v;
                        h = hash_of(v, u16);
                        E = tget(s, h, u16);
                    }
                    EPC(7);
                    // shared hashes in the batch: tag write, read back.  A lane
                    // that reads another lane's tag shares its hash; the lowest
                    // lane m of any such pair has no predecessor in the batch, so
                    // lanes [0, m] are exact and the batch is cut after m.
                    const uint32_t tag = (uint32_t)l + 1u;
                    if (on) {
                        if (u16) ((uint16_t *)s.table)[h] = (uint16_t)tag;
                        else s.table[h] = tag;
                    }
                    __builtin_amdgcn_wave_barrier();
                    uint32_t cm = 64u;
                    if (on) {
                        const uint32_t t = tget(s, h, u16);
                        if (t != tag) cm = umin32((uint32_t)l, t - 1u);
                    }
                    const int ncut = (int)dwave_min(cm) + 1;  // 65: no shared hash
                    const int nb = ncut < nl ? ncut : nl;     // lanes [0, nb) are exact
                    if (on && l >= nb) {  // beyond the cut: pre-batch entries back (same hash, same entry)
                        if (u16) ((uint16_t *)s.table)[h] = (uint16_t)E;
                        else s.table[h] = E;
                    }
                    const int64_t cand = u16 ? (int64_t)E : (int64_t)(E & e.pmask);
                    bool pass = l < nb && (u16 || cand + 65535 >= P) && may_match(e, E, cv, u16);
                    const uint64_t pm0 = __ballot(pass);
                    if (pm0) {
                        EPC(9);
                        const int j0 = (int)__builtin_ctzll(pm0);
                        pre_ip = pk + (int64_t)readlane(inc - (uint32_t)sk, j0);
                        pre_m = (int64_t)readlane((uint32_t)cand, j0);
                        int64_t lim = pre_ip - anchor;
                        if (pre_m < lim) lim = pre_m;
                        const int64_t kk = 1 + l, ax = pre_ip + 4 + l, dlt = pre_ip - pre_m;
                        p_ca = 0; p_cb = 1; p_xa = 0; p_xb = 1; p_lit = -1;
                        if (kk <= lim) { p_ca = src[pre_ip - kk]; p_cb = src[pre_m - kk]; }
                        if (l < pre_ip - anchor) p_lit = src[anchor + l];
                        if (ax < matchlimit) { p_xa = src[ax]; p_xb = src[ax - dlt]; }
                        if (pass) pass = src32(s, e, cand) == cv;
                    }
                    const uint64_t hm = __ballot(pass);
                    const int jm = hm ? (int)__builtin_ctzll(hm) : 64;
                    if (l < nb) {
                        if (l <= jm) tput(s, e, h, (uint32_t)P, cv, u16);
                        else if (u16) ((uint16_t *)s.table)[h] = (uint16_t)E;
                        else s.table[h] = E;
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (hm) {
                        ip = pk + (int64_t)readlane(inc - (uint32_t)sk, jm);
                        match = (int64_t)readlane((uint32_t)cand, jm);
                        pre_ok = ip == pre_ip && match == pre_m;
                        break;
                    }
                    if (nb == nl && endm && jend <= jspan) { last = true; break; }  // the schedule passed mflimit
                    pk += (int64_t)readlane(inc, nb - 1);
                    k0 += nb;
                }
                if (false)
#endif
                {
                    int64_t fip = ip;
                    int32_t step = 1, snb = 1 << 6;
                    for (;;) {
                        const uint32_t h = fh;
                        const int64_t cur = fip;
                        const uint32_t cv = (uint32_t)fv;
                        const uint32_t ent = tget(s, h, u16);
                        ip = fip;
                        fip += step;
                        step = snb++ >> 6;
                        if (fip > mflimitP1) { last = true; break; }
                        match = u16 ? ent : (ent & e.pmask);
                        fv = src64(s, e, fip);
                        fh = hash_of(fv, u16);
                        tput(s, e, h, (uint32_t)cur, cv, u16);
                        EPC(7);
                        if (!u16 && match + 65535 < cur) continue;
                        if (!may_match(e, ent, cv, u16)) continue;
                        EP(0);
                        EPC(9);
                        const bool hit = src32(s, e, match) == cv;
                        EP(1);
                        if (hit) break;
                    }
                }
                EP(0);
                if (last) break;
                EPC(8);
                // One HBM round trip for the first 64 bytes of the three
                // byte-parallel phases: catch-up (before ip / match), literals
                // (from anchor) and the forward extension (from ip+4 / match+4;
                // it does not depend on the catch-up: the match end is absolute).
                int32_t lit_pre = -1;
                int64_t xend;   // ip-side end of the match (first differing byte or matchlimit)
                bool xmore;     // the first 64 extension bytes all matched
                {
                    int64_t lim = ip - anchor;
                    if (match < lim) lim = match;
                    const int64_t kk = 1 + l, ax = ip + 4 + l, dlt = ip - match;
                    uint32_t ca = p_ca, cb = p_cb, xa = p_xa, xb = p_xb;
                    lit_pre = p_lit;
                    if (!pre_ok) {
                        ca = 0; cb = 1; xa = 0; xb = 1; lit_pre = -1;
                        if (kk <= lim) { ca = src[ip - kk]; cb = src[match - kk]; }
                        if (l < ip - anchor) lit_pre = src[anchor + l];
                        if (ax < matchlimit) { xa = src[ax]; xb = src[ax - dlt]; }
                    }
                    const uint64_t xne = ~__ballot(ax < matchlimit && xa == xb);
                    const int xr = xne ? (int)__builtin_ctzll(xne) : 64;
                    xend = ip + 4 + xr;
                    xmore = xr == 64;
                    // ---- catch up (backwards, 64 bytes per step)
                    const uint64_t cne = ~__ballot(kk <= lim && ca == cb);
                    int64_t back = cne ? (int)__builtin_ctzll(cne) : 64;
                    bool cmore = back == 64;
                    while (cmore && back < lim) {
                        const int64_t k = back + 1 + l;
                        const bool eq = k <= lim && src[ip - k] == src[match - k];
                        const uint64_t ne = ~__ballot(eq);
                        const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        back += run;
                        cmore = run == 64;
                    }
                    if (back > lim) back = lim;
                    ip -= back;
                    match -= back;
                }
                EP(2);
                // ---- literals
                int64_t tp = e.op;
                uint32_t token;
                {
                    int64_t lit = ip - anchor;
                    e.op++;  // token slot
                    if (lit >= 15) { token = 15u << 4; put_len(s, e, (uint32_t)(lit - 15)); }
                    else token = (uint32_t)lit << 4;
                    put_lits(s, e, anchor, lit, tp, lit_pre);
                }
                EP(3);
                for (;;) {  // next_match
                    uint32_t off = (uint32_t)(ip - match);
                    put1(s, e, off & 255);
                    put1(s, e, off >> 8);
                    // match length: equal bytes from ip+4 / match+4 up to matchlimit
                    // (the first 64 were compared when the match was found)
                    while (xmore) {
                        const int64_t a = xend + l;
                        const bool eq = a < matchlimit && src[a] == src[a - (int64_t)off];
                        const uint64_t ne = ~__ballot(eq);
                        const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        xend += run;
                        xmore = run == 64;
                    }
                    const int64_t mc = xend - (ip + 4);
                    ip = xend;
                    if (mc >= 15) {
                        token += 15;
                        put_len(s, e, (uint32_t)(mc - 15));
                    } else {
                        token += (uint32_t)mc;
                    }
                    EP(4);
                    put_token(s, e, tp, token);
                    maybe_flush(s, e, INT64_MAX);
                    EP(5);
                    anchor = ip;
                    if (ip >= mflimitP1) break;
                    // bytes at ip - 2 and ip: one window check, both reads issued together
                    uint64_t v2, vi;
                    sw_need(s, e, ip + 2, 8);
                    if (sw_has(e, ip - 2, 12)) {
                        v2 = sw_rd64(s, e, ip - 2);
                        vi = sw_rd64(s, e, ip);
                    } else {
                        v2 = src64(s, e, ip - 2);
                        vi = src64(s, e, ip);
                    }
                    tput(s, e, hash_of(v2, u16), (uint32_t)(ip - 2), (uint32_t)v2, u16);
                    const uint32_t h = hash_of(vi, u16);
                    const uint32_t ent = tget(s, h, u16);
                    const uint32_t mi = u16 ? ent : (ent & e.pmask);
                    tput(s, e, h, (uint32_t)ip, (uint32_t)vi, u16);
                    bool rm = (u16 || (int64_t)mi + 65535 >= ip) && may_match(e, ent, (uint32_t)vi, u16);
                    if (rm) {  // the 4-byte check and the first 64 extension bytes in one round trip
                        const int64_t ax = ip + 4 + l, dlt = ip - (int64_t)mi;
                        uint32_t xa = 0, xb = 1;
                        if (ax < matchlimit) { xa = src[ax]; xb = src[ax - dlt]; }
                        rm = src32(s, e, mi) == (uint32_t)vi;
                        const uint64_t xne = ~__ballot(ax < matchlimit && xa == xb);
                        const int xr = xne ? (int)__builtin_ctzll(xne) : 64;
                        xend = ip + 4 + xr;
                        xmore = xr == 64;
                    }
                    EP(6);
                    if (rm) {
                        EPC(10);
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
                fv = src64(s, e, ip);
                fh = hash_of(fv, u16);
                EP(0);
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
    EP_FLUSH();
}

}  // namespace lz4e
}  // namespace jfs

extern "C" int jfs_launch_lz4_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4e::lz4_encode_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

#ifdef JFS_PROF
extern "C" int jfs_eprof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::lz4e::g_eprof), sizeof(unsigned long long) * 12) == hipSuccess ? 0 : -1;
}
extern "C" int jfs_eprof_reset() {
    unsigned long long z[12] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::lz4e::g_eprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
