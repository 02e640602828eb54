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
constexpr int64_t kMaxInput = 0x7E000000;
constexpr int64_t kSegMinInput = 65536 + 12 - 1;  // byU32 table (smaller blocks: byU16, serial kernel only)
// LDS of one block's wave.  Smem<false> (20 KiB, 8 blocks per CU): byU32
// entries = position + check bits (byU16 view: the same 16 KiB), 2 KiB output
// ring, 2 KiB source window.  Smem<true> ("compact", 10 KiB, 16 blocks per
// CU; byU32 blocks of the large-batch kernel only): 17-bit position entries
// (u16 + a bit plane, see ctab_*), no check bits, 512-byte output ring,
// 1 KiB source window.
template <bool C>
struct Smem {
    static constexpr bool kCompact = C;
    static constexpr int OB = C ? 512 : 2048;  // output staging ring (the put_* paths assume OB >= 2 * OFLUSH + slack)
    static constexpr int OBMASK = OB - 1;
    static constexpr int OFLUSH = C ? 128 : 1024;
    static constexpr int SW = C ? 1024 : 2048;  // source window (LDS), slides in SW/2 steps
    static constexpr int SWMASK = SW - 1;
    static constexpr int SWSTEP = SW / 2;       // = 64 lanes x PIECE bytes
    static constexpr int PIECE = SWSTEP / 64;
    static constexpr int SPAN = C ? 448 : 512;  // search batch reach (bytes past its first position)
    alignas(16) uint32_t table[C ? 2048 + 128 : 4096];
    alignas(16) uint8_t ob[OB];
    alignas(16) uint8_t sw[SW];
};
static_assert(sizeof(Smem<true>) == 10240, "compact layout: 16 blocks per CU");

struct Enc {
    const gc_u8 *src;
    g_u8 *dst;
    int64_t n, cap;
    int64_t op;  // output bytes produced
    int64_t F;   // flushed up to
    uint32_t dmis;
    // source window: covers "aligned offsets" q in [wq, wq + SW), q = p + smis
    // for source position p; pf = this lane's PIECE bytes of [wq + SW, wq + SW + SWSTEP)
    const gc_u4 *sa;  // src rounded down to 16 bytes
    int64_t smis, wq, nq;
    uint4 pf;
    int pb;        // position bits of a byU32 table entry (check bits above)
    uint32_t pmask;
    int64_t rlast;  // compact table: position of the last refresh (ctab_refresh)
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
template <class SM>
__device__ __forceinline__ uint4 sw_chunk(const Enc &e, int64_t q) {  // PIECE bytes at aligned offset q
    uint4 v = make_uint4(0, 0, 0, 0);
    if (q < e.nq) {
        if constexpr (SM::PIECE == 16) {
            v = e.sa[q >> 4];
        } else {
            const uint2 w = ((const gc_u2 *)e.sa)[q >> 3];
            v.x = w.x;
            v.y = w.y;
        }
    }
    return v;
}
template <class SM>
__device__ __forceinline__ void sw_put(SM &s, int64_t q, const uint4 &v) {
    if constexpr (SM::PIECE == 16) *(uint4 *)(s.sw + (uint32_t)(q & SM::SWMASK)) = v;
    else *(uint2 *)(s.sw + (uint32_t)(q & SM::SWMASK)) = make_uint2(v.x, v.y);
}
// (re)fill the window to start at aligned offset wq (multiple of SWSTEP)
template <class SM>
__device__ __forceinline__ void sw_fill(SM &s, Enc &e, int64_t wq) {
    const int l = lane_id();
    constexpr int P = SM::PIECE;
    const uint4 a = sw_chunk<SM>(e, wq + P * l), b = sw_chunk<SM>(e, wq + SM::SWSTEP + P * l);
    e.pf = sw_chunk<SM>(e, wq + SM::SW + P * l);
    sw_put(s, wq + P * l, a);
    sw_put(s, wq + SM::SWSTEP + P * l, b);
    e.wq = wq;
    __builtin_amdgcn_wave_barrier();
}
// make source bytes [p, p + len) readable from the window (len <= 16)
template <class SM>
__device__ __forceinline__ void sw_need(SM &s, Enc &e, int64_t p, int len) {
    const int64_t q = p + e.smis;
    if (q + len <= e.wq + SM::SW) return;
    if (q + len <= e.wq + SM::SW + SM::SWSTEP && q >= e.wq + SM::SWSTEP) {
        // slide by one step: the prefetched chunk replaces the oldest half
        const int l = lane_id();
        sw_put(s, e.wq + SM::SW + SM::PIECE * l, e.pf);
        e.wq += SM::SWSTEP;
        e.pf = sw_chunk<SM>(e, e.wq + SM::SW + SM::PIECE * l);
        __builtin_amdgcn_wave_barrier();
        return;
    }
    // refill: the step holding the last needed byte becomes the window's second half
    constexpr int64_t ST = SM::SWSTEP;
    const int64_t w = ((q + len - 1) & ~(ST - 1)) - ST;
    sw_fill(s, e, w > 0 ? w : 0);
}
template <class SM>
__device__ __forceinline__ bool sw_has(const Enc &e, int64_t p, int len) {
    const int64_t q = p + e.smis;
    return q >= e.wq && q + len <= e.wq + SM::SW;
}
template <class SM>
__device__ __forceinline__ uint32_t sw_rd32(const SM &s, const Enc &e, int64_t p) {
    const uint32_t q = (uint32_t)(p + e.smis);
    const uint32_t a = q & ~3u, sh = q & 3u;
    const uint32_t w0 = *(const uint32_t *)(s.sw + (a & SM::SWMASK)), w1 = *(const uint32_t *)(s.sw + ((a + 4) & SM::SWMASK));
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
}
template <class SM>
__device__ __forceinline__ uint64_t sw_rd64(const SM &s, const Enc &e, int64_t p) {
    const uint32_t q = (uint32_t)(p + e.smis);
    const uint32_t a = q & ~3u, sh = q & 3u;
    const uint32_t w0 = *(const uint32_t *)(s.sw + (a & SM::SWMASK)),
                   w1 = *(const uint32_t *)(s.sw + ((a + 4) & SM::SWMASK)),
                   w2 = *(const uint32_t *)(s.sw + ((a + 8) & SM::SWMASK));
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}
// 8 bytes at p through the window (slides it forward as needed)
template <class SM>
__device__ __forceinline__ uint64_t src64(SM &s, Enc &e, int64_t p) {
    sw_need(s, e, p, 8);
    if (sw_has<SM>(e, p, 8)) return sw_rd64(s, e, p);
    const uint32_t lo = ld32u(e.src + p), hi = ld32u(e.src + p + 4);  // (window just reset below p)
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
// 4 bytes at an arbitrary earlier position (window if present, else HBM)
template <class SM>
__device__ __forceinline__ uint32_t src32(const SM &s, const Enc &e, int64_t p) {
    if (sw_has<SM>(e, p, 4)) return sw_rd32(s, e, p);
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

// ---- hash table ------------------------------------------------------------
// Smem<false>: byU32 entries (position | check bits) or byU16 entries.
// Smem<true> (byU32 only): entry h = the low 17 bits of its position, 16 in
// lo[h] = ((u16 *)table)[h] and bit 16 in the plane hb = table + 2048 (bit h &
// 31 of hb[h >> 5]).  A lookup at P decodes it as the unique position == e
// (mod 2^17) in (P - 2^17, P]; that is the true position while every entry
// is at least P - 2^17 + 1, which ctab_refresh keeps (see there).  Raw values
// below: the 17-bit entry (compact), the u32 / u16 entry (otherwise).
template <class SM>
__device__ __forceinline__ uint32_t tget(const SM &s, uint32_t h, bool u16) {
    if constexpr (SM::kCompact)
        return (uint32_t)((const uint16_t *)s.table)[h] | (((s.table[2048 + (h >> 5)] >> (h & 31)) & 1u) << 16);
    return u16 ? (uint32_t)((const uint16_t *)s.table)[h] : s.table[h];
}
// insert position pos whose first 4 bytes are v
template <class SM>
__device__ __forceinline__ void tput(SM &s, const Enc &e, uint32_t h, uint32_t pos, uint32_t v, bool u16) {
    if constexpr (SM::kCompact) {
        ((uint16_t *)s.table)[h] = (uint16_t)pos;
        const uint32_t m = 1u << (h & 31);
        if (pos & 0x10000u)
            (void)__hip_atomic_fetch_or(&s.table[2048 + (h >> 5)], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else
            (void)__hip_atomic_fetch_and(&s.table[2048 + (h >> 5)], ~m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return;
    }
    if (u16) ((uint16_t *)s.table)[h] = (uint16_t)pos;
    else s.table[h] = pos | check_of(e, v);
}
// the search batch's temporary lane tags (a tag never outlives its batch:
// lanes restore or overwrite it), their read-back, and the restore of an
// entry read before the batch (compact: only the u16 half was tagged)
template <class SM>
__device__ __forceinline__ void ttag(SM &s, uint32_t h, uint32_t tag, bool u16) {
    if (SM::kCompact || u16) ((uint16_t *)s.table)[h] = (uint16_t)tag;
    else s.table[h] = tag;
}
template <class SM>
__device__ __forceinline__ uint32_t ttag_rd(const SM &s, uint32_t h, bool u16) {
    if (SM::kCompact || u16) return (uint32_t)((const uint16_t *)s.table)[h];
    return s.table[h];
}
template <class SM>
__device__ __forceinline__ void trestore(SM &s, uint32_t h, uint32_t E, bool u16) {
    if (SM::kCompact || u16) ((uint16_t *)s.table)[h] = (uint16_t)E;
    else s.table[h] = E;
}
// candidate position of raw entry E looked up at position P
template <class SM>
__device__ __forceinline__ int64_t tcand(const Enc &e, uint32_t E, int64_t P, bool u16) {
    if constexpr (SM::kCompact) return P - (int64_t)(((uint32_t)P - E) & 0x1FFFFu);
    return u16 ? (int64_t)E : (int64_t)(E & e.pmask);
}
// can the entry (found for 4 bytes v) be a match?  (byU16, compact: always ask HBM)
template <class SM>
__device__ __forceinline__ bool may_match(const Enc &e, uint32_t ent, uint32_t v, bool u16) {
    if constexpr (SM::kCompact) return true;
    return u16 || (ent & ~e.pmask) == check_of(e, v);
}
// Compact table upkeep, before any lookup or insert at pos (wave-uniform):
// once pos is 32 KiB past the last refresh R, every entry older than
// pos - 65535 (stale for LZ4's distance check at every later position) is
// rewritten as pos - 65536 (stale as well).  Between refreshes every entry is
// >= R - 65536 and every lookup / insert is below R + 32768 + SPAN + 8, so
// entries span less than 2^17 and decode exactly, here relative to
// R + 49152 and in the lookups relative to their own position.
template <class SM>
__device__ __forceinline__ void ctab_refresh(SM &s, Enc &e, int64_t pos) {
    if constexpr (SM::kCompact) {
        if (pos - e.rlast < 32768) return;
        const int l = lane_id();
        const uint32_t ref = (uint32_t)(e.rlast + 49152), sent = (uint32_t)(pos - 65536) & 0x1FFFFu;
        uint16_t *lo = (uint16_t *)s.table;
        uint32_t *hb = s.table + 2048;
        __builtin_amdgcn_wave_barrier();
        for (int k = 0; k < 64; ++k) {
            const uint32_t h = 64u * (uint32_t)k + (uint32_t)l;
            const uint32_t E = (uint32_t)lo[h] | (((hb[h >> 5] >> (h & 31)) & 1u) << 16);
            const int64_t t = (int64_t)ref - (int64_t)((ref - E) & 0x1FFFFu);
            const uint32_t ne = t + 65535 < pos ? sent : E;
            lo[h] = (uint16_t)ne;
            const uint64_t m = __ballot((ne >> 16) & 1u);
            if (l == 0) *(uint2 *)(hb + 2 * k) = make_uint2((uint32_t)m, (uint32_t)(m >> 32));
        }
        __builtin_amdgcn_wave_barrier();
        e.rlast = pos;
    }
}

// staging slot of output position x (mirrors HBM 16-byte alignment)
template <class SM>
__device__ __forceinline__ uint32_t obidx(const Enc &e, int64_t x) { return (uint32_t)((x + e.dmis) & SM::OBMASK); }

template <class SM>
__device__ __forceinline__ void oflush2(SM &s, Enc &e, int64_t to) {
    const int l = lane_id();
    if (to > e.cap) to = e.cap;
    int64_t F = e.F;
    if (to <= F) return;
    int64_t a = F + (int64_t)((16u - ((e.dmis + (uint32_t)F) & 15u)) & 15u);
    if (a > to) a = to;
    if (l < a - F) e.dst[F + l] = s.ob[obidx<SM>(e, F + l)];
    int64_t b = a + ((to - a) & ~(int64_t)15);
    for (int64_t x = a + 16 * l; x < b; x += 1024) *(g_u4 *)(e.dst + x) = *(const uint4 *)(s.ob + obidx<SM>(e, x));
    if (l < to - b) e.dst[b + l] = s.ob[obidx<SM>(e, b + l)];
    e.F = to;
}

template <class SM>
__device__ __forceinline__ void maybe_flush(SM &s, Enc &e, int64_t keep_from) {
    // flush everything below min(op, keep_from) once enough is pending
    int64_t lim = e.op < keep_from ? e.op : keep_from;
    if (lim - e.F >= SM::OFLUSH) {
        int64_t to = ((lim + e.dmis) & ~(int64_t)15) - e.dmis;
        oflush2(s, e, to);
    }
}

// one byte written by lane 0 (uniform position)
template <class SM>
__device__ __forceinline__ void put1(SM &s, Enc &e, uint32_t v) {
    if (lane_id() == 0) s.ob[obidx<SM>(e, e.op)] = (uint8_t)v;
    e.op++;
}

template <class SM>
__device__ __forceinline__ void put_len(SM &s, Enc &e, uint32_t len) {
    // 255-run then remainder; lanes write the run in parallel
    const int l = lane_id();
    uint32_t runs = len / 255;
    for (uint32_t k = 0; k < runs; k += 64) {
        if (e.op + 64 + 16 - e.F > SM::OB) oflush2(s, e, ((e.op + e.dmis) & ~(int64_t)15) - e.dmis);  // room for 64
        if (k + l < runs) s.ob[obidx<SM>(e, e.op + l)] = 255;
        e.op += (runs - k < 64 ? runs - k : 64);
        maybe_flush(s, e, INT64_MAX);
    }
    put1(s, e, len % 255);
}

// Copy source bytes [spos, spos + len) to output positions [dpos, ...) in HBM
// directly (nothing at or beyond cap): aligned 16-byte stores, the source
// read as dwords + v_alignbyte, four pieces per lane in flight (4 KiB per
// step).  For long literal runs (incompressible data), which through the LDS
// ring cost one dependent byte load per 64 bytes.
__device__ void copy_direct(Enc &e, int64_t dpos, int64_t spos, int64_t len) {
    const int l = lane_id();
    int64_t end = dpos + len;
    if (end > e.cap) end = e.cap;
    if (end <= dpos) return;
    const int64_t delta = spos - dpos;
    int64_t a = dpos + (int64_t)((16u - ((e.dmis + (uint32_t)dpos) & 15u)) & 15u);
    if (a > end) a = end;
    if (l < a - dpos) e.dst[dpos + l] = e.src[dpos + l + delta];
    int64_t lim = end;
    if (lim > e.n - 4 - delta) lim = e.n - 4 - delta;  // the dword reads stay inside the source
    const int64_t b = lim > a ? a + ((lim - a) & ~(int64_t)15) : a;
    for (int64_t x0 = a + 16 * l; x0 < b; x0 += 4096) {
        uint4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t x = x0 + 1024 * u;
            if (x < b) {
                const uintptr_t p = (uintptr_t)(e.src + x + delta);
                const gc_u32 *w = (const gc_u32 *)(p & ~(uintptr_t)3);
                const uint32_t sh = (uint32_t)(p & 3);
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
                v[u] = make_uint4(__builtin_amdgcn_alignbyte(w1, w0, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                                  __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh));
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t x = x0 + 1024 * u;
            if (x < b) *(g_u4 *)(e.dst + x) = v[u];
        }
    }
    for (int64_t x = b + l; x < end; x += 64) e.dst[x] = e.src[x + delta];
}

// copy literals src[from, from+len) into the output
template <class SM>
__device__ __forceinline__ void put_lits(SM &s, Enc &e, int64_t from, int64_t len, int64_t keep_from,
                                         int32_t pre = -1) {
    const int l = lane_id();
    if (len >= 2048) {  // long run: flush the ring (token and length bytes), copy HBM -> HBM
        oflush2(s, e, e.op);
        copy_direct(e, e.op, from, len);
        e.op += len;
        e.F = e.op < e.cap ? e.op : e.cap;
        return;
    }
    for (int64_t k = 0; k < len; k += 64) {
        maybe_flush(s, e, keep_from);
        if (e.op + 64 + 16 - e.F > SM::OB) {
            // token pending too far back: flush past it (the token is patched in
            // HBM); the 16 bytes of slack hold the offset bytes that follow the
            // run before the next flush, so the ring never wraps onto unflushed bytes
            int64_t to = ((e.op + e.dmis) & ~(int64_t)15) - e.dmis;
            oflush2(s, e, to);
        }
        int64_t i = k + l;
        if (i < len) s.ob[obidx<SM>(e, e.op + l)] = (k == 0 && pre >= 0) ? (uint8_t)pre : e.src[from + i];
        e.op += (len - k < 64 ? len - k : 64);
    }
}

// set the token byte at output position tp
template <class SM>
__device__ __forceinline__ void put_token(SM &s, Enc &e, int64_t tp, uint32_t v) {
    if (lane_id() == 0) {
        if (tp >= e.F) s.ob[obidx<SM>(e, tp)] = (uint8_t)v;
        else if (tp < e.cap) e.dst[tp] = (uint8_t)v;
    }
}

// Extend a match from xend (all bytes before it equal) by up to 4 KiB:
// lane l compares the 16-byte pieces at xend + 16 l + 1024 u (u < 4) with the
// bytes `off` earlier (source bytes: overlap is irrelevant), bytes at or past
// matchlimit count as different.  Advances xend to the first difference (or by
// 4 KiB); returns whether all 4 KiB were equal.
__device__ __forceinline__ bool extend_wide(const Enc &e, int64_t &xend, uint32_t off, int64_t matchlimit) {
    const int l = lane_id();
    uint32_t fd[4];
    uint32_t xw[4][4], yw[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t a = xend + 1024 * u + 16 * l;
        if (a + 16 <= matchlimit) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                xw[u][i] = ld32u(e.src + a + 4 * i);
                yw[u][i] = ld32u(e.src + a - (int64_t)off + 4 * i);
            }
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int64_t a = xend + 1024 * u + 16 * l;
        fd[u] = 16;
        if (a + 16 <= matchlimit) {
#pragma unroll
            for (int i = 3; i >= 0; --i) {
                const uint32_t d = xw[u][i] ^ yw[u][i];
                if (d) fd[u] = 4 * i + (__builtin_ctz(d) >> 3);
            }
        } else {
            fd[u] = 0;
            while (a + fd[u] < matchlimit && e.src[a + fd[u]] == e.src[a + fd[u] - (int64_t)off]) ++fd[u];
        }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const uint64_t ne = __ballot(fd[u] < 16);
        if (ne) {
            const int k = (int)__builtin_ctzll(ne);
            xend += 1024 * u + 16 * k + (int64_t)readlane(fd[u], k);
            return false;
        }
    }
    xend += 4096;
    return true;
}

// ---- segment mode (lz4_eseg) ----------------------------------------------
// A search state of the parse: the next search position P, the start of the
// pending literal run, the skip-schedule index of P (0 right after a match).
struct SegState {
    int64_t P, anchor;
    int32_t k0, end;  // end: the parse finished (last literals) before or in this segment
    int64_t pad;
};
// one sequence of the segment's output: literal count, match length - 4 (or
// kLastSeq: the block's last literals), offset
struct Seq {
    uint32_t lit, ml, off;
};
constexpr uint32_t kLastSeq = 0xFFFFFFFFu;
constexpr int kSegRoundsMax = 16;
// settled-round histogram of segment-mode blocks (index 0: unsettled -> serial kernel)
__device__ unsigned long long g_eseg[kSegRoundsMax + 1];
struct SegCtl {
    int round, nseg, nblk, cap;
    int64_t warm;  // round 1: segment k > 0 starts its parse this many bytes before its nominal start
    int32_t *seg_blk, *seg_k, *seq_n, *first, *nsegb, *fail, *todo, *diff;
    int64_t *seg_lo, *seg_hi, *anchor0, *seg_bytes, *map_off, *mlen;
    void *st;  // SegState [2][nseg]: round r writes half r & 1
    Seq *seq;  // [nseg][cap]
    uint8_t *map;  // per block two halves of mlen bytes: round r marks its insertions with r in half r & 1
};
// the round at which block b's segments reached their fixed point (0: not yet)
__device__ __forceinline__ int seg_conv(const SegCtl &c, int b, int upto) {
    if (c.fail[b]) return 0;
    if (c.nsegb[b] == 1) return 1;  // one segment starts at the true start: exact at once
    for (int r = 2; r <= upto; ++r)
        if (c.diff[r * c.nblk + b] == 0) return r;
    return 0;
}
// The hash table at search position P: for every hash, the latest position
// before P that the parse inserted (map byte == rv); only the last 65,535
// positions matter (older entries fail the distance check, like position 0).
__device__ void seg_table(Smem<false> &s, const Enc &e, const uint8_t *mapr, uint8_t rv, int64_t P) {
    const int l = lane_id();
    for (int k = l; k < 4096; k += 64) s.table[k] = 0;
    __builtin_amdgcn_wave_barrier();
    const int64_t w0 = P > 65535 ? P - 65535 : 0;
    for (int64_t q = (w0 & ~(int64_t)15) + 16 * l; q < P; q += 1024) {
        const uint4 m = *(const gc_u4 *)(mapr + q);
        const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t p = q + i;
            if (((mw[i >> 2] >> (8 * (i & 3))) & 255u) == rv && p >= w0 && p < P) {
                const uint64_t v = (uint64_t)ld32u(e.src + p) | ((uint64_t)ld32u(e.src + p + 4) << 32);
                atomicMax(&s.table[hash_of(v, false)], (uint32_t)p);
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    for (int k = l; k < 4096; k += 64) {
        const uint32_t pos = s.table[k];
        s.table[k] = pos | check_of(e, ld32u(e.src + pos));
    }
    __builtin_amdgcn_wave_barrier();
}

// Residency: 20 KiB of LDS per block -> 8 blocks (waves) per CU.
//
// SEG = false: one workgroup per block, the whole parse, output bytes.
// SEG = true: one workgroup per segment of a block (lz4_eseg below): the parse
// from the segment's start state up to the first search position at or past
// the segment's end, recording the positions it inserts (map) and its
// sequences instead of output bytes.
template <bool SEG, bool C>
__global__ __launch_bounds__(64) void lz4_encode_kernel_t(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                         int32_t *__restrict__ ret, const int32_t *__restrict__ todo,
                                                         SegCtl c, int only) {
    static_assert(!(SEG && C), "segment mode keeps the check-bit table");
    using SM = Smem<C>;
    __shared__ SM s;
    int b, j = 0;
    if constexpr (SEG) {
        j = blockIdx.x;
        if (j >= c.nseg) return;
        b = c.seg_blk[j];
        if (c.nsegb[b] == 0 || c.fail[b] || (c.round >= 2 && seg_conv(c, b, c.round - 1))) return;
    } else {
        b = blockIdx.x;
        if (b >= nblk) return;
        if (todo && !todo[b]) return;
    }
    const int l = lane_id();
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    if (only) {  // 1: the byU32 blocks only (the compact kernel's), 2: the others only
        const bool big = d.src_len >= kSegMinInput && d.src_len <= kMaxInput;
        if (big != (only == 1)) return;
    }
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
    e.rlast = 0;
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
        const uint32_t init = (u16 || C) ? 0u : (n >= 4 ? check_of(e, sw_rd32(s, e, 0)) : 0u);
        const int64_t mflimitP1 = n - 12 + 1, matchlimit = n - 5;
        int64_t ip = 0, anchor = 0;
        // segment mode: start state, insertion map, sequence list
        int32_t seg_k = 0, k0s = 0, ns = 0;
        int64_t seg_hi = INT64_MAX, hand_P = -1, hand_k0 = 0, anchor0 = 0;
        int64_t rec_lo = 0;  // positions below are warm-up: parsed, not marked
        bool from0 = true;   // the parse starts at the block start
        bool rec_seq = true; // sequences are kept (round 1 is a guess for segments k > 0)
        bool ovf = false;
        uint8_t *mapw = nullptr;
        Seq *sq = nullptr;
        const uint8_t rv = (uint8_t)c.round;
        if constexpr (SEG) {
            seg_k = c.seg_k[j];
            seg_hi = c.seg_hi[j];
            uint8_t *mb = c.map + c.map_off[b];
            mapw = mb + ((c.round & 1) ? c.mlen[b] : 0);
            sq = c.seq + (int64_t)j * c.cap;
            if (seg_k == 0) {
                ip = 1;
            } else if (c.round == 1) {
                // a guess: a fresh parse from `warm` bytes before the nominal
                // start (or from the block start), whose table and state at
                // the nominal start are then close to the serial parse's
                rec_lo = c.seg_lo[j];
                if (rec_lo - c.warm > 0) {
                    ip = anchor = rec_lo - c.warm;
                    from0 = false;
                }
            } else {
                from0 = false;
                const SegState st = ((const SegState *)c.st)[(int64_t)((c.round - 1) & 1) * c.nseg + j - 1];
                if (st.end) {
                    if (l == 0) {
                        SegState o = {0, 0, 0, 1, 0};
                        ((SegState *)c.st)[(int64_t)(c.round & 1) * c.nseg + j] = o;
                        c.seq_n[j] = 0;
                        c.anchor0[j] = 0;
                    }
                    return;
                }
                ip = st.P;
                anchor = st.anchor;
                k0s = st.k0;
            }
            anchor0 = anchor;
            rec_seq = c.round >= 2 || seg_k == 0;
            if (!from0 && c.round >= 2) {
                seg_table(s, e, mb + (((c.round - 1) & 1) ? c.mlen[b] : 0), (uint8_t)(c.round - 1), ip);
            } else {
                for (int k = l; k < 4096; k += 64) s.table[k] = init;
            }
        } else {
            for (int k = l; k < (int)(sizeof(s.table) / 4); k += 64) s.table[k] = init;
        }
        __builtin_amdgcn_wave_barrier();
        if (n >= 13) {
            if (from0) {
                uint64_t v0 = src64(s, e, 0);
                tput(s, e, hash_of(v0, u16), 0, (uint32_t)v0, u16);
                if (SEG && l == 0 && rec_lo == 0) mapw[0] = rv;
                ip = 1;
            }
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
                // Lane-parallel: lane j takes the j-th next position of the
                // schedule; every lane reads its table entry before any insert
                // of the batch, which is the serial order exactly when no two
                // positions of the batch share a hash (checked by a tagged
                // write + read-back).  The first lane whose candidate matches
                // ends the search; positions up to it are inserted, the others'
                // entries are restored.
                int32_t k0 = k0s;  // schedule index of lane 0
                k0s = 0;
                int64_t pk = ip;
                for (;;) {
                    if (SEG && pk >= seg_hi) {  // hand the search over to the next segment
                        hand_P = pk;
                        hand_k0 = k0;
                        break;
                    }
                    ctab_refresh(s, e, pk);
                    const int32_t k = k0 + l;
                    const int32_t sk = k == 0 ? 1 : (63 + k) >> 6;
                    const uint32_t inc = dpp_scan_add((uint32_t)sk);
                    const int64_t P = pk + (int64_t)(inc - (uint32_t)sk), Pn = pk + (int64_t)inc;
                    const bool span = P - pk <= SM::SPAN;
                    const uint64_t endm = __ballot(span && Pn > mflimitP1), spm = __ballot(span);
                    const int jend = endm ? (int)__builtin_ctzll(endm) : 64;
                    const int jspan = ~spm ? (int)__builtin_ctzll(~spm) : 64;
                    int nl = jend < jspan ? jend : jspan;  // lanes [0, nl) are looked up
                    int jstop = 64;
                    if constexpr (SEG) {  // positions at or past the segment end belong to the next segment
                        const uint64_t stm = __ballot(P >= seg_hi);
                        jstop = stm ? (int)__builtin_ctzll(stm) : 64;
                        if (jstop < nl) nl = jstop;
                    }
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
                    if (on) ttag(s, h, tag, u16);
                    __builtin_amdgcn_wave_barrier();
                    uint32_t cm = 64u;
                    if (on) {
                        const uint32_t t = ttag_rd(s, h, u16);
                        if (t != tag) cm = umin32((uint32_t)l, t - 1u);
                    }
                    const int ncut = (int)dwave_min(cm) + 1;  // 65: no shared hash
                    const int nb = ncut < nl ? ncut : nl;     // lanes [0, nb) are exact
                    if (on && l >= nb) trestore(s, h, E, u16);  // beyond the cut: pre-batch entries back (same hash, same entry)
                    const int64_t cand = tcand<SM>(e, E, P, u16);
                    bool pass = l < nb && (u16 || cand + 65535 >= P) && may_match<SM>(e, E, cv, u16);
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
                        if (l <= jm) {
                            tput(s, e, h, (uint32_t)P, cv, u16);
                            if (SEG && P >= rec_lo) mapw[P] = rv;
                        }
                        else trestore(s, h, E, u16);
                    }
                    __builtin_amdgcn_wave_barrier();
                    if (hm) {
                        ip = pk + (int64_t)readlane(inc - (uint32_t)sk, jm);
                        match = (int64_t)readlane((uint32_t)cand, jm);
                        pre_ok = ip == pre_ip && match == pre_m;
                        break;
                    }
                    if (nb == nl && endm && jend <= jspan && jend <= jstop) { last = true; break; }  // the schedule passed mflimit
                    pk += (int64_t)readlane(inc, nb - 1);
                    k0 += nb;
                }
                EP(0);
                if (last) break;
                if (SEG && hand_P >= 0) break;
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
                uint32_t token = 0;
                uint32_t seq_lit = (uint32_t)(ip - anchor);
                if constexpr (!SEG) {
                    int64_t lit = ip - anchor;
                    e.op++;  // token slot
                    if (lit >= 15) { token = 15u << 4; put_len(s, e, (uint32_t)(lit - 15)); }
                    else token = (uint32_t)lit << 4;
                    put_lits(s, e, anchor, lit, tp, lit_pre);
                }
                EP(3);
                for (;;) {  // next_match
                    uint32_t off = (uint32_t)(ip - match);
                    if constexpr (!SEG) {
                        put1(s, e, off & 255);
                        put1(s, e, off >> 8);
                    }
                    // match length: equal bytes from ip+4 / match+4 up to matchlimit
                    // (the first 64 were compared when the match was found)
                    // beyond the first 64 bytes (long matches: runs, zero pages):
                    // 4 KiB per step, 16-byte pieces per lane, loads issued together
                    while (xmore) xmore = extend_wide(e, xend, off, matchlimit);
                    const int64_t mc = xend - (ip + 4);
                    ip = xend;
                    if constexpr (SEG) {
                        if (rec_seq) {
                            if (ns >= c.cap) { ovf = true; break; }
                            if (l == 0) { Seq q = {seq_lit, (uint32_t)mc, off}; sq[ns] = q; }
                        }
                        ++ns;
                        seq_lit = 0;
                    } else {
                        if (mc >= 15) {
                            token += 15;
                            put_len(s, e, (uint32_t)(mc - 15));
                        } else {
                            token += (uint32_t)mc;
                        }
                        EP(4);
                        put_token(s, e, tp, token);
                        maybe_flush(s, e, INT64_MAX);
                    }
                    EP(5);
                    anchor = ip;
                    if (ip >= mflimitP1) break;
                    // bytes at ip - 2 and ip: one window check, both reads issued together
                    uint64_t v2, vi;
                    ctab_refresh(s, e, ip);
                    sw_need(s, e, ip + 2, 8);
                    if (sw_has<SM>(e, ip - 2, 12)) {
                        v2 = sw_rd64(s, e, ip - 2);
                        vi = sw_rd64(s, e, ip);
                    } else {
                        v2 = src64(s, e, ip - 2);
                        vi = src64(s, e, ip);
                    }
                    tput(s, e, hash_of(v2, u16), (uint32_t)(ip - 2), (uint32_t)v2, u16);
                    const uint32_t h = hash_of(vi, u16);
                    const uint32_t ent = tget(s, h, u16);
                    const int64_t mi = tcand<SM>(e, ent, ip, u16);
                    tput(s, e, h, (uint32_t)ip, (uint32_t)vi, u16);
                    if (SEG && l == 0) {
                        if (ip - 2 >= rec_lo) mapw[ip - 2] = rv;
                        if (ip >= rec_lo) mapw[ip] = rv;
                    }
                    bool rm = (u16 || mi + 65535 >= ip) && may_match<SM>(e, ent, (uint32_t)vi, u16);
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
                        if constexpr (!SEG) {
                            tp = e.op;
                            e.op++;
                        }
                        token = 0;
                        continue;
                    }
                    break;
                }
                if (SEG && ovf) break;
                if (anchor >= mflimitP1) break;
                ++ip;
                EP(0);
            }
        }
        if constexpr (SEG) {
            bool end = false;
            if (!ovf && hand_P < 0) {  // the parse reached the end: last literals
                if (rec_seq && ns >= c.cap) ovf = true;
                else {
                    if (l == 0 && rec_seq) { Seq q = {(uint32_t)(n - anchor), kLastSeq, 0}; sq[ns] = q; }
                    ++ns;
                    end = true;
                }
            }
            // no match in the whole first segment (incompressible data): the
            // skip schedule's state then runs through every segment and only
            // settles one segment per round -- the serial kernel is faster
            if (c.round == 1 && seg_k == 0 && ns == 0 && hand_P >= 0) ovf = true;
            if (l == 0) {
                if (ovf) c.fail[b] = 1;
                SegState o = {hand_P, anchor, (int32_t)hand_k0, (ovf || end) ? 1 : 0, 0};
                ((SegState *)c.st)[(int64_t)(c.round & 1) * c.nseg + j] = o;
                c.seq_n[j] = ns;
                c.anchor0[j] = anchor0;
            }
            return;
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

// ---- segment mode: plan, fixed-point check, output ---------------------------
//
// A lone block is one serial parse (~0.5 s for 4 MiB of text on one wave).
// Segment mode cuts each block at nominal boundaries k*L and parses all
// segments at once, in rounds.  Round 1 starts segment k > 0 with a fresh
// search at k*L and an empty table (a guess).  Round r starts segment k from
// the search state at which segment k-1 stopped in round r-1 (the first
// search position at or past k*L) and rebuilds the table from the positions
// round r-1 inserted in the 64 KiB before it.  When a round's stop states and
// insertion maps equal the previous round's, each segment's inputs are what
// the segment before produced, and by induction from segment 0 (always exact)
// every segment is the serial parse: the output is LZ4_compress_default's,
// byte for byte.  Blocks that do not settle within the round limit (or
// overflow a sequence list) are encoded by the serial kernel.

constexpr int kPlanThreads = 1024;
__global__ __launch_bounds__(kPlanThreads) void eseg_plan_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                                 int64_t L, SegCtl c) {
    __shared__ int64_t sa[kPlanThreads], sb[kPlanThreads];
    const int t = threadIdx.x;
    int64_t carry_s = 0, carry_m = 0;
    for (int base = 0; base < nblk; base += kPlanThreads) {
        const int b = base + t;
        const int64_t n = b < nblk ? (int64_t)((const gc_blk *)blocks)[b].src_len : 0;
        const int64_t ns = (b < nblk && n >= kSegMinInput && n <= kMaxInput) ? (n / L > 0 ? n / L : 1) : 0;
        const int64_t ml = ns ? ((n + 63) & ~(int64_t)63) : 0;
        sa[t] = ns;
        sb[t] = 2 * ml;
        __syncthreads();
        for (int d = 1; d < kPlanThreads; d <<= 1) {
            const int64_t xa = t >= d ? sa[t - d] : 0, xb = t >= d ? sb[t - d] : 0;
            __syncthreads();
            sa[t] += xa;
            sb[t] += xb;
            __syncthreads();
        }
        const int64_t first = carry_s + sa[t] - ns, moff = carry_m + sb[t] - 2 * ml;
        if (b < nblk) {
            c.first[b] = (int32_t)first;
            c.nsegb[b] = (int32_t)ns;
            c.map_off[b] = moff;
            c.mlen[b] = ml;
            c.todo[b] = ns == 0;
            for (int64_t k = 0; k < ns; ++k) {
                const int64_t jj = first + k;
                c.seg_blk[jj] = b;
                c.seg_k[jj] = (int32_t)k;
                c.seg_lo[jj] = k * L;
                c.seg_hi[jj] = k == ns - 1 ? n : (k + 1) * L;
            }
        }
        carry_s += sa[kPlanThreads - 1];
        carry_m += sb[kPlanThreads - 1];
        __syncthreads();
    }
}

// after round r: did any stop state or map byte of block b change?
constexpr int64_t kCmpChunk = 1 << 20;
__global__ __launch_bounds__(256) void eseg_cmp_kernel(SegCtl c) {
    const int b = blockIdx.y;
    if (c.nsegb[b] <= 1 || c.fail[b] || seg_conv(c, b, c.round - 1)) return;
    const int r = c.round;
    const uint8_t *mb = c.map + c.map_off[b];
    const uint8_t *A = mb + ((r & 1) ? c.mlen[b] : 0), *B = mb + (((r - 1) & 1) ? c.mlen[b] : 0);
    const uint32_t ra = (uint32_t)r * 0x01010101u, rb = (uint32_t)(r - 1) * 0x01010101u;
    bool d = false;
    const int64_t lo = (int64_t)blockIdx.x * kCmpChunk, hi = lo + kCmpChunk < c.mlen[b] ? lo + kCmpChunk : c.mlen[b];
    for (int64_t q = lo + 16 * threadIdx.x; q < hi; q += 16 * 256) {
        const uint4 x = *(const gc_u4 *)(A + q), y = *(const gc_u4 *)(B + q);
        const uint32_t xs[4] = {x.x, x.y, x.z, x.w}, ys[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t ex = xs[i] ^ ra, ey = ys[i] ^ rb;  // zero bytes: marked in that round
#pragma unroll
            for (int k = 0; k < 4; ++k) d |= (((ex >> (8 * k)) & 255u) == 0) != (((ey >> (8 * k)) & 255u) == 0);
        }
    }
    if (blockIdx.x == 0) {
        const SegState *sa = (const SegState *)c.st + (int64_t)(r & 1) * c.nseg;
        const SegState *sb = (const SegState *)c.st + (int64_t)((r - 1) & 1) * c.nseg;
        for (int k = threadIdx.x; k < c.nsegb[b]; k += 256) {
            const SegState x = sa[c.first[b] + k], y = sb[c.first[b] + k];
            d |= x.end != y.end || (!x.end && (x.P != y.P || x.anchor != y.anchor || x.k0 != y.k0));
        }
    }
    if (__syncthreads_or(d) && threadIdx.x == 0) atomicOr(&c.diff[r * c.nblk + b], 1);
}

__device__ __forceinline__ uint32_t len_bytes(uint32_t v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }
__device__ __forceinline__ uint32_t seq_bytes(const Seq &q) {
    uint32_t n = 1 + len_bytes(q.lit) + q.lit;
    if (q.ml != kLastSeq) n += 2 + len_bytes(q.ml);
    return n;
}

// output bytes of each settled segment; unsettled blocks go to the serial kernel
__global__ __launch_bounds__(64) void eseg_size_kernel(SegCtl c, int rounds) {
    const int j = blockIdx.x, l = lane_id();
    if (j >= c.nseg) return;
    const int b = c.seg_blk[j];
    if (c.nsegb[b] == 0) return;
    const int rc = seg_conv(c, b, rounds);
    if (rc == 0) {
        if (c.seg_k[j] == 0 && l == 0) {
            c.todo[b] = 1;
            atomicAdd(&g_eseg[0], 1ull);
        }
        return;
    }
    if (c.seg_k[j] == 0 && l == 0) atomicAdd(&g_eseg[rc], 1ull);
    const Seq *sq = c.seq + (int64_t)j * c.cap;
    uint32_t tot = 0;  // a block's output is below 2^31 (bound of n <= kMaxInput)
    for (int i = l; i < c.seq_n[j]; i += 64) tot += seq_bytes(sq[i]);
    tot = dwave_sum(tot);
    if (l == 0) c.seg_bytes[j] = (int64_t)tot;
}

// write each settled segment's sequences at its offset in the block's output
__global__ __launch_bounds__(64) void eseg_emit_kernel(const jfs_dev_block *__restrict__ blocks, int32_t *__restrict__ ret,
                                                       SegCtl c, int rounds) {
    __shared__ uint32_t lo_s[64], ls_s[64];
    __shared__ int64_t so_s[64], do_s[64];
    const int j = blockIdx.x, l = lane_id();
    if (j >= c.nseg) return;
    const int b = c.seg_blk[j];
    if (c.nsegb[b] == 0 || seg_conv(c, b, rounds) == 0) return;
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    const int k = c.seg_k[j], f = c.first[b], nsb = c.nsegb[b];
    uint32_t before = 0, total = 0;
    for (int i = l; i < nsb; i += 64) {
        const uint32_t v = (uint32_t)c.seg_bytes[f + i];
        total += v;
        if (i < k) before += v;
    }
    before = dwave_sum(before);
    total = dwave_sum(total);
    if (total > (uint64_t)d.dst_cap) {
        if (k == 0 && l == 0) ret[b] = 0;
        return;
    }
    if (k == 0 && l == 0) ret[b] = (int32_t)total;
    const gc_u8 *src = (const gc_u8 *)d.src;
    g_u8 *dst = (g_u8 *)d.dst;
    const Seq *sq = c.seq + (int64_t)j * c.cap;
    const int nsq = c.seq_n[j];
    int64_t op = (int64_t)before, sp = c.anchor0[j];
    for (int g = 0; g < nsq; g += 64) {
        const int i = g + l;
        Seq q = {0, kLastSeq, 0};
        if (i < nsq) q = sq[i];
        const uint32_t ob = i < nsq ? seq_bytes(q) : 0;
        const uint32_t sb_ = i < nsq ? q.lit + (q.ml == kLastSeq ? 0 : q.ml + 4) : 0;
        const uint32_t oinc = dpp_scan_add(ob), sinc = dpp_scan_add(sb_);
        const int64_t o = op + (int64_t)(oinc - ob), sx = sp + (int64_t)(sinc - sb_);
        // token and literal-length bytes
        const uint32_t lb = len_bytes(q.lit);
        const int64_t lo_out = o + 1 + lb;  // first literal byte
        if (i < nsq) {
            const uint32_t mlc = q.ml == kLastSeq ? 0 : (q.ml >= 15 ? 15 : q.ml);
            dst[o] = (uint8_t)(((q.lit >= 15 ? 15 : q.lit) << 4) | mlc);
            if (lb) {
                for (uint32_t t = 0; t + 1 < lb; ++t) dst[o + 1 + t] = 255;
                dst[o + lb] = (uint8_t)((q.lit - 15) % 255);
            }
            if (q.ml != kLastSeq) {
                const int64_t mo = lo_out + q.lit;
                dst[mo] = (uint8_t)(q.off & 255);
                dst[mo + 1] = (uint8_t)(q.off >> 8);
                const uint32_t mb = len_bytes(q.ml);
                if (mb) {
                    for (uint32_t t = 0; t + 1 < mb; ++t) dst[mo + 2 + t] = 255;
                    dst[mo + 1 + mb] = (uint8_t)((q.ml - 15) % 255);
                }
            }
        }
        // literals of the group: the wave copies them together, byte t of
        // the group's literal bytes found by a binary search over the prefix
        const uint32_t lit = i < nsq ? q.lit : 0;
        const uint32_t linc = dpp_scan_add(lit);
        lo_s[l] = linc - lit;
        ls_s[l] = lit;
        so_s[l] = sx;
        do_s[l] = lo_out;
        __builtin_amdgcn_wave_barrier();
        const uint32_t T = (uint32_t)readlane(linc, 63);
        for (uint32_t t0 = 0; t0 < T; t0 += 256) {
            uint8_t v[4];
            int64_t to[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const uint32_t t = t0 + (uint32_t)(u * 64 + l);
                to[u] = -1;
                if (t < T) {
                    int lo = 0, hi = 63;  // last lane whose literal run starts at or before t
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (lo_s[mid] <= t) lo = mid;
                        else hi = mid - 1;
                    }
                    const uint32_t r = t - lo_s[lo];
                    v[u] = src[so_s[lo] + r];
                    to[u] = do_s[lo] + r;
                }
            }
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (to[u] >= 0) dst[to[u]] = v[u];
        }
        __builtin_amdgcn_wave_barrier();
        op += (int64_t)readlane(oinc, 63);
        sp += (int64_t)readlane(sinc, 63);
    }
}

}  // namespace lz4e
}  // namespace jfs

using jfs::lz4e::SegCtl;

extern "C" int jfs_launch_lz4_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    if (nblk <= 0) return 0;
    // More blocks than the 20 KiB kernel holds at once (8 per CU): byU32
    // blocks (>= 64 KiB + 11) on the compact-table kernel (16 per CU), the
    // rest on the check-bit kernel, each grid skipping the other's blocks.
    // Smaller batches all take the check-bit kernel: resident either way, its
    // parse is 19 % faster (no HBM compare per candidate).
    static int ncu = [] {
        int dev = 0, v = 0;
        (void)hipGetDevice(&dev);
        return hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0 ? v : 256;
    }();
    const char *force = getenv("JFS_LZ4E_COMPACT");  // "1" / "0": always / never (tests, experiments)
    if (force ? force[0] == '0' : nblk <= 8 * ncu) {
        hipLaunchKernelGGL((jfs::lz4e::lz4_encode_kernel_t<false, false>), dim3(nblk), dim3(64), 0, stream, d_blocks,
                           nblk, d_ret, (const int32_t *)nullptr, SegCtl{}, 0);
        return hipGetLastError() == hipSuccess ? 0 : -1;
    }
    hipLaunchKernelGGL((jfs::lz4e::lz4_encode_kernel_t<false, true>), dim3(nblk), dim3(64), 0, stream, d_blocks, nblk,
                       d_ret, (const int32_t *)nullptr, SegCtl{}, 1);
    hipLaunchKernelGGL((jfs::lz4e::lz4_encode_kernel_t<false, false>), dim3(nblk), dim3(64), 0, stream, d_blocks, nblk,
                       d_ret, (const int32_t *)nullptr, SegCtl{}, 2);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

namespace {
int eseg_rounds() {
    static int v = [] {
        const char *e = getenv("JFS_LZ4E_SEG_ROUNDS");
        const int r = e ? atoi(e) : jfs::lz4e::kSegRoundsMax;
        return r < 2 ? 2 : (r > jfs::lz4e::kSegRoundsMax ? jfs::lz4e::kSegRoundsMax : r);
    }();
    return v;
}
int64_t eseg_warm() {
    static int64_t v = [] {
        const char *e = getenv("JFS_LZ4E_SEG_WARM_KB");
        return (int64_t)(e ? atoi(e) : 64) << 10;
    }();
    return v;
}
// Segment length: about 2,048 segments over the batch (8 waves per CU), at
// least 32 KiB (JFS_LZ4E_SEG_MIN_KB).  A difference between two rounds travels
// about one segment per round, and some persist for tens of KiB of input
// (hash-table entries live until overwritten), so shorter segments need more
// rounds (scripts/eseg_timing.py, 4 MiB text, round 6): 64 KiB settles in 4-6
// rounds (1 block 37.1 ms, 8 blocks 53.3), 32 KiB in 6-9 (34.7, 45.6), 16 KiB
// in 9-13 (30.9, 42.2) -- too close to the 16-round cap past which a block
// takes the serial parse.
int64_t eseg_len(int nblk, const int32_t *lens) {
    static int64_t lmin = [] {
        const char *e = getenv("JFS_LZ4E_SEG_MIN_KB");
        return (int64_t)(e ? atoi(e) : 32) << 10;
    }();
    int64_t tot = 0;
    for (int b = 0; b < nblk; ++b) tot += lens[b] > 0 ? lens[b] : 0;
    int64_t L = lmin;
    while (L * 2048 < tot) L <<= 1;
    return L;
}
struct EsegLayout {
    int64_t nseg, L, cap, o_int, o_i64, o_st, o_seq, o_map, total;
};
int64_t a16(int64_t x) { return (x + 15) & ~(int64_t)15; }
EsegLayout eseg_layout(int nblk, const int32_t *lens) {
    using namespace jfs::lz4e;
    EsegLayout y;
    y.L = eseg_len(nblk, lens);
    y.cap = y.L / 8 + 1024;  // sequences per segment (more: the block takes the serial kernel)
    y.nseg = 0;
    int64_t maps = 0;
    for (int b = 0; b < nblk; ++b) {
        const int64_t n = lens[b];
        if (n >= kSegMinInput && n <= kMaxInput) {
            y.nseg += n / y.L > 0 ? n / y.L : 1;
            maps += 2 * ((n + 63) & ~(int64_t)63);
        }
    }
    const int64_t S = y.nseg, B = nblk;
    y.o_int = 0;  // seg_blk, seg_k, seq_n [S]; first, nsegb, fail, todo [B]; diff [(R+1) B]
    y.o_i64 = a16(y.o_int + 4 * (3 * S + 4 * B + (kSegRoundsMax + 1) * B));
    y.o_st = a16(y.o_i64 + 8 * (4 * S + 2 * B));  // seg_lo, seg_hi, anchor0, seg_bytes [S]; map_off, mlen [B]
    y.o_seq = a16(y.o_st + (int64_t)sizeof(SegState) * 2 * S);
    y.o_map = (y.o_seq + (int64_t)sizeof(Seq) * y.cap * S + 63) & ~(int64_t)63;
    y.total = y.o_map + maps;
    return y;
}
}  // namespace

extern "C" int64_t jfs_lz4_eseg_scratch_bytes(int nblk, const int32_t *lens) {
    return nblk > 0 ? eseg_layout(nblk, lens).total : 0;
}

extern "C" int jfs_launch_lz4_encode_seg(const jfs_dev_block *d_blocks, int nblk, const int32_t *lens, int32_t *d_ret,
                                         void *scratch, int64_t scratch_cap, hipStream_t st) {
    using namespace jfs::lz4e;
    if (nblk <= 0) return 0;
    const EsegLayout y = eseg_layout(nblk, lens);
    if (y.total > scratch_cap) return -1;
    uint8_t *base = (uint8_t *)scratch;
    const int64_t S = y.nseg, B = nblk;
    SegCtl c{};
    c.nseg = (int)S;
    c.nblk = nblk;
    c.cap = (int)y.cap;
    c.warm = eseg_warm();
    int32_t *pi = (int32_t *)(base + y.o_int);
    c.seg_blk = pi;
    c.seg_k = pi + S;
    c.seq_n = pi + 2 * S;
    c.first = pi + 3 * S;
    c.nsegb = c.first + B;
    c.fail = c.nsegb + B;
    c.todo = c.fail + B;
    c.diff = c.todo + B;
    int64_t *pl = (int64_t *)(base + y.o_i64);
    c.seg_lo = pl;
    c.seg_hi = pl + S;
    c.anchor0 = pl + 2 * S;
    c.seg_bytes = pl + 3 * S;
    c.map_off = pl + 4 * S;
    c.mlen = c.map_off + B;
    c.st = base + y.o_st;
    c.seq = (Seq *)(base + y.o_seq);
    c.map = base + y.o_map;
    // counters, flags and stop states zeroed; the maps zeroed (no stale round marks)
    if (hipMemsetAsync(base, 0, (size_t)y.o_seq, st) != hipSuccess) return -1;
    if (y.total > y.o_map && hipMemsetAsync(base + y.o_map, 0, (size_t)(y.total - y.o_map), st) != hipSuccess) return -1;
    hipLaunchKernelGGL(eseg_plan_kernel, dim3(1), dim3(kPlanThreads), 0, st, d_blocks, nblk, y.L, c);
    const int R = eseg_rounds();
    int64_t maxml = 0;
    for (int b = 0; b < nblk; ++b) maxml = lens[b] > maxml ? lens[b] : maxml;
    const unsigned nchunk = (unsigned)((maxml + 63 + kCmpChunk - 1) / kCmpChunk);
    if (S > 0) {
        for (int r = 1; r <= R; ++r) {
            c.round = r;
            hipLaunchKernelGGL((lz4_encode_kernel_t<true, false>), dim3((unsigned)S), dim3(64), 0, st, d_blocks, nblk,
                               d_ret, (const int32_t *)nullptr, c, 0);
            if (r >= 2) hipLaunchKernelGGL(eseg_cmp_kernel, dim3(nchunk, (unsigned)B), dim3(256), 0, st, c);
        }
        hipLaunchKernelGGL(eseg_size_kernel, dim3((unsigned)S), dim3(64), 0, st, c, R);
        hipLaunchKernelGGL(eseg_emit_kernel, dim3((unsigned)S), dim3(64), 0, st, d_blocks, d_ret, c, R);
    }
    // blocks below the segment size, unsettled or overflowed: the serial parse
    hipLaunchKernelGGL((lz4_encode_kernel_t<false, false>), dim3(nblk), dim3(64), 0, st, d_blocks, nblk, d_ret,
                       (const int32_t *)c.todo, SegCtl{}, 0);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jfs_lz4_eseg_counts(uint64_t *out, int reset) {
    unsigned long long z[jfs::lz4e::kSegRoundsMax + 1] = {0};
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::lz4e::g_eseg), sizeof(z)) != hipSuccess) return -1;
    if (reset && hipMemcpyToSymbol(HIP_SYMBOL(jfs::lz4e::g_eseg), z, sizeof(z)) != hipSuccess) return -1;
    return 0;
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
