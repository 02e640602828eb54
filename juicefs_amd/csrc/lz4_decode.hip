// LZ4 block decoder for gfx950 -- one workgroup of two wavefronts per block.
//
// Replaces LZ4_decompress_safe reached from pkg/compress/compress.go:120-125
// (LZ4.Decompress -> lz4.DecompressSafe).  Result semantics (decoded size, or
// the same negative error value liblz4 1.9.3 returns) are restated in
// oracle/lz4_oracle.c; parity is tested in tests/test_lz4_gpu.py.
//
// Design:
//   The compressed stream is processed in windows of CW bytes staged in LDS,
//   double-buffered: the parser wave finds window k's token chain while the
//   copier wave produces window k-1's output (two barriers per window).
//   Parser: lane k owns the k-th P-byte piece; an exit table built backwards
//   over the piece (8 VGPRs) gives, for every entry offset, where the chain
//   leaves the piece; fix-up rounds propagate the true entry (exit of the
//   previous piece, DPP wave shift) until nothing changes; the chain
//   positions go to a u16 table in LDS.  Near the input end a speculative
//   walk with the exact end-of-input rules is used instead.
//   Copier: lane per token, 64 consecutive tokens per batch; DPP prefix sums
//   give output offsets and the liblz4 output-side checks; literal runs,
//   far matches (source older than the LDS output ring, read from HBM),
//   source substitution, then near matches in rounds (ready once no pending
//   destination overlaps the source).  Every ring write is an LDS atomic OR of
//   whole dwords into a zeroed span.  The ring streams to HBM in 128-byte
//   lines.  Tokens longer than LMAX are copied by the whole wave.
//   Everything the fast path does not cover (the last bytes of input /
//   output, malformed input, very long length fields) runs through an
//   exact, wave-uniform restatement of the liblz4 1.9.3 state machine.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4d {

// Tuning: every value below was measured against its alternatives (DESIGN.md
// 3, 6b-6d); the superseded variants live in the history, not in this file.
constexpr int P = 32;                  // window bytes per lane of the token table
constexpr int CW = 64 * P;             // compressed window bytes handled per pass
constexpr int CWIN = CW + 80;          // LDS staging incl. lookahead (multiple of 16)
constexpr int R = 4096;                // output ring bytes (power of two)
constexpr int RMASK = R - 1;
constexpr int SEG = 128;               // segment-walk parser: bytes per lane
constexpr int TMAX = CW / 3 + 2;       // max tokens in a window (interior token >= 3 bytes)
// Table capacity per window.  Windows with more tokens (only runs of 3..5-byte
// tokens) end at token TCAP and the next window starts there; the cap keeps the
// workgroup within 10 KiB of LDS so that 16 blocks (32 waves) fit on a CU.
constexpr int TCAP = 448 < TMAX ? 448 : TMAX;
// Diagnostic builds only (timing of phase knock-outs, WRONG output; never in
// the product .so): -DJFS_DIAG=<mask of D_*>.
#ifndef JFS_DIAG
#define JFS_DIAG 0
#endif
enum : unsigned {
    D_SKIP_ZERO = 1,    // no ring zeroing
    D_SKIP_LIT = 2,     // no literal copies
    D_SKIP_FAR = 4,     // no far-match copies
    D_SKIP_SUBST = 8,   // no source substitution
    D_SKIP_NEAR = 16,   // no near-match copies
    D_PARSEONLY = 32,   // the copier skips every window (the parser wave alone)
    D_NOCOPY = 64,      // parse and batching, no batch copies
};
constexpr unsigned DIAG = JFS_DIAG;
constexpr uint32_t STOP = 0x80000000u;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int KEXT = 64;               // max 255-extension bytes handled by the fast path
constexpr int FLUSH_T = 1024;          // flush the ring when this many bytes are pending
constexpr int LMAX = 64;               // longer literal runs / matches are copied by the whole wave
constexpr int BSPAN = 2048;            // max output span of one lane-parallel batch
static_assert(BSPAN + FLUSH_T + 128 <= R, "ring must hold the unflushed tail plus one batch");
static_assert(R - BSPAN >= LMAX + 16, "far sources must lie below the flushed prefix");

#ifdef JFS_PROF
// diagnostic build only: per-phase cycle sums (s_memtime), never in the product .so
#define NPROF 20  // 0..9 phase cycles, 10..19 event counts
__device__ uint64_t g_prof[NPROF];
struct Prof {
    uint64_t t, acc[NPROF];
    __device__ void start() {
        t = __builtin_amdgcn_s_memtime();
        for (int i = 0; i < NPROF; i++) acc[i] = 0;
    }
    __device__ void stamp(int k) {
        uint64_t x = __builtin_amdgcn_s_memtime();
        acc[k] += x - t;
        t = x;
    }
    __device__ void flush_out() {
        if (__lane_id() == 0)
            for (int i = 0; i < NPROF; i++) atomicAdd((unsigned long long *)&g_prof[i], acc[i]);
    }
};
#define PSTAMP(k) pr.stamp(k)
#define PCOUNT(k, n) (pr.acc[k] += (n))
#define PROF_ARG , Prof &pr
#define PROF_PASS , pr
#else
#define PSTAMP(k)
#define PCOUNT(k, n)
#define PROF_ARG
#define PROF_PASS
#endif

// Published by the parser wave for each window it stages (double-buffered).
enum { W_NONE = 0, W_WIN = 1, W_SER = 2, W_BUG = 3 };
struct Meta {
    int32_t kind, wbase, cbase;
    uint32_t T, efin;
};
// Published by the copier wave after each pipeline step.
struct Ctl {
    int32_t done, restart, rip;
    int32_t step;  // the copier's pipeline step, written as it reaches the step's first barrier
};

struct Smem {
    alignas(16) uint8_t ring[R];
    alignas(16) uint8_t cwin[2][CWIN];
    alignas(16) uint16_t tab[2][TCAP];  // token positions relative to cbase, stream order
    Meta meta[2];
    Ctl ctl;
};

struct Ctx {
    const gc_u8 *src;
    g_u8 *dst;
    int32_t n;      // compressed size
    int32_t cap;    // dst capacity
    int32_t F;      // ring flushed up to (output position)
    int32_t Fw;     // flushed and waited for (HBM loads below this are safe)
    uint32_t dmis;  // dst address mod 16 (ring slots mirror HBM alignment)
    int32_t cbase;  // input position of cw[0]
    int32_t bug;    // set when an internal bound trips (kernel bug guard; never expected)
    uint8_t *cw;    // staged window (one of Smem::cwin)
    uint32_t cwoff; // its byte offset in Smem (LDS address of cw[0])
    uint16_t *tab;  // its token table
};

// dword vectors that are only 4-byte aligned (global_load_dwordx4 / x2 at any dword address)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2), aligned(4)));
typedef JFS_GLOBAL const u32x4 gc_x4;
typedef JFS_GLOBAL const u32x2 gc_x2;

__device__ __forceinline__ uint32_t slot(const Ctx &c, int32_t pos) { return (uint32_t)(pos + (int32_t)c.dmis) & RMASK; }

// Far-match source bytes: the 6 dwords from the dword holding HBM address a.
// A dword that lies wholly below dst's first dword holds no source byte (only
// bytes the write mask drops) and is not read: it reads as 0.
__device__ __forceinline__ void far_load(const Ctx &c, uintptr_t a, uint32_t &d0, uint32_t &d1, uint32_t &d2,
                                         uint32_t &d3, uint32_t &d4, uint32_t &d5) {
    const uintptr_t b = a & ~(uintptr_t)3, lo = (uintptr_t)c.dst & ~(uintptr_t)3;
    const bool under = b < lo;
    const gc_x4 *q = (const gc_x4 *)(under ? lo : b);
    const u32x4 v = q[0];
    const u32x2 w = *(const gc_x2 *)(q + 1);
    d0 = v.x; d1 = v.y; d2 = v.z; d3 = v.w; d4 = w.x; d5 = w.y;
    if (__ballot(under)) {
        if (under) { d5 = d4; d4 = d3; d3 = d2; d2 = d1; d1 = d0; d0 = 0; }
    }
}

// ---------------------------------------------------------------------------
// staging and byte access
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cb(const Smem &s, const Ctx &c, int32_t p) {
    int32_t r = p - c.cbase;
    if ((uint32_t)r < (uint32_t)CWIN) return c.cw[r];
    return (p >= 0 && p < c.n) ? c.src[p] : 0u;
}

// Stage input [cbase, cbase+CWIN) with 16-byte loads aligned in HBM.
__device__ __forceinline__ void stage_window(Smem &s, Ctx &c, int32_t wbase) {
    const int l = lane_id();
    const uint32_t mis = (uint32_t)(((uintptr_t)c.src + (uint32_t)wbase) & 15u);
    c.cbase = wbase - (int32_t)mis;
    // all loads first, then the LDS writes: one HBM latency per window, not three
    constexpr int NCH = (CWIN / 16 + 63) / 64;
    uint4 v[NCH];
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
        const int k = l + 64 * j;
        const int32_t p = c.cbase + 16 * k;
        v[j] = make_uint4(0, 0, 0, 0);
        if (k < CWIN / 16 && p < c.n) v[j] = *(const gc_u4 *)(c.src + p);  // chunk holds a valid byte: same page
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
        const int k = l + 64 * j;
        if (k < CWIN / 16) *(uint4 *)(c.cw + 16 * k) = v[j];
    }
    // bytes outside [0, n) must read as 0 (they are never part of a fast-path token)
    if (c.cbase < 0 || c.cbase + CWIN > c.n) {
        for (int k = l; k < CWIN; k += 64) {
            int32_t p = c.cbase + k;
            if (p >= c.n || p < 0) c.cw[k] = 0;
        }
    }
}

// ---------------------------------------------------------------------------
// fast-path token parse (LZ4_decompress_generic fast loop, input-side checks)
// ---------------------------------------------------------------------------
struct Tok {
    int32_t nxt;   // next token position, or STOP|p
    int32_t ll;    // literal length
    int32_t ml;    // match length (incl. MINMATCH)
    int32_t off;   // match offset
    int32_t lit;   // literal source position
    int32_t llx;   // literal length used the 255-extension (RUN_MASK)
};

__device__ __forceinline__ Tok parse_tok(const Smem &s, const Ctx &c, int32_t p) {
    Tok t;
    const int32_t n = c.n;
    t.ll = t.ml = t.off = t.lit = t.llx = 0;
    if (p > n - 18) { t.nxt = (int32_t)(STOP | (uint32_t)p); return t; }
    uint32_t tb = cb(s, c, p);
    int32_t q = p + 1;
    int32_t ll = (int32_t)(tb >> 4);
    if (ll == 15) {
        t.llx = 1;
        int k = 0;
        uint32_t sv;
        do {
            sv = cb(s, c, q);
            q++;
            ll += (int32_t)sv;
            if (q >= n - 15 || ++k > KEXT) { t.nxt = (int32_t)(STOP | (uint32_t)p); return t; }
        } while (sv == 255);
        if (q + ll > n - 32) { t.nxt = (int32_t)(STOP | (uint32_t)p); return t; }
    }
    t.lit = q;
    t.ll = ll;
    q += ll;
    t.off = (int32_t)(cb(s, c, q) | (cb(s, c, q + 1) << 8));
    q += 2;
    int32_t ml = (int32_t)(tb & 15);
    if (ml == 15) {
        int k = 0;
        uint32_t sv;
        do {
            sv = cb(s, c, q);
            q++;
            ml += (int32_t)sv;
            if (q >= n - 4 || ++k > KEXT) { t.nxt = (int32_t)(STOP | (uint32_t)p); return t; }
        } while (sv == 255);
    }
    t.ml = ml + 4;
    t.nxt = q;
    return t;
}

// The same parse from the staged window only, without branches or HBM reads:
// reads are clamped to the window, and `slow` marks tokens that need bytes
// beyond it or a second 255-extension byte (those go through parse_tok).
struct FTok {
    int32_t nxt, lit;
    uint32_t ll, ml, off, llx;
    bool slow, stop;
};

__device__ __forceinline__ uint32_t w8(const Ctx &c, int32_t r) { return c.cw[r < CWIN - 1 ? r : CWIN - 1]; }

__device__ __forceinline__ FTok parse_fast(const Smem &s, const Ctx &c, int32_t p) {
    FTok t;
    const int32_t n = c.n, b0 = c.cbase;
    const int32_t r = p - b0;
    const uint32_t tb = w8(c, r), e1 = w8(c, r + 1);
    const bool llx = (tb >> 4) == 15;
    int32_t q = r + 1 + (llx ? 1 : 0);
    t.ll = (tb >> 4) + (llx ? e1 : 0u);
    bool slow = llx && e1 == 255;
    bool stop = p > n - 18;
    stop |= llx && (b0 + q >= n - 15 || b0 + q + (int32_t)t.ll > n - 32);
    t.lit = b0 + q;
    q += (int32_t)t.ll;
    slow |= q + 3 > CWIN;  // offset and the first match-length extension byte must be staged
    const uint32_t o0 = w8(c, q), o1 = w8(c, q + 1), e2 = w8(c, q + 2);
    q += 2;
    const bool mlx = (tb & 15) == 15;
    t.ml = (tb & 15) + (mlx ? e2 : 0u) + 4;
    q += mlx ? 1 : 0;
    slow |= mlx && e2 == 255;
    stop |= mlx && b0 + q >= n - 4;
    t.off = o0 | (o1 << 8);
    t.llx = llx ? 1u : 0u;
    t.nxt = b0 + q;
    t.slow = slow;
    t.stop = stop;
    return t;
}

// ---------------------------------------------------------------------------
// output ring <-> HBM
// ---------------------------------------------------------------------------
// Write ring[F, to) to dst[F, to).  `to` is a 128-byte aligned HBM boundary
// (or the block end).  The stores are not waited for here: Fw (the prefix
// whose stores are known complete) only advances where an HBM read of the
// output needs it (far matches, need_flushed), so the copier does not stall
// on every flush.
__device__ __forceinline__ void flush(Smem &s, Ctx &c, int32_t to) {
    const int l = lane_id();
    int32_t F = c.F;
    if (to <= F) return;
    int32_t a = F + (int32_t)((16u - ((c.dmis + (uint32_t)F) & 15u)) & 15u);
    if (a > to) a = to;
    if (l < a - F) c.dst[F + l] = s.ring[slot(c, F + l)];
    int32_t b = a + ((to - a) & ~15);
    for (int32_t x = a + 16 * l; x < b; x += 1024) {
        uint4 v = *(const uint4 *)(s.ring + slot(c, x));
        *(g_u4 *)(c.dst + x) = v;
    }
    if (l < to - b) c.dst[b + l] = s.ring[slot(c, b + l)];
    c.F = to;
}

__device__ __forceinline__ void flush_to_line(Smem &s, Ctx &c, int32_t hi) {
    int32_t to = (int32_t)(((uint32_t)hi + c.dmis) & ~127u) - (int32_t)c.dmis;
    if (to > c.F) flush(s, c, to);
}

__device__ __forceinline__ uint32_t out_byte(const Smem &s, const Ctx &c, int32_t x, int32_t ringfloor) {
    if (x >= ringfloor) return s.ring[slot(c, x)];
    return c.dst[x];
}

__device__ __forceinline__ void need_flushed(Ctx &c, int32_t lim) {
    if (lim > c.Fw) {
        wait_vm();
        c.Fw = c.F;
    }
}

// ---------------------------------------------------------------------------
// whole-wave copies (serial path and long tokens)
// ---------------------------------------------------------------------------
// Long literal runs (incompressible data: a 4 MiB block is one run) go HBM to
// HBM: the ring is flushed up to op, the run except its last R bytes is
// copied with 16-byte stores (1 KiB per wave step, 4 steps in flight), and
// the last R bytes go through the ring as usual, so every later source inside
// the ring's reach finds its bytes there and older ones are read from HBM
// (F advanced; far reads wait for these stores through Fw).
constexpr int32_t LIT_DIRECT = 2 * R;
__device__ __forceinline__ void direct_lit(Smem &s, Ctx &c, int32_t srcpos, int32_t op, int32_t body) {
    const int l = lane_id();
    flush(s, c, op);
    const gc_u8 *sp = c.src + srcpos - op;  // sp[x] = source byte of output x
    int32_t x = op;
    const int32_t ha = (int32_t)((16u - (((uint32_t)(uintptr_t)(c.dst + x)) & 15u)) & 15u);
    if (l < ha) c.dst[x + l] = sp[x + l];
    x += ha;
    for (; x + 4096 <= body; x += 4096) {
        u32x4 v[4];
        uint32_t w[4];
        const uint32_t sh = (uint32_t)((uintptr_t)(sp + x) & 3u);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uintptr_t a = (uintptr_t)(sp + x + 1024 * j + 16 * l) & ~(uintptr_t)3;
            v[j] = *(const gc_x4 *)a;
            w[j] = *(const gc_u32 *)(a + 16);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            uint4 o;
            o.x = __builtin_amdgcn_alignbyte(v[j].y, v[j].x, sh);
            o.y = __builtin_amdgcn_alignbyte(v[j].z, v[j].y, sh);
            o.z = __builtin_amdgcn_alignbyte(v[j].w, v[j].z, sh);
            o.w = __builtin_amdgcn_alignbyte(w[j], v[j].w, sh);
            *(g_u4 *)(c.dst + x + 1024 * j + 16 * l) = o;
        }
    }
    for (; x < body; x += 64)
        if (x + l < body) c.dst[x + l] = sp[x + l];
    c.F = body;
}

__device__ __forceinline__ void coop_lit(Smem &s, Ctx &c, int32_t srcpos, int32_t op, int32_t len) {
    const int l = lane_id();
    if (len >= LIT_DIRECT) {
        const int32_t body = op + len - R;
        direct_lit(s, c, srcpos, op, body);
        srcpos += body - op;
        len -= body - op;
        op = body;
    }
    for (int32_t k = 0; k < len; k += 64) {
        if (op + k - c.F >= FLUSH_T) flush_to_line(s, c, op + k);
        int32_t i = k + l;
        if (i < len) s.ring[slot(c, op + i)] = cb(s, c, srcpos + i);
    }
}

// Long matches whose offset divides 16 (runs of one byte or of a 2/4/8/16-byte
// pattern: zero-filled regions) are pure stores: every 16-byte-aligned chunk
// of the run holds the same 16 bytes.  The run except its last R bytes is
// written straight to HBM (4 KiB per wave step), the 16 bytes before the tail
// are put in the ring (the tail's period source) and the tail goes through
// the ring as usual.  Returns the output position where the ring part starts.
__device__ __forceinline__ int32_t direct_fill(Smem &s, Ctx &c, int32_t op, int32_t off, int32_t len) {
    const int l = lane_id();
    const int32_t body = op + len - R;
    flush(s, c, op);
    const uint32_t amis = (uint32_t)(uintptr_t)(c.dst + op) & 15u;
    const int32_t x0 = op + (int32_t)((16u - amis) & 15u);  // first 16-byte aligned output position
    // byte b of every aligned chunk = P[(x0 - op + b) mod off], P = the off bytes before op (in the ring)
    uint32_t q[4] = {0, 0, 0, 0};
#pragma unroll
    for (int b = 0; b < 16; ++b) {
        const uint32_t v = s.ring[slot(c, op - off + (int32_t)(((uint32_t)(x0 - op) + (uint32_t)b) % (uint32_t)off))];
        q[b >> 2] |= v << (8 * (b & 3));
    }
    const uint4 chunk = make_uint4(q[0], q[1], q[2], q[3]);
    if (op + l < x0) c.dst[op + l] = s.ring[slot(c, op - off + (l % off))];  // head (< 16 bytes)
    int32_t x = x0;
    for (; x + 4096 <= body; x += 4096) {
#pragma unroll
        for (int j = 0; j < 4; ++j) *(g_u4 *)(c.dst + x + 1024 * j + 16 * l) = chunk;
    }
    for (; x + 16 <= body; x += 1024)
        if (x + 16 * l + 16 <= body) *(g_u4 *)(c.dst + x + 16 * l) = chunk;
    const int32_t xe = x0 + ((body - x0) & ~15);  // end of the aligned chunks written
    if (xe + l < body) c.dst[xe + l] = (uint8_t)(q[l >> 2 & 3] >> (8 * (l & 3)));  // (< 16 bytes, same phase)
    // the ring gets the 16 bytes before `body` (the tail's source period)
    if (l < 16) {
        const int32_t y = body - 16 + l;
        s.ring[slot(c, y)] = s.ring[slot(c, op - off + (int32_t)((uint32_t)(y - op) % (uint32_t)off))];
    }
    c.F = body;
    return body;
}

__device__ __forceinline__ void coop_match(Smem &s, Ctx &c, int32_t op, int32_t off, int32_t len) {
    const int l = lane_id();
    if (len >= LIT_DIRECT && off > 0 && off <= 16 && (16 % off) == 0) {
        const int32_t b = direct_fill(s, c, op, off, len);
        len -= b - op;
        op = b;
    }
    int32_t m = 0, step = 0;
    if (off > 0 && off < 64) { m = l % off; step = 64 % off; }
    for (int32_t k = 0; k < len; k += 64) {
        int32_t hi = op + k;
        if (hi - c.F >= FLUSH_T) flush_to_line(s, c, hi);
        int32_t ringfloor = hi + 64 - R;
        int32_t i = k + l;
        uint32_t v = 0;
        int32_t x = 0;
        if (off > 0) x = (off >= 64) ? op - off + i : op - off + m;
        bool needg = (i < len) && off > 0 && x < ringfloor;
        if (__ballot(needg)) need_flushed(c, ringfloor);
        if (i < len) {
            if (off > 0) v = out_byte(s, c, x, ringfloor);
            s.ring[slot(c, op + i)] = (uint8_t)v;
        }
        if (off > 0 && off < 64) { m += step; if (m >= off) m -= off; }
    }
}

// ---------------------------------------------------------------------------
// exact serial restatement (wave-uniform): LZ4_decompress_generic 1.9.3
// ---------------------------------------------------------------------------
enum { SER_CONT = 0, SER_DONE = 1, SER_ERR = 2 };

struct Ser {
    int32_t ip, op;
    int fast;   // still in the fast loop
    int32_t ret;
};

__device__ __forceinline__ uint32_t gb(const Ctx &c, int32_t p) { return c.src[p]; }

__device__ __forceinline__ int rvl(const Ctx &c, int32_t *ip, int32_t lencheck, int loop_check, int initial_check,
                                   int64_t *len) {
    if (initial_check && *ip >= lencheck) return 1;
    uint32_t sv;
    do {
        sv = gb(c, *ip);
        (*ip)++;
        *len += sv;
        if (loop_check && *ip >= lencheck) return 2;
    } while (sv == 255);
    return 0;
}

__device__ __forceinline__ int ser_seq(Smem &s, Ctx &c, Ser &st) {
    const int32_t n = c.n, cap = c.cap;
    int32_t ip = st.ip, op = st.op;
    uint32_t token;
    int64_t length;
    int32_t offset = 0, match = 0;
    int64_t cpy;
    if (st.fast) {
        token = gb(c, ip++);
        length = token >> 4;
        if (length == 15) {
            if (rvl(c, &ip, n - 15, 1, 1, &length) == 1) goto err;
            cpy = op + length;
            if (cpy > cap - 32 || ip + length > n - 32) goto safe_lit;
        } else {
            cpy = op + length;
            if (ip > n - 17) goto safe_lit;
        }
        coop_lit(s, c, ip, op, (int32_t)length);
        ip += (int32_t)length;
        op = (int32_t)cpy;
        offset = (int32_t)(gb(c, ip) | (gb(c, ip + 1) << 8));
        ip += 2;
        match = op - offset;
        length = token & 15;
        if (length == 15) {
            if (match < 0) goto err;
            if (rvl(c, &ip, n - 4, 1, 0, &length) != 0) goto err;
            length += 4;
            if (op + length >= cap - 64) goto safe_match;
        } else {
            length += 4;
            if (op + length >= cap - 64) goto safe_match;
        }
        if (match < 0) goto err;
        coop_match(s, c, op, offset, (int32_t)length);
        op += (int32_t)length;
        st.ip = ip;
        st.op = op;
        return SER_CONT;
    }
    token = gb(c, ip++);
    length = token >> 4;
    if (length != 15 && ip < n - 16 && op <= cap - 32) {
        coop_lit(s, c, ip, op, (int32_t)length);
        op += (int32_t)length;
        ip += (int32_t)length;
        length = token & 15;
        offset = (int32_t)(gb(c, ip) | (gb(c, ip + 1) << 8));
        ip += 2;
        match = op - offset;
        if (length != 15 && offset >= 8 && match >= 0) {
            coop_match(s, c, op, offset, (int32_t)length + 4);
            op += (int32_t)length + 4;
            st.ip = ip;
            st.op = op;
            return SER_CONT;
        }
        goto copy_match;
    }
    if (length == 15) {
        if (rvl(c, &ip, n - 15, 1, 1, &length) == 1) goto err;
    }
    cpy = op + length;
safe_lit:
    st.fast = 0;
    if (cpy > cap - 12 || ip + length > n - 8) {
        if (ip + length != n || cpy > cap) goto err;
        coop_lit(s, c, ip, op, (int32_t)length);
        ip += (int32_t)length;
        op += (int32_t)length;
        st.ip = ip;
        st.op = op;
        st.ret = op;
        return SER_DONE;
    }
    coop_lit(s, c, ip, op, (int32_t)length);
    ip += (int32_t)length;
    op = (int32_t)cpy;
    offset = (int32_t)(gb(c, ip) | (gb(c, ip + 1) << 8));
    ip += 2;
    match = op - offset;
    length = token & 15;
copy_match:
    if (length == 15) {
        if (rvl(c, &ip, n - 4, 1, 0, &length) != 0) goto err;
    }
    length += 4;
safe_match:
    st.fast = 0;
    if (match < 0) goto err;
    cpy = op + length;
    if (cpy > cap - 12 && cpy > cap - 5) goto err;
    coop_match(s, c, op, offset, (int32_t)length);
    op = (int32_t)cpy;
    st.ip = ip;
    st.op = op;
    return SER_CONT;
err:
    st.ip = ip;
    st.ret = -ip - 1;
    return SER_ERR;
}

// ---------------------------------------------------------------------------
// lane-parallel copies (<= 16 bytes per step, byte-exact ring writes)
// ---------------------------------------------------------------------------
// Bytes [0, k) of a dword, k clamped to [0, 4].
__device__ __forceinline__ uint32_t lomask(int32_t k) {
    k = k < 0 ? 0 : k;
    return k >= 4 ? 0xFFFFFFFFu : ((1u << (8 * k)) - 1u);
}

__device__ __forceinline__ void lds_or(uint8_t *ring, uint32_t a, uint32_t v) {  // a % 4 == 0
    __hip_atomic_fetch_or(reinterpret_cast<uint32_t *>(ring) + (a >> 2), v, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Write bytes [ha, ha + m) (1 <= m <= 16, ha = da & 3) of the 20-byte span
// whose dwords are w0..w4 to the ring at slot da (dword 0 at da & ~3).
// The batch's output span is zeroed before it is produced, so every lane ORs
// its bytes in with whole-dword LDS atomics: lanes sharing a boundary dword
// cannot clobber each other, and no byte stores or branches are needed.
__device__ __forceinline__ void put16(Smem &s, uint32_t da, int32_t m, uint32_t w0, uint32_t w1, uint32_t w2,
                                      uint32_t w3, uint32_t w4) {
    uint8_t *ring = s.ring;
    const int32_t ha = (int32_t)(da & 3u), e8 = 8 * (ha + m);  // byte span [ha, ha + m) of the 20 bytes, in bits
    const uint32_t D0 = da & ~3u;
    // lomask(k) = high half of 0x00000000FFFFFFFF << 8k (k clamped to [0, 4])
    auto lm = [](int32_t b) -> uint32_t {
        const uint32_t sh = (uint32_t)(b < 0 ? 0 : b > 32 ? 32 : b);
        return (uint32_t)((0xFFFFFFFFull << sh) >> 32);
    };
    lds_or(ring, D0, w0 & lm(e8) & ~lm(8 * ha));
    lds_or(ring, (D0 + 4) & RMASK, w1 & lm(e8 - 32));
    lds_or(ring, (D0 + 8) & RMASK, w2 & lm(e8 - 64));
    lds_or(ring, (D0 + 12) & RMASK, w3 & lm(e8 - 96));
    lds_or(ring, (D0 + 16) & RMASK, w4 & lm(e8 - 128));
}

// Zero ring bytes of output [O0, O1) (bytes below O0 in the first dword are kept).
__device__ __forceinline__ void zero_span(Smem &s, const Ctx &c, int32_t O0, int32_t O1) {
    const int l = lane_id();
    const uint32_t a = slot(c, O0), h = a & 3u;
    const int32_t A = O0 + (int32_t)((4u - h) & 3u);  // first dword-aligned position >= O0
    if (l == 0 && h)
        __hip_atomic_fetch_and(reinterpret_cast<uint32_t *>(s.ring) + (a >> 2), lomask((int32_t)h), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    for (int32_t x = A + 4 * l; x < O1; x += 256) *(uint32_t *)(s.ring + slot(c, x)) = 0u;
}

// Copy m (1..16) bytes from LDS source byte address sa to ring slot da.
// RING: sa is a ring slot (dword reads wrap); else an offset into Smem.
template <bool RING>
__device__ __forceinline__ void copy16(Smem &s, uint32_t sa, uint32_t da, int32_t m) {
    const uint8_t *lds = (const uint8_t *)&s;
    const uint32_t ha = da & 3u;
    const uint32_t sb = sa - ha, S0 = sb & ~3u, sh = sb & 3u;
    uint32_t r[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t a = RING ? ((S0 + 4 * j) & RMASK) : (S0 + 4 * j);
        r[j] = *(const uint32_t *)(lds + a);
    }
    put16(s, da, m, __builtin_amdgcn_alignbyte(r[1], r[0], sh), __builtin_amdgcn_alignbyte(r[2], r[1], sh),
          __builtin_amdgcn_alignbyte(r[3], r[2], sh), __builtin_amdgcn_alignbyte(r[4], r[3], sh),
          __builtin_amdgcn_alignbyte(r[5], r[4], sh));
}


// Whole-wave copy of len bytes to output op from output op - D (all inside the
// ring), in chunks of at most D bytes so that self-overlapping matches repeat
// their period; plain byte stores (the bytes are not written by anyone else).
__device__ __forceinline__ void wave_near(Smem &s, const Ctx &c, int32_t op, int32_t D, int32_t len) {
    const int l = lane_id();
    const int32_t step = D < 64 ? D : 64;
    for (int32_t k = 0; k < len; k += step) {
        const int32_t i = k + l;
        if (l < step && i < len) s.ring[slot(c, op + i)] = s.ring[slot(c, op + i - D)];
    }
}
// Whole-wave copy of literal bytes [from, len) of a run staged at cw + litr.
__device__ __forceinline__ void wave_lit(Smem &s, const Ctx &c, int32_t op, uint32_t litr, int32_t from, int32_t len) {
    const int l = lane_id();
    for (int32_t k = from; k < len; k += 64) {
        const int32_t i = k + l;
        if (i < len) s.ring[slot(c, op + i)] = c.cw[litr + (uint32_t)i];
    }
}

// One lane-parallel batch: lanes with act hold consecutive tokens producing
// output [O0, O1), O1 - O0 <= BSPAN, every ll/ml <= LMAX.
__device__ __forceinline__ void batch(Smem &s, Ctx &c, bool act, int32_t o, uint32_t ll, uint32_t ml, uint32_t off,
                                      uint32_t litr, int32_t O0, int32_t O1 PROF_ARG) {
    // sources below hz come from HBM: the ring slots of [hz, O1) are intact
    // (zero_span may clear up to 3 bytes past O1, i.e. the slots of O1 - R ..)
    const int32_t hz = O1 + 4 - R;
    PCOUNT(14, 1);
    if (O0 - c.F >= FLUSH_T) flush_to_line(s, c, O0);
    if constexpr (!(DIAG & D_SKIP_ZERO)) zero_span(s, c, O0, O1);
    const int32_t ms = o + (int32_t)ll, msrc = ms - (int32_t)off;
    const bool hasm = act && ml > 0;
    const bool zero = hasm && off == 0;
    const bool far = hasm && off != 0 && msrc < hz;
    if (__ballot(far) && hz + LMAX > c.Fw) {
        wait_vm();
        c.Fw = c.F;
        if (hz + LMAX > c.Fw) c.bug = 4;
    }
    // far prefetch: the 24 bytes from the dword holding source byte (src - ha),
    // ha = the destination's offset in its dword, so that output dword j is
    // alignbyte(d[j+1], d[j], sh) with no dword selection
    uint32_t fd0 = 0, fd1 = 0, fd2 = 0, fd3 = 0, fd4 = 0, fd5 = 0;
    const uint32_t fha = slot(c, ms) & 3u;
    if (__ballot(far)) {
        if (far) far_load(c, (uintptr_t)(c.dst + msrc) - fha, fd0, fd1, fd2, fd3, fd4, fd5);
    }
    // literal runs (source: staged window, addressed as ring + R + litr)
    for (uint32_t k = 0; !(DIAG & D_SKIP_LIT) && __ballot(act && k < ll); k += 16) {
        PCOUNT(16, 1);
        if (act && k < ll) {
            const int32_t m = ll - k < 16u ? (int32_t)(ll - k) : 16;
            copy16<false>(s, c.cwoff + litr + k, slot(c, o + (int32_t)k), m);
        }
    }
    PSTAMP(4);
    // far matches (offset-0 matches write zeros: the span is already zero)
    if (!(DIAG & D_SKIP_FAR) && __ballot(far)) {
        for (uint32_t k = 0; __ballot(far && k < ml); k += 16) {
            PCOUNT(17, 1);
            if (far && k < ml) {
                const int32_t m = ml - k < 16u ? (int32_t)(ml - k) : 16;
                const uint32_t da = slot(c, ms + (int32_t)k);  // da & 3 == fha
                const uint32_t sh = (uint32_t)((uintptr_t)(c.dst + msrc + (int32_t)k) - fha) & 3u;
                put16(s, da, m, __builtin_amdgcn_alignbyte(fd1, fd0, sh), __builtin_amdgcn_alignbyte(fd2, fd1, sh),
                      __builtin_amdgcn_alignbyte(fd3, fd2, sh), __builtin_amdgcn_alignbyte(fd4, fd3, sh),
                      __builtin_amdgcn_alignbyte(fd5, fd4, sh));
            }
            const bool more = far && k + 16 < ml;
            if (__ballot(more)) {
                if (more) far_load(c, (uintptr_t)(c.dst + msrc + (int32_t)k + 16) - fha, fd0, fd1, fd2, fd3, fd4, fd5);
            }
        }
    }
    PSTAMP(5);
    // source substitution: out[x] == out[x - off_i] for every byte x a match i
    // writes, so a pending match whose whole source lies inside another pending
    // match of this batch can read that match's source instead (repeatedly).
    // This shortens the dependency chains the rounds below must walk.
    bool pend = hasm && !far && !zero;
    int32_t src = msrc;
    const uint64_t am = __ballot(act);
    const int first = am ? (int)__builtin_ctzll(am) : 0;
    const uint32_t key = act ? (uint32_t)ms : (lane_id() < first ? 0u : 0xFFFFFFFFu);  // non-decreasing
    bool litsrc = false;  // the source lies wholly inside one literal run of this batch (written above)
    {
        // one hop (measured: 1 > 2 > 3 hops with the whole-wave tail below)
        const uint32_t mek = pend ? (uint32_t)(ms + (int32_t)ml) : 0u;
        const bool want = !(DIAG & D_SKIP_SUBST) && pend && off >= ml && src >= O0;
        if (__ballot(want)) {
            int lo = 0;  // last lane with key <= src
#pragma unroll
            for (int stp = 32; stp; stp >>= 1) {
                const uint32_t v = (uint32_t)__shfl((int)key, lo + stp, 64);
                lo = v <= (uint32_t)src ? lo + stp : lo;
            }
            const uint32_t vms = (uint32_t)__shfl((int)key, lo, 64);
            const uint32_t vme = (uint32_t)__shfl((int)mek, lo, 64);
            const int32_t voff = __shfl((int)off, lo, 64);
            const bool ok = want && vms <= (uint32_t)src && (uint32_t)(src + (int32_t)ml) <= vme && voff > 0 &&
                            src - voff >= hz;
            // past the end of lane lo's match and before the next lane's match
            // start: inside the next token's literal run, already in the ring
            const uint32_t nms = (uint32_t)__shfl((int)key, lo + 1 < 64 ? lo + 1 : 63, 64);
            litsrc = want && vms <= (uint32_t)src && (uint32_t)src >= vme && lo < 63 &&
                     (uint32_t)(src + (int32_t)ml) <= nms;
            src = ok ? src - voff : src;
        }
    }
    // near matches: one round in which every ready lane (source wholly before
    // the batch, or inside one of its literal runs) copies its first (<= 16
    // byte) step; what is left (lanes whose source waits on a match of this
    // batch, matches longer than one step) is copied by the whole wave in lane
    // order, which is output order, so every source is complete when its
    // lane's turn comes
    int32_t pos = ms, rem = (int32_t)ml, D = ms - src;
    const int32_t send = src + (int32_t)ml < ms ? src + (int32_t)ml : ms;
    if (!(DIAG & D_SKIP_NEAR)) {
        PCOUNT(18, 1);
        const bool go = pend && (send <= O0 || litsrc);
        if (__ballot(go)) {
            PCOUNT(15, 1);
            if (go) {
                const int32_t m = rem < 16 ? (rem < D ? rem : D) : (D < 16 ? D : 16);
                copy16<true>(s, slot(c, pos - D), slot(c, pos), m);
                pos += m;
                rem -= m;
                if (rem <= 0) pend = false;
            }
        }
        for (uint64_t pmk = __ballot(pend); pmk; pmk &= pmk - 1) {
            const int j = (int)__builtin_ctzll(pmk);
            PCOUNT(19, 1);
            wave_near(s, c, (int32_t)readlane((uint32_t)pos, j), (int32_t)readlane((uint32_t)D, j),
                      (int32_t)readlane((uint32_t)rem, j));
        }
    }
    PSTAMP(6);
}

// Copy the window's tokens [0, T) (positions in s.tab, relative to cbase),
// starting at output op0.  Returns the number of tokens copied; fewer than T
// when an output-side fast-loop check declines a token (*bad_ip = its input
// position).  *end_op = output position after the copied tokens.
__device__ __forceinline__ uint32_t copy_tokens(Smem &s, Ctx &c, uint32_t T, int32_t op0, int32_t *end_op,
                                                int32_t *bad_ip PROF_ARG) {
    const int l = lane_id();
    int32_t op = op0;
    const int32_t cap = c.cap;
    if constexpr ((DIAG & D_PARSEONLY) != 0) {
        *end_op = op0;
        return T;
    }
    for (uint32_t g0 = 0; g0 < T; g0 += 64) {
        const uint32_t n0 = T - g0 < 64u ? T - g0 : 64u;
        const bool in0 = (uint32_t)l < n0;
        const int32_t p = c.cbase + (in0 ? (int32_t)c.tab[g0 + l] : 0);
        FTok t = parse_fast(s, c, p);
        const bool sl = in0 && t.slow;
        if (__ballot(sl)) {
            if (sl) {
                const Tok u = parse_tok(s, c, p);
                t.lit = u.lit;
                t.ll = (uint32_t)u.ll;
                t.ml = (uint32_t)u.ml;
                t.off = (uint32_t)u.off;
                t.llx = (uint32_t)u.llx;
            }
        }
        const uint32_t ll = in0 ? t.ll : 0u, ml = in0 ? t.ml : 0u, off = t.off;
        const uint32_t litr = (uint32_t)(t.lit - c.cbase);
        const uint32_t len = ll + ml;
        const uint32_t incl = dpp_scan_add(len);
        const int32_t o = op + (int32_t)(incl - len);
        const int32_t om = o + (int32_t)ll;
        const bool bad = in0 && ((t.llx && om > cap - 32) || (om + (int32_t)ml >= cap - 64) || ((int32_t)off > om));
        const uint64_t bm = __ballot(bad);
        const uint32_t n = bm ? (uint32_t)__builtin_ctzll(bm) : n0;
        const bool in = (uint32_t)l < n;
        const int32_t endo = o + (int32_t)len;
        const bool lng = in && (ll > (uint32_t)LMAX || ml > (uint32_t)LMAX);
        PSTAMP(2);
        uint32_t j = 0;
        while (j < n) {
            const int32_t oj = (int32_t)readlane((uint32_t)o, (int)j);
            if (readlane(lng ? 1u : 0u, (int)j)) {  // one long token, whole wave
                const uint32_t jll = readlane(ll, (int)j), jml = readlane(ml, (int)j), joff = readlane(off, (int)j);
                const uint32_t jlit = readlane(litr, (int)j);
                coop_lit(s, c, c.cbase + (int32_t)jlit, oj, (int32_t)jll);
                coop_match(s, c, oj + (int32_t)jll, (int32_t)joff, (int32_t)jml);
                PSTAMP(7);
                j++;
                continue;
            }
            const bool ok = (uint32_t)l >= j && in && !lng && endo - oj <= BSPAN;
            const uint64_t stop = __ballot(!ok) & (~0ull << j);
            const uint32_t e = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
            const uint32_t eb = e > n ? n : e;
            const bool act = (uint32_t)l >= j && (uint32_t)l < eb;
            const int32_t O1 = (int32_t)readlane((uint32_t)endo, (int)eb - 1);
            PSTAMP(3);
            if constexpr (!(DIAG & D_NOCOPY)) batch(s, c, act, o, ll, ml, off, litr, oj, O1 PROF_PASS);
            j = eb;
        }
        if (bm) {
            *bad_ip = (int32_t)readlane((uint32_t)p, (int)n);
            *end_op = (int32_t)readlane((uint32_t)o, (int)n);
            return g0 + n;
        }
        op += (int32_t)readlane(incl, 63);
    }
    *end_op = op;
    return T;
}

// ---------------------------------------------------------------------------
// segment-walk parser (round 3): the token chain of a span of SW = 64 * SEG
// compressed bytes at once, one SEG-byte segment per lane, read straight from
// HBM (no staging).  Each lane walks its segment speculatively from SPRE bytes
// before it (lane 0 from the exact entry), fix-up rounds take each segment's
// true entry (the previous segment's exit) until nothing changes.  The chain
// positions stay in the lanes' registers (SEG bits each) while the windows of
// the span are staged and tabled.  A long segment amortizes the pre-roll and
// the fix-up over ~SEG/5.6 tokens per lane; the window exit-table parser spent
// ~29 VALU per byte offset.
// ---------------------------------------------------------------------------
static_assert(SEG == 128, "segment bit sets are two u64 per lane");
constexpr int SW = 64 * SEG;
constexpr int SPRE = 32;         // speculative pre-roll before each segment (16 / 48 measured no better)
constexpr int SEG_BUDGET = 64;   // at most this many walk steps of the next span per window
constexpr int SEG_MIN = 4;       // at least this many (more while the copier is busy)

// Next token position after p (or STOP | p): the exact chain rule of
// parse_tok, bytes from HBM.
__device__ __noinline__ uint32_t g_next_exact(const Ctx &c, int32_t p) {
    const int32_t n = c.n;
    if (p > n - 18) return STOP | (uint32_t)p;
    const uint32_t tb = c.src[p];
    int32_t q = p + 1;
    int32_t ll = (int32_t)(tb >> 4);
    if (ll == 15) {
        int k = 0;
        uint32_t sv;
        do {
            sv = c.src[q];
            q++;
            ll += (int32_t)sv;
            if (q >= n - 15 || ++k > KEXT) return STOP | (uint32_t)p;
        } while (sv == 255);
        if (q + ll > n - 32) return STOP | (uint32_t)p;
    }
    q += ll + 2;
    if ((tb & 15u) == 15u) {
        int k = 0;
        uint32_t sv;
        do {
            sv = c.src[q];
            q++;
            if (q >= n - 4 || ++k > KEXT) return STOP | (uint32_t)p;
        } while (sv == 255);
    }
    return (uint32_t)q;
}

// Lean step from HBM: the token byte and the byte after it, then the first
// match-length byte (two dependent load rounds).  A literal length with one
// extension byte is taken here; tokens with a 255 extension byte (runs of
// >= 270 literals or >= 274-byte matches) take g_next_exact.
__device__ __forceinline__ uint32_t g_step(const Ctx &c, int32_t p, bool act) {
    // unsigned 32-bit offsets from the uniform base: saddr loads, no 64-bit
    // address arithmetic; bitwise 0/1 logic: no exec-mask branches
    const int32_t n = c.n;
    const uint32_t edge = (uint32_t)(p > n - 18);
    const uint32_t up = (uint32_t)p;
    const uint32_t tb = c.src[edge ? 0u : up], e1 = c.src[edge ? 0u : up + 1u];
    const uint32_t hi = tb >> 4;
    const uint32_t llx = (uint32_t)(hi == 15u);
    const uint32_t L = llx ? 15u + e1 : hi;
    const uint32_t lstop = llx & ((uint32_t)(p + 2 >= n - 15) | (uint32_t)(p + 2 + (int32_t)L > n - 32));
    const uint32_t q = up + 3u + llx + L;  // first match-length extension byte
    const uint32_t e2 = c.src[(edge | lstop) ? 0u : q];
    const uint32_t mlx = (uint32_t)((tb & 15u) == 15u);
    uint32_t x = q + mlx;
    const uint32_t slow = (uint32_t)act & (edge ^ 1u) & (lstop ^ 1u) & ((llx & (uint32_t)(e1 == 255u)) | (mlx & (uint32_t)(e2 == 255u)));
    x = (edge | lstop | (mlx & (uint32_t)((int32_t)x >= n - 4))) ? (STOP | up) : x;
    if (__ballot(slow)) {
        if (slow) x = g_next_exact(c, p);
    }
    return x;
}

// 128-bit sets as two u64 (bit d = position plo + d)
__device__ __forceinline__ bool tbit2(uint64_t a0, uint64_t a1, uint32_t d) {
    return (((d < 64u ? a0 : a1) >> (d & 63u)) & 1ull) != 0;
}
__device__ __forceinline__ void sbit2(uint64_t &a0, uint64_t &a1, uint32_t d) {
    const uint64_t m = 1ull << (d & 63u);
    a0 |= d < 64u ? m : 0ull;
    a1 |= d < 64u ? 0ull : m;
}
__device__ __forceinline__ uint64_t from_lo(uint32_t d) { return d < 64u ? (~0ull << (d & 63u)) : 0ull; }
__device__ __forceinline__ uint64_t from_hi(uint32_t d) { return d < 64u ? ~0ull : (~0ull << (d & 63u)); }

// Chain of the span [base, base + SW), resumable: advance() runs at most
// `budget` walk steps (one HBM load round each) and returns true once the
// chain is final, so the parser wave can walk the next span a few steps per
// window while the copier works (the walk is bound by load latency).
// Result: vt0/vt1 = true chain positions of this lane's segment, ex = its
// true exit (first position >= its end, or STOP | p).
struct SegWalk {
    int32_t base, plo, phi;
    int32_t q;            // walk position of a moving lane
    uint32_t cur;         // entry the current result assumes
    uint32_t sx, ex;      // speculative / true exit
    uint64_t vs0, vs1;    // speculative chain positions
    uint64_t vt0, vt1;    // true chain positions
    uint64_t vp0, vp1;    // positions of a fix-up walk
    bool mv;              // this lane is walking
    int phase;            // 0 speculative walk, 1 fix-up rounds, 2 final
    bool round;           // a fix-up round is to be started
    int steps, rounds;

    __device__ __forceinline__ void start(int32_t b) {
        const int l = lane_id();
        base = b;
        plo = b + l * SEG;
        phi = plo + SEG;
        cur = l == 0 ? (uint32_t)b : (uint32_t)(plo - SPRE);
        q = (int32_t)cur;
        vs0 = vs1 = vt0 = vt1 = vp0 = vp1 = 0;
        sx = ex = 0;
        mv = true;
        phase = 0;
        round = false;
        steps = rounds = 0;
    }

    __device__ __forceinline__ bool advance(Ctx &c, int budget PROF_ARG) {
        // speculative walks (one load round trip per step for every lane)
        if (phase == 0) {
            for (; budget > 0 && __ballot(mv); --budget) {
                PCOUNT(11, 1);
                if (mv) {
                    const uint32_t x = g_step(c, q, true);
                    const bool stop = (x & STOP) != 0;
                    if (!stop && q >= plo) sbit2(vs0, vs1, (uint32_t)(q - plo));
                    const bool out = stop || (int32_t)x >= phi;
                    sx = out ? x : sx;
                    mv = !out;
                    q = (int32_t)x;
                }
                if (++steps > SEG + SPRE) { c.bug = 6; phase = 2; return true; }
            }
            if (budget == 0) return false;
            vt0 = vs0;
            vt1 = vs1;
            ex = sx;
            phase = 1;
            round = true;
        }
        // fix-up rounds: true entry = exit of the previous segment; an entry
        // off the speculative chain walks until it joins it (or leaves)
        while (phase == 1 && budget > 0) {
            if (round) {
                const uint32_t In = dpp_shift_up(ex, (uint32_t)base);
                const bool ch = In != cur;
                if (!__ballot(ch)) { phase = 2; break; }
                if (++rounds > 64) { c.bug = 3; phase = 2; break; }
                PCOUNT(12, 1);
                mv = false;
                if (ch) {
                    cur = In;
                    const uint32_t d = In - (uint32_t)plo;
                    if ((In & STOP) || (int32_t)In >= phi) {
                        vt0 = vt1 = 0;
                        ex = In;
                    } else if (tbit2(vs0, vs1, d)) {
                        vt0 = vs0 & from_lo(d);
                        vt1 = vs1 & from_hi(d);
                        ex = sx;
                    } else {
                        mv = true;
                    }
                }
                q = (int32_t)In;
                vp0 = vp1 = 0;
                steps = 0;
                round = false;
            }
            for (; budget > 0 && __ballot(mv); --budget) {
                PCOUNT(13, 1);
                if (mv) {
                    const uint32_t d = (uint32_t)(q - plo);
                    const bool join = tbit2(vs0, vs1, d);
                    const uint32_t x = g_step(c, q, !join);
                    const bool stop = !join && (x & STOP) != 0;
                    if (!join && !stop) sbit2(vp0, vp1, d);
                    const bool out = join || stop || (int32_t)x >= phi;
                    if (out) {
                        vt0 = vp0 | (join ? vs0 & from_lo(d) : 0ull);
                        vt1 = vp1 | (join ? vs1 & from_hi(d) : 0ull);
                        ex = join ? sx : x;
                    }
                    mv = !out;
                    q = (int32_t)x;
                }
                if (++steps > SEG + 1) { c.bug = 7; phase = 2; return true; }
            }
            if (!__ballot(mv)) round = true;
        }
        return phase == 2;
    }
};

// Dword k (0..4*64-1) of the span's bit set; lane k/4 holds it as dword k%4 of
// (vt0, vt1).  Out-of-span dwords read as 0.
__device__ __forceinline__ uint32_t span_dword(uint64_t vt0, uint64_t vt1, int32_t k) {
    const int src = (k >> 2) & 63;
    const uint32_t d0 = (uint32_t)__shfl((int)(uint32_t)vt0, src, 64);
    const uint32_t d1 = (uint32_t)__shfl((int)(uint32_t)(vt0 >> 32), src, 64);
    const uint32_t d2 = (uint32_t)__shfl((int)(uint32_t)vt1, src, 64);
    const uint32_t d3 = (uint32_t)__shfl((int)(uint32_t)(vt1 >> 32), src, 64);
    const uint32_t j = (uint32_t)k & 3u;
    const uint32_t v = j == 0 ? d0 : j == 1 ? d1 : j == 2 ? d2 : d3;
    return (k >= 0 && k < 4 * 64) ? v : 0u;
}

// The chain of one span (seg_chain), kept by the parser wave across windows.
struct Span {
    uint64_t v0, v1;  // this lane's segment bits
    int32_t base;     // span start (a true chain position)
    uint32_t exit;    // first chain position >= base + SW, or STOP | p
};

// Stage the window at wbase and table its tokens from the span's chain: the
// window ends at cbase + CW or at the span's end, whichever comes first.
__device__ __forceinline__ void parse_window_seg(Smem &s, Ctx &c, int32_t wbase, const Span &sp, uint32_t *T_out,
                                                 uint32_t *efin_out PROF_ARG) {
    static_assert(P == 32, "a window lane covers one dword of the span bit set");
    const int l = lane_id();
    stage_window(s, c, wbase);
    const int32_t cbase = c.cbase;
    PCOUNT(10, 1);
    __builtin_amdgcn_wave_barrier();
    PSTAMP(0);
    const int32_t send = sp.base + SW;
    const int32_t wend = cbase + CW < send ? cbase + CW : send;
    // lane l: positions [cbase + 32 l, + 32) = span bits [o, o + 32)
    const int32_t o = cbase - sp.base + 32 * l;  // >= -15
    const int32_t K = o >> 5;
    const uint32_t lo = span_dword(sp.v0, sp.v1, K), hi = span_dword(sp.v0, sp.v1, K + 1);
    uint32_t field = __builtin_amdgcn_alignbit(hi, lo, (uint32_t)o & 31u);
    const int32_t plo = cbase + 32 * l;
    const int32_t a = wbase - plo, b = wend - plo;  // keep bits [a, b)
    const uint32_t ma = a <= 0 ? 0xFFFFFFFFu : a >= 32 ? 0u : (0xFFFFFFFFu << a);
    const uint32_t mb = b >= 32 ? 0xFFFFFFFFu : b <= 0 ? 0u : ((1u << b) - 1u);
    field &= ma & mb;
    PSTAMP(1);
    // token table: positions (relative to cbase) in stream order
    const uint32_t cnt = (uint32_t)__builtin_popcount(field);
    const uint32_t cinc = dpp_scan_add(cnt);
    const uint32_t tall = readlane(cinc, 63);
    *T_out = tall < (uint32_t)TCAP ? tall : (uint32_t)TCAP;
    uint32_t ex = 0;
    {
        uint32_t idx = cinc - cnt;
        uint32_t v = field;
        while (__ballot(v != 0)) {
            if (v) {
                const uint32_t bb = (uint32_t)__builtin_ctz(v);
                if (idx < (uint32_t)TCAP) c.tab[idx] = (uint16_t)((uint32_t)l * P + bb);
                else if (idx == (uint32_t)TCAP) ex = (uint32_t)plo + bb;  // first token left to the next window
                idx++;
                v &= v - 1;
            }
        }
    }
    if (tall > (uint32_t)TCAP) {  // the window ends at token TCAP
        const uint64_t hit = __ballot(cinc - cnt <= (uint32_t)TCAP && (uint32_t)TCAP < cinc);
        *efin_out = readlane(ex, (int)__builtin_ctzll(hit));
    } else if (wend >= send) {
        *efin_out = sp.exit;
    } else {
        // first chain position >= wend inside the span, else the span's exit
        const int32_t d = wend - sp.base - l * SEG;
        const uint32_t dd = d < 0 ? 0u : (uint32_t)d;
        const uint64_t m0 = d >= SEG ? 0ull : sp.v0 & from_lo(dd), m1 = d >= SEG ? 0ull : sp.v1 & from_hi(dd);
        const uint64_t any = __ballot((m0 | m1) != 0ull);
        if (any) {
            const int f = (int)__builtin_ctzll(any);
            const uint32_t bit = m0 ? (uint32_t)__builtin_ctzll(m0) : 64u + (uint32_t)__builtin_ctzll(m1 | (1ull << 63));
            *efin_out = (uint32_t)sp.base + (uint32_t)(f * SEG) + readlane(bit, f);
        } else {
            *efin_out = sp.exit;
        }
    }
    PSTAMP(2);
}

// LDS-only workgroup barrier between the parser and copier waves
__device__ __forceinline__ void wg_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ void use_buffer(Smem &s, Ctx &c, int buf) {
    c.cw = s.cwin[buf];
    c.cwoff = (uint32_t)((const uint8_t *)s.cwin[buf] - (const uint8_t *)&s);
    c.tab = s.tab[buf];
}

// Pipeline: in step k the parser stages and parses window k into buffer k&1
// while the copier copies window k-1 from the other buffer; two barriers per
// step.  When the copier has to take tokens exactly (a stop token, an
// output-side check, the end of the block) it runs the serial restatement
// and, if the fast path applies again, restarts the parser at the new input
// position (the window the parser produced meanwhile is skipped).
__device__ __forceinline__ void parser_wave(Smem &s, Ctx &c PROF_ARG) {
    int32_t pip = 0;
    bool pstop = false;
    Span sp;
    sp.v0 = sp.v1 = 0;
    sp.base = 0;
    sp.exit = 0;
    bool spv = false;  // sp describes the chain from sp.base
    bool nxt = false;  // wk walks the span that follows sp
    SegWalk wk;
    wk.start(0);
    for (uint32_t k = 0;; ++k) {
        const int buf = (int)(k & 1u);
        Meta m;
        m.kind = W_NONE;
        m.wbase = pip;
        m.cbase = 0;
        m.T = 0;
        m.efin = 0;
        if (!pstop) {
            if (pip < c.n - 64) {
                use_buffer(s, c, buf);
                uint32_t T, efin;
                if (!spv || pip >= sp.base + SW) {
                    // the span at pip: the walk started ahead of time, or a fresh one
                    if (!(spv && nxt && wk.base == pip)) wk.start(pip);
                    wk.advance(c, 1 << 20 PROF_PASS);
                    PSTAMP(1);
                    sp.v0 = wk.vt0;
                    sp.v1 = wk.vt1;
                    sp.base = pip;
                    sp.exit = readlane(wk.ex, 63);
                    spv = true;
                    nxt = !(sp.exit & STOP) && !c.bug;
                    if (nxt) wk.start((int32_t)sp.exit);  // walk the next span during this one's windows
                }
                parse_window_seg(s, c, pip, sp, &T, &efin PROF_PASS);
                if (nxt) {
                    // walk the next span while the copier is still busy with its
                    // window (at least SEG_MIN steps per window)
                    bool fin = wk.advance(c, SEG_MIN PROF_PASS);
                    for (int g = SEG_MIN; !fin && g < SEG_BUDGET; g += 2) {
                        if (__hip_atomic_load(&s.ctl.step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (int32_t)k)
                            break;
                        fin = wk.advance(c, 2 PROF_PASS);
                    }
                }
                PSTAMP(1);
                m.kind = c.bug ? W_BUG : W_WIN;
                m.cbase = c.cbase;
                m.T = T;
                m.efin = efin;
                if ((efin & STOP) || c.bug) pstop = true;
                else pip = (int32_t)efin;
            } else {
                m.kind = W_SER;
                pstop = true;
            }
        }
        if (lane_id() == 0) s.meta[buf] = m;
        wg_sync();
        const int32_t done = (int32_t)uniform((uint32_t)s.ctl.done), restart = (int32_t)uniform((uint32_t)s.ctl.restart),
                      rip = (int32_t)uniform((uint32_t)s.ctl.rip);
        wg_sync();
        PSTAMP(9);
        if (done) break;
        if (restart) {
            pip = rip;
            pstop = false;
            spv = false;
            nxt = false;
        }
    }
}

__device__ __forceinline__ void copier_wave(Smem &s, Ctx &c, int32_t *retp PROF_ARG) {
    __builtin_amdgcn_s_setprio(1);  // the copier is the critical wave of the pair (2 / 3: no better)
    Ser st;
    st.ip = 0;
    st.op = 0;
    st.fast = c.cap >= 64;
    st.ret = 0;
    bool skip = false;
    int32_t result = INT32_MIN;
    int64_t nser = 0;
    if (lane_id() == 0) __hip_atomic_store(&s.ctl.step, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    for (uint32_t k = 0;; ++k) {
        int32_t done = 0, restart = 0, rip = 0;
        if (k > 0 && !skip) {
            const int buf = (int)((k - 1) & 1u);
            Meta m;
            m.kind = (int32_t)uniform((uint32_t)s.meta[buf].kind);
            m.wbase = (int32_t)uniform((uint32_t)s.meta[buf].wbase);
            m.cbase = (int32_t)uniform((uint32_t)s.meta[buf].cbase);
            m.T = uniform(s.meta[buf].T);
            m.efin = uniform(s.meta[buf].efin);
            bool ser = false;
            if (m.kind == W_BUG || m.kind == W_NONE || m.wbase != st.ip) {
                c.bug |= 8;
            } else if (m.kind == W_WIN && st.fast && st.ip < c.n - 64 && st.op < c.cap - 128) {
                use_buffer(s, c, buf);
                c.cbase = m.cbase;
                int32_t end_op = st.op, bad_ip = 0;
                const uint32_t dn = m.T > 0 ? copy_tokens(s, c, m.T, st.op, &end_op, &bad_ip PROF_PASS) : 0u;
                st.op = end_op;
                if (dn < m.T) {
                    st.ip = bad_ip;
                    ser = true;
                } else {
                    st.ip = (int32_t)(m.efin & ~STOP);
                    ser = (m.efin & STOP) != 0;
                }
            } else {
                ser = true;  // W_SER, or the window's start is not fast-path eligible
            }
            if (ser && !c.bug) {
                // tokens the fast path declines: exact, wave-uniform liblz4 1.9.3 steps
                c.cbase = 0x3fffffff;  // no staged window describes st.ip
                for (;;) {
                    const int status = ser_seq(s, c, st);
                    if (status != SER_CONT) {
                        if (status == SER_DONE) flush(s, c, st.op);
                        result = st.ret;
                        done = 1;
                        break;
                    }
                    if (++nser > (int64_t)c.n + 64) { c.bug |= 16; break; }
                    if (st.fast && st.ip < c.n - 64 && st.op < c.cap - 128) {
                        restart = 1;
                        rip = st.ip;
                        break;
                    }
                }
                PSTAMP(7);
            }
            if (c.bug) {
                done = 1;
                restart = 0;
                result = INT32_MIN;
            }
        }
        if (k > (uint32_t)c.n + 64) {  // every step consumes input or finishes the block
            done = 1;
            result = INT32_MIN;
        }
        if (lane_id() == 0) {
            s.ctl.done = done;
            s.ctl.restart = restart;
            s.ctl.rip = rip;
            __hip_atomic_store(&s.ctl.step, (int32_t)k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        wg_sync();
        wg_sync();
        PSTAMP(8);
        if (done) break;
        skip = restart != 0;
    }
    if (lane_id() == 0) *retp = result;
}

// Residency: 4096 blocks on 256 CUs is 16 workgroups (32 waves) per CU, all
// resident at once only with <= 64 VGPRs, <= 10 KiB of LDS and <= 80 SGPRs
// (above 80 the CU admits 7 waves per SIMD, above 96 six).  The SGPR cap
// costs some SGPR spills to VGPR lanes and buys 16% (measured: 229 -> 267 GiB/s).
#define JFS_LZ4_ATTR __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(8)))
// lens (optional): per-block input lengths produced on the device by the
// previous kernel of a fused chain (AES-GCM open); < 0 = that step failed.
// todo (optional): only the blocks with todo[b] != 0 are decoded (the others
// were decoded by lz4_split.hip and keep its results).
__global__ __launch_bounds__(128) JFS_LZ4_ATTR void lz4_decode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                        int32_t *__restrict__ ret,
                                                        const int32_t *__restrict__ lens,
                                                        const int32_t *__restrict__ todo) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    if (b >= nblk) return;
    if (todo && !todo[b]) return;
    const int wave = (int)uniform(threadIdx.x >> 6);
    jfs_dev_block d = ((const gc_blk *)blocks)[b];
    Ctx c;
    c.src = (const gc_u8 *)d.src;
    c.dst = (g_u8 *)d.dst;
    c.n = lens ? lens[b] : d.src_len;
    if (lens && c.n < 0) {  // the chained step failed: report it, decode nothing
        if (threadIdx.x == 64) ret[b] = JFS_CHAIN_FAILED;
        return;
    }
    c.cap = d.dst_cap;
    c.F = 0;
    c.Fw = 0;
    c.dmis = (uint32_t)((uintptr_t)d.dst & 15u);
    c.cbase = 0x3fffffff;
    c.bug = 0;
    use_buffer(s, c, 0);
#ifdef JFS_PROF
    Prof pr;
    pr.start();
#endif
    // inputs that never reach the decode loop (no barrier: both waves return)
    int32_t early = 1, result = 0;
    if (d.src == nullptr || c.n < 0 || c.cap < 0) result = -1;
    else if (c.cap == 0) result = (c.n == 1 && c.src[0] == 0) ? 0 : -1;
    else if (c.n == 0) result = -1;
    else early = 0;
    if (early) {
        if (wave == 1 && lane_id() == 0) ret[b] = result;
        return;
    }
    if (wave == 0) parser_wave(s, c PROF_PASS);
    else copier_wave(s, c, ret + b PROF_PASS);
#ifdef JFS_PROF
    pr.flush_out();
#endif
}

}  // namespace lz4d
}  // namespace jfs

#ifdef JFS_PROF
extern "C" int jfs_prof_read(uint64_t *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::lz4d::g_prof), sizeof(uint64_t) * NPROF) == hipSuccess ? 0 : -1;
}
extern "C" int jfs_prof_reset() {
    uint64_t z[NPROF] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::lz4d::g_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int jfs_launch_lz4_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    return jfs_launch_lz4_decode_lens(d_blocks, nblk, d_ret, nullptr, stream);
}

extern "C" int jfs_launch_lz4_decode_lens(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, const int32_t *d_lens,
                                          hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4d::lz4_decode_kernel, dim3(nblk), dim3(128), 0, stream, d_blocks, nblk, d_ret, d_lens,
                       (const int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int jfs_launch_lz4_decode_todo(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, const int32_t *d_todo,
                                          hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4d::lz4_decode_kernel, dim3(nblk), dim3(128), 0, stream, d_blocks, nblk, d_ret,
                       (const int32_t *)nullptr, d_todo);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
