// LZ4 block decoder for gfx950 -- one wavefront per block.
//
// Replaces LZ4_decompress_safe reached from pkg/compress/compress.go:120-125
// (LZ4.Decompress -> lz4.DecompressSafe).  Result semantics (decoded size, or
// the same negative error value liblz4 1.9.3 returns) are restated in
// oracle/lz4_oracle.c; parity is tested in tests/test_lz4_gpu.py.
//
// Design (DESIGN.md "LZ4 decode"):
//   The compressed stream is processed in windows of CW bytes staged in LDS.
//   1. Parse DP: each lane owns a 32-byte piece of the window and, walking its
//      piece backwards, computes for EVERY byte position p the position where
//      the token chain that would start at p leaves the piece (exit[p]).
//      Tokens that need the exact liblz4 end-of-buffer rules, or whose length
//      fields are very long, are marked STOP.
//   2. Fix-up: the true entry of every piece, from the window entry.  Done as
//      parallel fixed-point rounds (entry_k <- exit_{k-1}(entry_{k-1}), one LDS
//      lookup per lane per round) followed by a wave-uniform verification
//      pass that only touches LDS where a guess was wrong.
//   3. Each lane walks the true chain of its piece, recording token positions;
//      DPP prefix sums give token indices and output offsets; tokens land in
//      an LDS table in stream order (SoA).
//   4. Copy (output-centric gather): the window's output is produced in
//      256-byte chunks, lane l owning bytes [4l, 4l+4).  Each lane finds its
//      token(s) from a per-chunk start marker + DPP max-scan, computes each
//      byte's source (literal in the staged input, earlier output in the LDS
//      ring, or HBM for offsets beyond the ring), and writes one dword.  Bytes
//      whose source lies earlier in the same chunk resolve in extra rounds.
//      Sources in HBM for chunk i+1 are loaded while chunk i is produced.
//      The ring is streamed to HBM with 16-byte stores at 128-byte lines.
//   5. Everything the fast path does not cover (the last bytes of input /
//      output, malformed input, very long length fields) runs through an
//      exact, wave-uniform restatement of the liblz4 1.9.3 state machine.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4d {

constexpr int P = 32;                  // bytes per lane piece
constexpr int CW = 64 * P;             // compressed window bytes handled per pass
constexpr int CWIN = CW + 80;          // LDS staging incl. lookahead (multiple of 16)
constexpr int R = 8192;                // output ring bytes
constexpr int RMASK = R - 1;
constexpr int TMAX = CW / 3 + 2;       // max tokens in a window (interior token >= 3 bytes)
constexpr int TPMAX = (P + 2) / 3;     // max tokens starting in one piece (11)
constexpr uint32_t STOP = 0x80000000u;
constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr int KEXT = 64;               // max 255-extension bytes handled by the fast path
constexpr int FLUSH_T = 1024;          // flush the ring when this many bytes are pending
constexpr int FIX_ROUNDS = 6;          // parallel fix-up rounds before the verification pass

#ifdef JFS_PROF
// diagnostic build only: per-phase cycle sums (s_memtime), never in the product .so
#define NPROF 10
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
#define PROF_ARG , Prof &pr
#define PROF_PASS , pr
#else
#define PSTAMP(k)
#define PROF_ARG
#define PROF_PASS
#endif

struct Smem {
    alignas(16) uint8_t ring[R];
    alignas(16) uint8_t cwin[CWIN];
    alignas(16) union {
        uint32_t ex[CW];
        struct {
            uint32_t o[TMAX + 1];    // output position of the token
            uint32_t lit[TMAX + 1];  // literal source position (input)
            uint32_t lo[TMAX + 1];   // ll | off << 16
        } tk;
    } u;
    uint32_t mk[64];  // per-chunk token-start markers
};

static_assert(__builtin_offsetof(Smem, cwin) == R, "chunk gather addresses cwin as ring + R");

struct Ctx {
    const gc_u8 *src;
    g_u8 *dst;
    int32_t n;      // compressed size
    int32_t cap;    // dst capacity
    int32_t F;      // ring flushed up to (output position)
    int32_t Fw;     // flushed and waited for (HBM loads below this are safe)
    uint32_t dmis;  // dst address mod 16 (ring slots mirror HBM alignment)
    int32_t cbase;  // input position of cwin[0]
    int32_t bug;    // set when an internal bound trips (kernel bug guard; never expected)
};

__device__ __forceinline__ uint32_t slot(const Ctx &c, int32_t pos) { return (uint32_t)(pos + (int32_t)c.dmis) & RMASK; }

// exit table index of window position p: column-major (index-in-piece * 64 +
// piece) so the 64 lanes, one piece each, touch 64 consecutive dwords
__device__ __forceinline__ uint32_t exi(const Ctx &c, int32_t p) {
    uint32_t r = (uint32_t)(p - c.cbase);
    return (r & (P - 1)) * 64 + (r / P);
}

// ---------------------------------------------------------------------------
// staging and byte access
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cb(const Smem &s, const Ctx &c, int32_t p) {
    int32_t r = p - c.cbase;
    if ((uint32_t)r < (uint32_t)CWIN) return s.cwin[r];
    return (p >= 0 && p < c.n) ? c.src[p] : 0u;
}

// Stage input [cbase, cbase+CWIN) with 16-byte loads aligned in HBM.
__device__ __forceinline__ void stage_window(Smem &s, Ctx &c, int32_t wbase) {
    const int l = lane_id();
    const uint32_t mis = (uint32_t)(((uintptr_t)c.src + (uint32_t)wbase) & 15u);
    c.cbase = wbase - (int32_t)mis;
    for (int k = l; k < CWIN / 16; k += 64) {
        int32_t p = c.cbase + 16 * k;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < c.n) v = *(const gc_u4 *)(c.src + p);  // chunk holds at least one valid byte: same page
        *(uint4 *)(s.cwin + 16 * k) = v;
    }
    // bytes outside [0, n) must read as 0 (they are never part of a fast-path token)
    if (c.cbase < 0 || c.cbase + CWIN > c.n) {
        for (int k = l; k < CWIN; k += 64) {
            int32_t p = c.cbase + k;
            if (p >= c.n || p < 0) s.cwin[k] = 0;
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

// rest of a 255-run of match-length extension bytes (rare): next position or STOP|p
__device__ __forceinline__ uint32_t ext_tail(const Smem &s, const Ctx &c, int32_t p, int32_t q) {
    const int32_t n = c.n;
    int k = 1;
    uint32_t sv;
    do {
        sv = cb(s, c, q);
        q++;
        if (q >= n - 4 || ++k > KEXT) return STOP | (uint32_t)p;
    } while (sv == 255);
    return (uint32_t)q;
}

// next-token position only (the DP's inner step); STOP|p when not a fast-path
// token.  tb = the byte at p (from registers).  The first match-length
// extension byte is read unconditionally (no divergent loop in the common case).
__device__ __forceinline__ uint32_t next_pos(const Smem &s, const Ctx &c, int32_t p, uint32_t tb) {
    const int32_t n = c.n;
    if (p > n - 18) return STOP | (uint32_t)p;
    uint32_t ll = tb >> 4;
    if (ll == 15) return (uint32_t)parse_tok(s, c, p).nxt;
    int32_t q = p + 3 + (int32_t)ll;  // first byte after the offset (<= p + 17: staged)
    uint32_t e1 = s.cwin[q - c.cbase];
    if ((tb & 15) == 15) {
        q++;
        if (q >= n - 4) return STOP | (uint32_t)p;
        if (e1 == 255) return ext_tail(s, c, p, q);
    }
    return (uint32_t)q;
}

// ---------------------------------------------------------------------------
// output ring <-> HBM
// ---------------------------------------------------------------------------
// Write ring[F, to) to dst[F, to).  `to` is a 128-byte aligned HBM boundary
// (or the block end).  The previous flush is waited for first; Fw tracks the
// prefix whose stores are known complete.
__device__ __forceinline__ void flush(Smem &s, Ctx &c, int32_t to) {
    const int l = lane_id();
    wait_vm();
    c.Fw = c.F;
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
// whole-wave copies (serial path)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void coop_lit(Smem &s, Ctx &c, int32_t srcpos, int32_t op, int32_t len) {
    const int l = lane_id();
    for (int32_t k = 0; k < len; k += 64) {
        if (op + k - c.F >= FLUSH_T) flush_to_line(s, c, op + k);
        int32_t i = k + l;
        if (i < len) s.ring[slot(c, op + i)] = cb(s, c, srcpos + i);
    }
}

__device__ __forceinline__ void coop_match(Smem &s, Ctx &c, int32_t op, int32_t off, int32_t len) {
    const int l = lane_id();
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
// chunk gather (copy phase)
// ---------------------------------------------------------------------------
// Byte source kinds
enum { K_LDS = 0, K_GLB = 1, K_ZERO = 2, K_OWN = 3, K_PEND = 4 };

struct Chunk {
    int32_t c0;       // output position of the chunk (ring slot 256-aligned)
    uint32_t kind;    // 4 x 4-bit kinds
    uint32_t own;     // 4 x 8-bit own-byte index (K_OWN) or source dword lane (K_PEND)
    uint32_t addr[4]; // LDS byte address (K_LDS, K_PEND)
    uint32_t g[4];    // prefetched HBM byte (K_GLB)
};

__device__ __forceinline__ uint32_t umod(uint32_t a, uint32_t b) {
    // a % b for a < 2^24, 1 <= b < 2^16, via float reciprocal + fix-ups
    uint32_t q = (uint32_t)((float)a * __builtin_amdgcn_rcpf((float)b));
    int32_t r = (int32_t)a - (int32_t)(q * b);
    if (r < 0) r += (int32_t)b;
    if (r < 0) r += (int32_t)b;
    if (r >= (int32_t)b) r -= (int32_t)b;
    if (r >= (int32_t)b) r -= (int32_t)b;
    return (uint32_t)r;
}

// Assign tokens to the chunk's dwords and compute every byte's source.
// ta: token containing the chunk start (or 0 for the window's first chunk);
// returns the token containing the chunk's last byte.
__device__ __forceinline__ uint32_t chunk_assign(Smem &s, Ctx &c, Chunk &ch, int32_t c0, uint32_t ta, uint32_t T,
                                                 int32_t lo, int32_t hi) {
    const int l = lane_id();
    const int32_t cend = c0 + 256;
    const int32_t q = c0 + 4 * l;
    ch.c0 = c0;
    // HBM reads below the ring floor must see completed flush stores (never
    // taken in steady state: flushes run ~1 KiB behind, the floor is ~8 KiB back)
    need_flushed(c, cend - R);
    // token-start markers: at most one token starts in any dword (tokens are >= 4 bytes)
    uint32_t t = ta + 1 + (uint32_t)l;
    bool tv = t < T;
    int32_t ot = tv ? (int32_t)s.u.tk.o[t] : 0;
    bool inch = tv && ot < cend;
    if (inch) s.mk[(ot - c0) >> 2] = t;
    __builtin_amdgcn_wave_barrier();
    uint32_t m = s.mk[l];
    s.mk[l] = NONE;
    uint32_t mv = (m == NONE) ? 0u : m + 1;  // 1-based for the max-scan
    uint32_t incl = dpp_scan_max(mv);
    uint32_t excl = dpp_shift_up(incl, 0u);
    uint32_t prev = excl ? excl - 1 : ta;  // last token starting before this dword
    if (prev < ta) prev = ta;
    uint32_t tnext = readlane(incl, 63);
    tnext = tnext ? tnext - 1 : ta;
    if (tnext < ta) tnext = ta;
    // records of the (up to) two tokens touching this dword
    uint32_t t0 = prev, t1 = NONE;
    int32_t o1 = 0;
    if (m != NONE) {
        o1 = (int32_t)s.u.tk.o[m];
        if (o1 == q) t0 = m;
        else t1 = m;
    }
    int32_t o0 = (int32_t)s.u.tk.o[t0];
    int32_t lit0 = (int32_t)s.u.tk.lit[t0];
    uint32_t lo0 = s.u.tk.lo[t0];
    int32_t lit1 = 0;
    uint32_t lo1 = 0;
    if (t1 != NONE) {
        lit1 = (int32_t)s.u.tk.lit[t1];
        lo1 = s.u.tk.lo[t1];
    }
    const int32_t ringfloor = cend - R;
    const int32_t rdy = c0 > lo ? c0 : lo;
    uint32_t kind = 0, own = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int32_t pos = q + k;
        const bool use1 = (t1 != NONE) && pos >= o1;
        const int32_t o = use1 ? o1 : o0;
        const int32_t lit = use1 ? lit1 : lit0;
        const uint32_t lw = use1 ? lo1 : lo0;
        const int32_t ll = (int32_t)(lw & 0xFFFFu);
        const int32_t off = (int32_t)(lw >> 16);
        const int32_t ms = o + ll;
        const bool inwin = pos >= lo && pos < hi;
        const bool islit = pos < ms;
        const int32_t sp = lit + (pos - o);
        const uint32_t rl = (uint32_t)(sp - c.cbase);
        uint32_t kk = (uint32_t)(pos - ms);
        if (inwin && !islit && off != 0 && kk >= (uint32_t)off) kk = umod(kk, (uint32_t)off);
        const int32_t x = ms - off + (int32_t)kk;
        // classify (selects, not branches)
        const bool lit_lds = rl < (uint32_t)CWIN;
        const bool m_ready = x < rdy;
        const bool m_ring = x >= ringfloor;
        const bool m_own = x >= q;
        uint32_t kd = !inwin ? K_LDS
                    : islit ? (lit_lds ? K_LDS : K_GLB)
                    : off == 0 ? K_ZERO
                    : m_ready ? (m_ring ? K_LDS : K_GLB)
                    : m_own ? K_OWN : K_PEND;
        uint32_t ad = !inwin ? slot(c, pos) : islit ? (uint32_t)R + rl : slot(c, x);
        uint32_t ow = m_own ? (uint32_t)(x - q) : (uint32_t)((x - c0) >> 2);
        uint32_t gv = 0;
        if (kd == K_GLB) gv = islit ? (uint32_t)c.src[sp] : (uint32_t)c.dst[x];
        kind |= kd << (4 * k);
        own |= (ow & 0xFFu) << (8 * k);
        ch.addr[k] = ad;
        ch.g[k] = gv;
    }
    ch.kind = kind;
    ch.own = own;
    return tnext;
}

__device__ __forceinline__ uint32_t pick_own(uint32_t j, uint32_t v0, uint32_t v1, uint32_t v2) {
    return j == 0 ? v0 : (j == 1 ? v1 : v2);
}

// Produce the chunk described by ch into the ring.
__device__ __forceinline__ void chunk_write(Smem &s, Ctx &c, const Chunk &ch) {
    const int l = lane_id();
    const uint8_t *lds = (const uint8_t *)&s;
    uint32_t v[4];
    uint32_t pend = 0;  // bit k: byte k not yet known
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        uint32_t kd = (ch.kind >> (4 * k)) & 15u;
        uint32_t x = 0;
        if (kd == K_LDS) x = lds[ch.addr[k]];
        else if (kd == K_GLB) x = ch.g[k];
        else if (kd == K_PEND) pend |= 1u << k;
        v[k] = x;
    }
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        uint32_t kd = (ch.kind >> (4 * k)) & 15u;
        if (kd == K_OWN) {
            uint32_t j = (ch.own >> (8 * k)) & 0xFFu;
            v[k] = pick_own(j, v[0], v[1], v[2]);
            if (pend & (1u << j)) pend |= 1u << k;
        }
    }
    const uint32_t dslot = slot(c, ch.c0 + 4 * l);
    if (pend == 0) *(uint32_t *)(s.ring + dslot) = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
    // in-chunk dependencies: resolve in rounds (lower dwords first); every
    // round resolves at least the lowest pending dword, so <= 64 rounds
    for (int guard = 0; __ballot(pend != 0); ++guard) {
        if (guard > 64) { c.bug = 1; break; }
        uint64_t done = __ballot(pend == 0);
        uint32_t dlo = (uint32_t)done, dhi = (uint32_t)(done >> 32);
        uint32_t was = pend;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            if (pend & (1u << k)) {
                uint32_t kd = (ch.kind >> (4 * k)) & 15u;
                if (kd == K_PEND) {
                    uint32_t d = (ch.own >> (8 * k)) & 0xFFu;
                    bool ok = d < 32 ? ((dlo >> d) & 1u) : ((dhi >> (d - 32)) & 1u);
                    if (ok) {
                        v[k] = lds[ch.addr[k]];
                        pend &= ~(1u << k);
                    }
                } else {  // K_OWN waiting on an earlier byte of this dword
                    uint32_t j = (ch.own >> (8 * k)) & 0xFFu;
                    if (!(pend & (1u << j))) {
                        v[k] = pick_own(j, v[0], v[1], v[2]);
                        pend &= ~(1u << k);
                    }
                }
            }
        }
        if (pend == 0 && was != 0) *(uint32_t *)(s.ring + dslot) = v[0] | (v[1] << 8) | (v[2] << 16) | (v[3] << 24);
    }
}

// ---------------------------------------------------------------------------
// fast path: one window
// ---------------------------------------------------------------------------
__device__ __forceinline__ void window(Smem &s, Ctx &c, Ser &st, int *stopped PROF_ARG) {
    const int l = lane_id();
    const int32_t wbase = st.ip;
    const int32_t op0 = st.op;
    stage_window(s, c, wbase);
    const int32_t cbase = c.cbase;
    PSTAMP(0);

    // 1. exit DP over this lane's piece, backwards
    const int32_t plo = cbase + l * P, phi = plo + P;
    uint32_t pw[8];
    {
        uint4 a = *(const uint4 *)(s.cwin + P * l);
        uint4 b = *(const uint4 *)(s.cwin + P * l + 16);
        pw[0] = a.x; pw[1] = a.y; pw[2] = a.z; pw[3] = a.w;
        pw[4] = b.x; pw[5] = b.y; pw[6] = b.z; pw[7] = b.w;
    }
    // positions in groups of three: a token is >= 3 bytes, so every next
    // position of the group lies above it and the three exit lookups are
    // independent (one LDS round trip per group instead of per position)
#pragma unroll
    for (int g = P - 1; g >= 0; g -= 3) {
        uint32_t nx[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = g - u;
            if (i < 0) continue;
            uint32_t tb = (pw[i >> 2] >> ((i & 3) * 8)) & 0xFFu;
            nx[u] = next_pos(s, c, plo + i, tb);
        }
        uint32_t e[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = g - u;
            if (i < 0) continue;
            uint32_t x = nx[u];
            bool direct = (x & STOP) || (int32_t)x >= phi;
            uint32_t idx = direct ? (uint32_t)l : ((uint32_t)((int32_t)x - plo)) * 64 + (uint32_t)l;
            uint32_t v = s.u.ex[idx];
            e[u] = direct ? x : v;
        }
#pragma unroll
        for (int u = 0; u < 3; ++u) {
            const int i = g - u;
            if (i < 0) continue;
            s.u.ex[(uint32_t)i * 64 + (uint32_t)l] = e[u];
        }
    }
    __builtin_amdgcn_wave_barrier();
    PSTAMP(1);

    // 2. fix-up: parallel fixed-point rounds, then verify
    uint32_t E = dpp_shift_up(s.u.ex[l], (uint32_t)wbase);
    uint32_t X = 0;
    bool conv = false;
    for (int r = 0; r < FIX_ROUNDS; ++r) {
        X = ((E & STOP) || (int32_t)E >= phi) ? E : s.u.ex[exi(c, (int32_t)E)];
        uint32_t En = dpp_shift_up(X, (uint32_t)wbase);
        uint64_t chg = __ballot(En != E);
        E = En;
        if (!chg) { conv = true; break; }
    }
    uint32_t ent, efin;
    X = ((E & STOP) || (int32_t)E >= phi) ? E : s.u.ex[exi(c, (int32_t)E)];
    if (conv) {
        ent = E;
        efin = readlane(X, 63);
    } else {
        uint32_t e = (uint32_t)wbase;
        ent = STOP;
        for (int k = 0; k < 64; ++k) {
            if (l == k) ent = e;
            uint32_t Ek = readlane(E, k);
            if (e == Ek) {
                e = readlane(X, k);
            } else if (!(e & STOP) && (int32_t)e < cbase + (k + 1) * P) {
                e = uniform(s.u.ex[exi(c, (int32_t)e)]);
            }
        }
        efin = e;
    }
    PSTAMP(2);

    // 3a. walk the true chain of this piece, recording every token's fields
    int32_t tpos[TPMAX], tlit[TPMAX];
    uint32_t tlm[TPMAX], tof[TPMAX];  // ll | ml << 16 ; off | llx << 16
    uint32_t cnt = 0, olen = 0;
    int32_t stop_ip = -1;
    {
        int32_t qq = (int32_t)ent;
        bool act = !(ent & STOP) && qq < phi;
#pragma unroll
        for (int j = 0; j < TPMAX; ++j) {
            tpos[j] = qq;
            tlit[j] = 0;
            tlm[j] = 0;
            tof[j] = 0;
            if (act) {
                Tok t = parse_tok(s, c, qq);
                if ((uint32_t)t.nxt & STOP) {
                    stop_ip = qq;
                    act = false;
                } else {
                    cnt++;
                    olen += (uint32_t)(t.ll + t.ml);
                    tlit[j] = t.lit;
                    tlm[j] = (uint32_t)t.ll | ((uint32_t)t.ml << 16);
                    tof[j] = (uint32_t)t.off | ((uint32_t)t.llx << 16);
                    qq = t.nxt;
                    if (qq >= phi) act = false;
                }
            }
        }
    }
    uint32_t cinc = dpp_scan_add(cnt), oinc = dpp_scan_add(olen);
    uint32_t tbase = cinc - cnt, obase = oinc - olen;
    uint32_t ntok = readlane(cinc, 63), nout = readlane(oinc, 63);
    __builtin_amdgcn_wave_barrier();

    // 3b. emit records, with the output-side fast-loop checks
    uint32_t bad_idx = NONE;
    int32_t bad_ip = 0, bad_op = 0;
    if (stop_ip >= 0) {
        bad_idx = tbase + cnt;
        bad_ip = stop_ip;
        bad_op = op0 + (int32_t)(obase + olen);
    }
    {
        int32_t o = op0 + (int32_t)obase;
        bool act = true;
        const int32_t cap = c.cap;
#pragma unroll
        for (int j = 0; j < TPMAX; ++j) {
            if (act && (uint32_t)j < cnt) {
                int32_t ll = (int32_t)(tlm[j] & 0xFFFFu), ml = (int32_t)(tlm[j] >> 16);
                int32_t off = (int32_t)(tof[j] & 0xFFFFu);
                bool llx = (tof[j] >> 16) != 0;
                int32_t om = o + ll;
                bool bad = (llx && om > cap - 32) || (om + ml >= cap - 64) || (off > om);
                uint32_t idx = tbase + (uint32_t)j;
                if (bad) {
                    bad_idx = idx;
                    bad_ip = tpos[j];
                    bad_op = o;
                    act = false;
                } else {
                    s.u.tk.o[idx] = (uint32_t)o;
                    s.u.tk.lit[idx] = (uint32_t)tlit[j];
                    s.u.tk.lo[idx] = (uint32_t)ll | ((uint32_t)off << 16);
                    o = om + ml;
                }
            }
        }
    }
    uint32_t T = dwave_min(bad_idx);
    int32_t end_ip, end_op;
    if (T == NONE) {
        T = ntok;
        end_ip = (int32_t)efin;
        end_op = op0 + (int32_t)nout;
        *stopped = (efin & STOP) ? 1 : 0;  // (cannot be STOP without a stop token)
    } else {
        uint64_t mm = __ballot(bad_idx == T);
        int src_l = (int)__builtin_ctzll(mm);
        end_ip = (int32_t)readlane((uint32_t)bad_ip, src_l);
        end_op = (int32_t)readlane((uint32_t)bad_op, src_l);
        *stopped = 1;
    }
    __builtin_amdgcn_wave_barrier();
    PSTAMP(3);

    // 4. chunk gather over output [op0, end_op)
    if (T > 0) {
        const int32_t lo = op0, hi = end_op;
        int32_t c0 = (int32_t)(((uint32_t)op0 + c.dmis) & ~255u) - (int32_t)c.dmis;
        // two chunk descriptors alternate roles (no register copies: a copy of
        // a prefetch destination would wait for the HBM load)
        Chunk A, B;
        uint32_t ta = chunk_assign(s, c, A, c0, 0u, T, lo, hi);
        for (;;) {
            int32_t c1 = c0 + 256;
            bool more = c1 < hi;
            if (more) ta = chunk_assign(s, c, B, c1, ta, T, lo, hi);
            PSTAMP(4);
            if (c0 - c.F >= FLUSH_T) flush_to_line(s, c, c0);
            PSTAMP(7);
            chunk_write(s, c, A);
            PSTAMP(5);
            if (!more) break;
            c0 = c1;
            c1 = c0 + 256;
            more = c1 < hi;
            if (more) ta = chunk_assign(s, c, A, c1, ta, T, lo, hi);
            PSTAMP(4);
            if (c0 - c.F >= FLUSH_T) flush_to_line(s, c, c0);
            PSTAMP(7);
            chunk_write(s, c, B);
            PSTAMP(5);
            if (!more) break;
            c0 = c1;
        }
    }
    st.ip = end_ip;
    st.op = end_op;
}

__global__ __launch_bounds__(64) void lz4_decode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                       int32_t *__restrict__ ret) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    if (b >= nblk) return;
    const int l = lane_id();
    jfs_dev_block d = ((const gc_blk *)blocks)[b];
    Ctx c;
    c.src = (const gc_u8 *)d.src;
    c.dst = (g_u8 *)d.dst;
    c.n = d.src_len;
    c.cap = d.dst_cap;
    c.F = 0;
    c.Fw = 0;
    c.dmis = (uint32_t)((uintptr_t)d.dst & 15u);
    c.cbase = 0x3fffffff;
    c.bug = 0;
    int32_t result;
#ifdef JFS_PROF
    Prof pr;
    pr.start();
#endif
    s.mk[l] = NONE;
    if (d.src == nullptr || c.n < 0 || c.cap < 0) {
        result = -1;
    } else if (c.cap == 0) {
        result = (c.n == 1 && c.src[0] == 0) ? 0 : -1;
    } else if (c.n == 0) {
        result = -1;
    } else {
        Ser st;
        st.ip = 0;
        st.op = 0;
        st.fast = c.cap >= 64;
        st.ret = 0;
        int status = SER_CONT;
        for (int64_t guard = 0;; ++guard) {
            if (c.bug || guard > (int64_t)c.n + 64) { status = SER_ERR; st.ret = INT32_MIN; c.bug = 1; break; }
            int32_t ip_before = st.ip;
            if (st.fast && st.ip < c.n - 64 && st.op < c.cap - 128) {
                int stopped = 0;
                window(s, c, st, &stopped PROF_PASS);
                if (st.ip <= ip_before && !stopped) { c.bug = 2; continue; }
                if (!stopped) continue;
            }
            // the token at st.ip is not a fast-path token: take it exactly
            c.cbase = 0x3fffffff;  // staged window no longer describes st.ip
            status = ser_seq(s, c, st);
            PSTAMP(8);
            if (status != SER_CONT) break;
        }
        if (status == SER_DONE) {
            flush(s, c, st.op);
            result = st.ret;
        } else {
            result = st.ret;
        }
    }
    if (l == 0) ret[b] = result;
#ifdef JFS_PROF
    pr.stamp(9);
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
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4d::lz4_decode_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
