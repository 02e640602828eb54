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
//   2. Fix-up: one wave-uniform pass over the 64 pieces turns the window entry
//      into each piece's true entry (one LDS lookup per piece, not per token).
//   3. Each lane walks the true chain of its piece (count, then emit): wave
//      prefix sums give token indices and output offsets; tokens land in an
//      LDS table in stream order.
//   4. Copy: tokens are copied in groups of up to 64 (lane = token) into an
//      LDS output ring.  Literals first, then matches in rounds: a match runs
//      once its source lies below the high-water mark (first unresolved match
//      start).  Long tokens are copied by the whole wave.  The ring is
//      streamed to HBM with 16-byte stores at 128-byte aligned boundaries;
//      matches reaching farther back than the ring read HBM.
//   5. Everything the fast path does not cover (the last bytes of input /
//      output, malformed input, very long length fields) runs through an
//      exact, wave-uniform restatement of the liblz4 1.9.3 state machine.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4d {

constexpr int CW = 2048;               // compressed window bytes handled per pass
constexpr int MARGIN = 64;             // lookahead staged beyond the window
constexpr int CWIN = CW + MARGIN + 16; // LDS staging (16-byte aligned source chunks)
constexpr int P = 32;                  // bytes per lane piece (64 lanes x 32 = CW)
constexpr int R = 8192;                // output ring bytes
constexpr int RMASK = R - 1;
constexpr int TMAX = CW / 3 + 2;       // max tokens in a window (interior token >= 3 bytes)
constexpr uint32_t STOP = 0x80000000u;
constexpr int KEXT = 64;               // max 255-extension bytes handled by the fast path
constexpr int SHORT_T = 64;            // tokens with ll or ml above this are copied by the whole wave
constexpr int GSPAN = 1536;            // max output span of one token group
constexpr int FLUSH_T = 1024;          // flush the ring when this many bytes are pending
constexpr int RING_BACK = R - GSPAN;   // sources >= group start - RING_BACK are read from the ring

struct Smem {
    alignas(16) uint8_t ring[R];
    alignas(16) uint8_t cwin[CWIN];
    union {
        uint32_t ex[CW];
        struct {
            uint32_t lit_src[TMAX + 1];
            uint32_t out_pos[TMAX + 1];
            uint32_t offml[TMAX + 1];  // off << 16 | ml
        } tk;
    } u;
};

struct Ctx {
    const uint8_t *src;
    uint8_t *dst;
    int32_t n;      // compressed size
    int32_t cap;    // dst capacity
    int32_t F;      // ring flushed up to (output position)
    int32_t Fw;     // flushed and waited for (global loads below this are safe)
    uint32_t dmis;  // dst address mod 16 (ring slots mirror HBM alignment)
    int32_t cbase;  // output position -> not used; window staging base (input position)
};

__device__ __forceinline__ uint32_t slot(const Ctx &c, int32_t pos) { return (uint32_t)(pos + c.dmis) & RMASK; }

// ---------------------------------------------------------------------------
// staging and byte access
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t cb(const Smem &s, const Ctx &c, int32_t p) {
    int32_t r = p - c.cbase;
    if ((uint32_t)r < (uint32_t)CWIN) return s.cwin[r];
    return (p >= 0 && p < c.n) ? c.src[p] : 0u;
}

// Stage input [cbase, cbase+CWIN) with 16-byte loads aligned in HBM.
__device__ void stage_window(Smem &s, Ctx &c, int32_t wbase) {
    const int l = lane_id();
    const uint32_t mis = (uint32_t)(((uintptr_t)c.src + (uint32_t)wbase) & 15u);
    c.cbase = wbase - (int32_t)mis;
    for (int k = l; k < CWIN / 16; k += 64) {
        int32_t p = c.cbase + 16 * k;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (p < c.n) v = *(const uint4 *)(c.src + p);  // chunk holds at least one valid byte: same page
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

// ---------------------------------------------------------------------------
// output ring <-> HBM
// ---------------------------------------------------------------------------
// Write ring[F, to) to dst[F, to).  `to` is a 128-byte aligned HBM boundary
// (or the block end).  The previous flush is waited for first; Fw tracks the
// prefix whose stores are known complete.
__device__ void flush(Smem &s, Ctx &c, int32_t to) {
    const int l = lane_id();
    wait_vm();
    c.Fw = c.F;
    int32_t F = c.F;
    if (to <= F) return;
    // head bytes up to the first 16-byte aligned HBM address
    int32_t a = F + (int32_t)((16u - ((c.dmis + (uint32_t)F) & 15u)) & 15u);
    if (a > to) a = to;
    if (l < a - F) c.dst[F + l] = s.ring[slot(c, F + l)];
    int32_t b = a + ((to - a) & ~15);
    for (int32_t x = a + 16 * l; x < b; x += 1024) {
        uint4 v = *(const uint4 *)(s.ring + slot(c, x));
        *(uint4 *)(c.dst + x) = v;
    }
    if (l < to - b) c.dst[b + l] = s.ring[slot(c, b + l)];
    c.F = to;
}

// flush everything below `hi` rounded down to a 128-byte HBM line boundary
__device__ __forceinline__ void flush_to_line(Smem &s, Ctx &c, int32_t hi) {
    int32_t to = (int32_t)(((uint32_t)hi + c.dmis) & ~127u) - (int32_t)c.dmis;
    if (to > c.F) flush(s, c, to);
}

// read an already-produced output byte x (x < hi, the next byte to be written)
// ringfloor: smallest position still guaranteed to be held by the ring.
__device__ __forceinline__ uint32_t out_byte(const Smem &s, const Ctx &c, int32_t x, int32_t ringfloor) {
    if (x >= ringfloor) return s.ring[slot(c, x)];
    return c.dst[x];  // flushed (x < Fw, 128-byte line aligned): plain load is coherent
}

// make sure any HBM read of positions < lim is ordered after the flush stores
__device__ __forceinline__ void need_flushed(Ctx &c, int32_t lim) {
    if (lim > c.Fw) {
        wait_vm();
        c.Fw = c.F;
    }
}

// ---------------------------------------------------------------------------
// whole-wave copies (long tokens, serial path)
// ---------------------------------------------------------------------------
__device__ void coop_lit(Smem &s, Ctx &c, int32_t srcpos, int32_t op, int32_t len) {
    const int l = lane_id();
    for (int32_t k = 0; k < len; k += 64) {
        if (op + k - c.F >= FLUSH_T) flush_to_line(s, c, op + k);
        int32_t i = k + l;
        if (i < len) s.ring[slot(c, op + i)] = cb(s, c, srcpos + i);
    }
}

__device__ void coop_match(Smem &s, Ctx &c, int32_t op, int32_t off, int32_t len) {
    const int l = lane_id();
    // position of byte i's source: op - off + (off >= 64 ? i : i mod off)
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

// read_variable_length: 0 ok, 1 initial error, 2 loop error
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

__device__ int ser_seq(Smem &s, Ctx &c, Ser &st) {
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
        st.ip = ip; st.op = op;
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
            st.ip = ip; st.op = op;
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
        st.ip = ip; st.op = op; st.ret = op;
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
    st.ip = ip; st.op = op;
    return SER_CONT;
err:
    st.ip = ip;
    st.ret = -ip - 1;
    return SER_ERR;
}

// ---------------------------------------------------------------------------
// fast path: one window
// ---------------------------------------------------------------------------
// Returns number of tokens copied; updates st.ip / st.op.  *stopped = 1 when
// the window ended at a token the fast path cannot take (serial takes it).
__device__ void window(Smem &s, Ctx &c, Ser &st, int *stopped) {
    const int l = lane_id();
    const int32_t wbase = st.ip;
    const int32_t op0 = st.op;
    stage_window(s, c, wbase);

    // 1. exit DP over this lane's piece, backwards
    const int32_t plo = wbase + l * P, phi = plo + P;
    for (int i = P - 1; i >= 0; --i) {
        int32_t p = plo + i;
        Tok t = parse_tok(s, c, p);
        uint32_t e;
        if ((uint32_t)t.nxt & STOP) e = (uint32_t)t.nxt;
        else if (t.nxt >= phi) e = (uint32_t)t.nxt;
        else e = s.u.ex[t.nxt - wbase];
        s.u.ex[p - wbase] = e;
    }
    __builtin_amdgcn_wave_barrier();

    // 2. wave-uniform fix-up: true entry of every piece
    uint32_t e = (uint32_t)wbase;
    uint32_t ent = STOP;
    for (int k = 0; k < 64; ++k) {
        if (l == k) ent = e;
        if (e & STOP) continue;
        if ((int32_t)e < wbase + (k + 1) * P) e = uniform(s.u.ex[(int32_t)e - wbase]);
    }

    // 3a. count walk
    uint32_t cnt = 0, olen = 0;
    int32_t stop_ip = -1;
    {
        int32_t q = (int32_t)ent;
        if (!(ent & STOP)) {
            while (q < phi) {
                Tok t = parse_tok(s, c, q);
                if ((uint32_t)t.nxt & STOP) { stop_ip = q; break; }
                cnt++;
                olen += (uint32_t)(t.ll + t.ml);
                q = t.nxt;
            }
        }
    }
    uint32_t ntok, nout;
    uint32_t tbase = wave_scan_excl(cnt, &ntok);
    uint32_t obase = wave_scan_excl(olen, &nout);

    // 3b. emit walk with the output-side fast-loop checks
    uint32_t bad_idx = 0xFFFFFFFFu;  // first token index this lane cannot take
    int32_t bad_ip = 0, bad_op = 0;
    if (stop_ip >= 0) { bad_idx = tbase + cnt; bad_ip = stop_ip; bad_op = op0 + (int32_t)(obase + olen); }
    __builtin_amdgcn_wave_barrier();
    {
        int32_t q = (int32_t)ent;
        uint32_t j = tbase;
        int32_t o = op0 + (int32_t)obase;
        for (uint32_t k = 0; k < cnt; ++k) {
            Tok t = parse_tok(s, c, q);
            int32_t om = o + t.ll;
            bool bad = (t.llx && o + t.ll > c.cap - 32) || (om + t.ml >= c.cap - 64) || (t.off > om);
            if (bad) { bad_idx = j; bad_ip = q; bad_op = o; break; }
            s.u.tk.lit_src[j] = (uint32_t)t.lit;
            s.u.tk.out_pos[j] = (uint32_t)o;
            s.u.tk.offml[j] = ((uint32_t)t.off << 16) | (uint32_t)t.ml;
            j++;
            o = om + t.ml;
            q = t.nxt;
        }
    }
    uint32_t T = wave_min(bad_idx);
    int32_t end_ip, end_op;
    if (T == 0xFFFFFFFFu) {
        T = ntok;
        end_ip = (int32_t)(e & ~STOP);  // e is not STOP here
        end_op = op0 + (int32_t)nout;
        *stopped = 0;
        if (e & STOP) {  // cannot happen without a stop token; be safe
            *stopped = 1;
        }
    } else {
        uint64_t m = __ballot(bad_idx == T);
        int src_l = (int)__builtin_ctzll(m);
        end_ip = (int32_t)lane_read((uint32_t)bad_ip, src_l);
        end_op = (int32_t)lane_read((uint32_t)bad_op, src_l);
        *stopped = 1;
    }
    if (l == 0) s.u.tk.out_pos[T] = (uint32_t)end_op;
    __builtin_amdgcn_wave_barrier();

    // 4. copy tokens [0, T)
    uint32_t j = 0;
    while (j < T) {
        uint32_t idx = j + (uint32_t)l;
        bool v = idx < T;
        int32_t o = 0, o1 = 0, off = 0, ml = 0, lit = 0;
        if (v) {
            o = (int32_t)s.u.tk.out_pos[idx];
            o1 = (int32_t)s.u.tk.out_pos[idx + 1];
            uint32_t w = s.u.tk.offml[idx];
            off = (int32_t)(w >> 16);
            ml = (int32_t)(w & 0xFFFFu);
            lit = (int32_t)s.u.tk.lit_src[idx];
        }
        int32_t ll = o1 - o - ml;
        int32_t o0 = (int32_t)uniform((uint32_t)o);  // lane 0 holds token j
        bool fit = v && ll <= SHORT_T && ml <= SHORT_T && (o1 - o0) <= GSPAN;
        uint64_t nf = __ballot(!fit);
        int g = nf ? (int)__builtin_ctzll(nf) : 64;
        if (c.F + FLUSH_T <= o0) flush_to_line(s, c, o0);
        if (g == 0) {
            // long token j: whole-wave copy
            int32_t ulit = (int32_t)uniform((uint32_t)lit);
            int32_t ull = (int32_t)uniform((uint32_t)ll);
            int32_t uoff = (int32_t)uniform((uint32_t)off);
            int32_t uml = (int32_t)uniform((uint32_t)ml);
            coop_lit(s, c, ulit, o0, ull);
            coop_match(s, c, o0 + ull, uoff, uml);
            j += 1;
            continue;
        }
        bool act = l < g;
        // literals
        uint32_t maxll = wave_max(act ? (uint32_t)ll : 0u);
        for (uint32_t i = 0; i < maxll; ++i) {
            if (act && (int32_t)i < ll) s.ring[slot(c, o + (int32_t)i)] = (uint8_t)cb(s, c, lit + (int32_t)i);
        }
        // matches: multi-round resolution
        int32_t om = o + ll;
        int32_t sp = om - off;
        const int32_t ringfloor = o0 - RING_BACK;
        bool needg = act && off > 0 && sp < ringfloor;
        if (__ballot(needg)) need_flushed(c, ringfloor);
        bool unres = act;
        while (__ballot(unres)) {
            uint32_t hwm = wave_min(unres ? (uint32_t)om : 0xFFFFFFFFu);
            int32_t need = sp + (ml < off ? ml : off);
            bool rdy = unres && (off == 0 || need <= (int32_t)hwm);
            uint32_t maxml = wave_max(rdy ? (uint32_t)ml : 0u);
            for (uint32_t i = 0; i < maxml; ++i) {
                if (rdy && (int32_t)i < ml) {
                    uint32_t b = 0;
                    if (off > 0) b = out_byte(s, c, sp + (int32_t)i, ringfloor);
                    s.ring[slot(c, om + (int32_t)i)] = (uint8_t)b;
                }
            }
            unres = unres && !rdy;
        }
        j += (uint32_t)g;
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
    jfs_dev_block d = blocks[b];
    Ctx c;
    c.src = d.src;
    c.dst = d.dst;
    c.n = d.src_len;
    c.cap = d.dst_cap;
    c.F = 0;
    c.Fw = 0;
    c.dmis = (uint32_t)((uintptr_t)d.dst & 15u);
    c.cbase = 0x7fffffff;
    int32_t result;
    if (d.src == nullptr || c.n < 0 || c.cap < 0) {
        result = -1;
    } else if (c.cap == 0) {
        result = (c.n == 1 && d.src[0] == 0) ? 0 : -1;
    } else if (c.n == 0) {
        result = -1;
    } else {
        Ser st;
        st.ip = 0;
        st.op = 0;
        st.fast = c.cap >= 64;
        st.ret = 0;
        int status = SER_CONT;
        for (;;) {
            if (st.fast && st.ip < c.n - 64 && st.op < c.cap - 128) {
                int stopped = 0;
                window(s, c, st, &stopped);
                if (!stopped) continue;
            }
            // the token at st.ip is not a fast-path token: take it exactly
            c.cbase = 0x7fffffff;  // staged window no longer describes st.ip
            status = ser_seq(s, c, st);
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
}

}  // namespace lz4d
}  // namespace jfs

extern "C" int jfs_launch_lz4_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    if (nblk <= 0) return 0;
    hipLaunchKernelGGL(jfs::lz4d::lz4_decode_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
