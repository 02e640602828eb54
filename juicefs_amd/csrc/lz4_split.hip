// LZ4 block decode for SMALL batches: every block is spread over the whole
// GPU instead of one workgroup (lz4_decode.hip).  This is the latency path of
// the one-call API: cachedStore.load (pkg/chunk/cached_store.go:755-823)
// decodes exactly one 4 MiB block per cache miss, and one workgroup's serial
// token chain takes ~21 ms on it; here a lone block takes a few hundred
// microseconds of kernel time.
//
// Parallel formulation of LZ4_decompress_safe (the C routine lz4.DecompressSafe
// reaches, compress.go:120-125), in eight steps, all on one stream:
//   plan     per-block scratch offsets and segment counts (one tiny kernel);
//   spec     the compressed stream is cut into SEG-byte segments, one lane
//            each; a lane walks the token chain from its segment's first byte
//            (a guess: that byte need not start a token), marks every chain
//            position in a bitmap and records where the chain leaves;
//   fix      repeated rounds: a lane walks the chain from its segment's
//            current entry until it meets a marked position (the two chains
//            have merged, so its exit is the speculative one) or leaves the
//            segment; a changed exit becomes the next segment's entry.  A round
//            that changes nothing proves every entry is the true one (entry 0
//            is 0, and each exit is the chain function of its entry);
//   count    output bytes of each segment's true tokens;
//   scan     exclusive prefix sum per block -> output offset of each segment;
//   emit     each lane walks its true tokens again, checks liblz4's
//            acceptance conditions (below) and writes the block's ORIGIN map:
//            org[p] = -(input position + 1) for a literal byte, else the output
//            position it copies (op - off + i mod off, so overlapped matches
//            point before the match);
//   jump     pointer jumping over org (in place; every pointer only moves to
//            an ancestor) until every entry is a literal: O(log chain) rounds;
//   gather   dst[p] = src[-org[p] - 1].
// Any block that this formulation does not cover EXACTLY -- a fix-up or jump
// that did not converge in its rounds, or a token that fails one of the
// conditions below -- is flagged and re-run by the exact one-workgroup kernel
// (lz4_decode.hip), which reproduces liblz4 1.9.3 return values on every
// input.  The conditions are sufficient for LZ4_decompress_safe to accept the
// stream with standard semantics (oracle/lz4_oracle.c, the liblz4 1.9.3 check
// order): for every sequence but the last, literal-length bytes end before
// iend-14, literals end at or before iend-8 and oend-12, 1 <= offset <= bytes
// produced, match-length bytes end before iend-4, the match ends at or before
// oend-5; the last sequence is literals only, ends exactly at iend and within
// oend (literal-length bytes before iend-14).  Encoder output always meets
// them; anything else takes the exact path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace lz4s {

constexpr int SEG = JFS_LZ4_SPLIT_SEG;  // compressed bytes per segment (one lane)
constexpr int FIX_ROUNDS = 6;
constexpr int JUMP_ROUNDS = 12;
constexpr int HOPS = 6;  // pointer hops per entry per jump round
constexpr int T = 256;   // threads per workgroup

struct SBlock {
    const uint8_t *src;
    uint8_t *dst;
    int32_t n, cap;
    int32_t seg0, nseg;
    int64_t bits_off;  // dwords into the bitmap area
    int64_t org_off;   // entries into the origin area (multiple of 4)
};

struct BStat {
    int32_t bad, last_ok, total, todo;
    int32_t unsettled;  // the gather met an entry that is not a literal yet
    int32_t fix[FIX_ROUNDS];
    int32_t jmp[JUMP_ROUNDS];
};

struct Scratch {
    SBlock *blk;
    BStat *st;
    int32_t *spec_exit, *entry, *cnt;
    uint32_t *bits;
    int32_t *org;
};

// one token at x (x < n): next token position, output bytes, and the fields
// the acceptance conditions need.  A token whose literals reach n is the last.
// 32-bit positions and lengths (the plan sends blocks with n or cap >= 2^30 to
// the exact kernel): the wave-per-segment emit parses in scalar registers, and
// 64-bit fields cost it two scalar ops per add and a VALU round trip per
// compare.  A length field stops growing at 2^30: such a token ends past n
// (or its match past cap) either way, so it is rejected as before.
constexpr int32_t LEN_CAP = 1 << 30;
struct Tok {
    uint32_t tok;    // the token byte
    int32_t lenip;   // input position after the literal-length bytes
    int32_t ll;      // literal length
    int32_t lit_end; // lenip + ll
    int32_t next;    // next token (n for the last token)
    int32_t mlip;    // input position after the match-length bytes
    int32_t ml;      // match length (0 for the last token)
    int32_t off;
    bool last, cut;  // cut: the stream ends inside the token's header fields
};

template <class RD>
__device__ __forceinline__ Tok parse_rd(RD s, int32_t n, int32_t x, bool want_off) {
    Tok t;
    t.cut = false;
    t.off = 0;
    t.ml = 0;
    const uint32_t tok = s[x];
    t.tok = tok;
    int32_t ip = x + 1;
    int32_t ll = (int32_t)(tok >> 4);
    if (ll == 15) {
        uint32_t b;
        do {
            if (ip >= n) {
                t.cut = true;
                break;
            }
            b = s[ip++];
            ll += (int32_t)b;
        } while (b == 255 && ll < LEN_CAP);
    }
    t.lenip = ip;
    t.ll = ll;
    t.lit_end = ip + ll;
    t.mlip = ip;
    if (t.cut || t.lit_end >= n) {
        t.last = true;
        t.next = n;
        return t;
    }
    t.last = false;
    int32_t q = t.lit_end;
    if (q + 2 > n) {
        t.cut = true;
        t.next = n;
        return t;
    }
    if (want_off) t.off = (int32_t)s[q] | ((int32_t)s[q + 1] << 8);
    q += 2;
    int32_t ml = (int32_t)(tok & 15);
    if (ml == 15) {
        uint32_t b;
        do {
            if (q >= n) {
                t.cut = true;
                break;
            }
            b = s[q++];
            ml += (int32_t)b;
        } while (b == 255 && ml < LEN_CAP);
    }
    t.mlip = q;
    t.ml = ml + 4;
    t.next = q;
    return t;
}
__device__ __forceinline__ Tok parse(const gc_u8 *s, int32_t n, int32_t x, bool want_off) {
    return parse_rd(s, n, x, want_off);
}

// block of global segment g (blocks are few: linear search over the seg0's)
// the block holding segment g: the last b with seg0 <= g (binary search)
__device__ __forceinline__ int block_of(const SBlock *blk, int nb, int g) {
    int lo = 0, hi = nb - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (blk[mid].seg0 <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// The scratch and the grids were sized on the host from its own (src_len,
// dst_cap) copies (nseg_all, max_cap, norg_all).  A block whose device
// descriptor asks for more than that budget leaves -- it would overrun the
// segment or origin-map scratch -- is planned empty and marked bad, so the
// exact one-workgroup kernel decodes it from its descriptor instead.
__global__ void plan_kernel(const jfs_dev_block *__restrict__ desc, int nb, Scratch sc, int64_t nseg_all,
                            int64_t max_cap, int64_t norg_all) {
    for (int i = threadIdx.x; i < nb * (int)(sizeof(BStat) / 4); i += blockDim.x) ((int32_t *)sc.st)[i] = 0;
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        int32_t seg = 0;
        int64_t bits = 0, org = 0;
        for (int b = 0; b < nb; b++) {
            const jfs_dev_block d = ((const gc_blk *)desc)[b];
            SBlock &s = sc.blk[b];
            s.src = d.src;
            s.dst = d.dst;
            s.n = d.src_len > 0 ? d.src_len : 0;
            s.cap = d.dst_cap > 0 ? d.dst_cap : 0;
            const int64_t ns = (s.n + SEG - 1) / SEG, no = ((int64_t)s.cap + 3) & ~3ll;
            if (s.cap > max_cap || seg + ns > nseg_all || org + no > norg_all || s.n >= LEN_CAP || s.cap >= LEN_CAP) {
                s.n = 0;
                s.cap = 0;
                sc.st[b].bad = 1;
            }
            s.seg0 = seg;
            s.nseg = (s.n + SEG - 1) / SEG;
            s.bits_off = bits;
            s.org_off = org;
            seg += s.nseg;
            bits += (int64_t)s.nseg * (SEG / 32);
            org += ((int64_t)s.cap + 3) & ~3ll;
        }
    }
}

__global__ __launch_bounds__(T) void spec_kernel(int nb, int nseg_all, Scratch sc) {
    const int g = blockIdx.x * T + threadIdx.x;
    if (g >= nseg_all) return;
    const int b = block_of(sc.blk, nb, g);
    const SBlock B = sc.blk[b];
    const gc_u8 *s = (const gc_u8 *)B.src;
    const int32_t n = B.n, k = g - B.seg0;
    const int32_t s0 = k * SEG, s1 = s0 + SEG < n ? s0 + SEG : n;
    uint32_t m[SEG / 32];
#pragma unroll
    for (int w = 0; w < SEG / 32; w++) m[w] = 0;
    int32_t x = s0;
    while (x < s1) {
        const uint32_t rel = (uint32_t)(x - s0), w = rel >> 5, bit = 1u << (rel & 31);
#pragma unroll
        for (int i = 0; i < SEG / 32; i++) m[i] |= (w == (uint32_t)i) ? bit : 0u;
        x = parse(s, n, x, false).next;
    }
    g_u32 *bits = (g_u32 *)(sc.bits + B.bits_off + k * (SEG / 32));
#pragma unroll
    for (int i = 0; i < SEG / 32; i++) bits[i] = m[i];
    const int32_t ex = x < n ? x : n;
    sc.spec_exit[g] = ex;
    if (k + 1 < B.nseg) sc.entry[g + 1] = ex;
    if (k == 0) sc.entry[g] = 0;
}

// exit of segment (s0, s1) entered at x: walk until the chain meets a marked
// position (then it is the speculative chain, whose exit is known) or leaves
__device__ __forceinline__ int32_t seg_exit(const gc_u8 *s, int32_t n, int32_t s0, int32_t s1, int32_t x,
                                           const gc_u32 *bits, int32_t spec_ex) {
    while (x < s1) {
        const uint32_t rel = (uint32_t)(x - s0);
        if ((bits[rel >> 5] >> (rel & 31)) & 1u) return spec_ex;
        x = parse(s, n, x, false).next;
    }
    return x < n ? x : n;
}

// One fix-up round.  Inside a workgroup the segments' entries live in LDS and
// the workgroup iterates to its own fixed point (a token that spans several
// segments, or a speculative chain that never merged, moves the next entry;
// every iteration settles at least the lowest unsettled lane).  Only a changed
// entry that crosses into the next workgroup needs another round, so rounds
// count workgroup-boundary cascades, not segments.
__global__ __launch_bounds__(T) void fix_kernel(int nb, int nseg_all, Scratch sc, int round) {
    __shared__ int32_t ent[T];
    const int t = threadIdx.x;
    const int g = blockIdx.x * T + t;
    const bool valid = g < nseg_all;
    int b = 0;
    SBlock B{};
    int32_t k = 0;
    bool active = false;
    if (valid) {
        b = block_of(sc.blk, nb, g);
        B = sc.blk[b];
        k = g - B.seg0;
        active = k + 1 < B.nseg && !(round > 0 && !sc.st[b].fix[round - 1]);
    }
    const int32_t e0 = valid ? sc.entry[g] : 0;
    ent[t] = e0;
    const gc_u8 *s = (const gc_u8 *)B.src;
    const int32_t n = B.n, s0 = k * SEG, s1 = s0 + SEG < n ? s0 + SEG : n;
    const gc_u32 *bits = (const gc_u32 *)(sc.bits + B.bits_off + k * (SEG / 32));
    const int32_t spec_ex = active ? sc.spec_exit[g] : 0;
    int32_t last_in = -1, ex = -1;
    __syncthreads();
    for (int it = 0; it <= T; it++) {
        int changed = 0;
        if (active) {
            const int32_t e = ent[t];
            if (e != last_in) {
                last_in = e;
                ex = seg_exit(s, n, s0, s1, e, bits, spec_ex);
                if (t + 1 < T && ent[t + 1] != ex) {
                    ent[t + 1] = ex;
                    changed = 1;
                }
            }
        }
        if (!__syncthreads_or(changed)) break;
    }
    if (valid && t > 0 && ent[t] != e0) sc.entry[g] = ent[t];
    if (active && t == T - 1 && sc.entry[g + 1] != ex) {  // the next workgroup's first entry
        sc.entry[g + 1] = ex;
        sc.st[b].fix[round] = 1;
    }
}

__global__ __launch_bounds__(T) void count_kernel(int nb, int nseg_all, Scratch sc) {
    const int g = blockIdx.x * T + threadIdx.x;
    if (g >= nseg_all) return;
    const int b = block_of(sc.blk, nb, g);
    if (sc.st[b].fix[FIX_ROUNDS - 1]) return;  // did not converge: exact path
    const SBlock B = sc.blk[b];
    const gc_u8 *s = (const gc_u8 *)B.src;
    const int32_t n = B.n, k = g - B.seg0;
    const int32_t s0 = k * SEG, s1 = s0 + SEG < n ? s0 + SEG : n;
    int32_t x = sc.entry[g];
    int64_t c = 0;
    while (x < s1) {
        const Tok t = parse(s, n, x, false);
        c += (int64_t)t.ll + t.ml;
        if (c > B.cap) break;
        x = t.next;
    }
    sc.cnt[g] = (int32_t)(c <= B.cap ? c : (int64_t)B.cap + 1);
}

// one workgroup per block: cnt -> exclusive output offsets, block total
__global__ __launch_bounds__(T) void scan_kernel(Scratch sc) {
    const int b = blockIdx.x;
    const SBlock B = sc.blk[b];
    BStat &st = sc.st[b];
    if (st.fix[FIX_ROUNDS - 1]) return;
    __shared__ int64_t part[T];
    const int per = (B.nseg + T - 1) / T, t = threadIdx.x;
    const int i0 = B.seg0 + t * per, i1 = min(i0 + per, B.seg0 + B.nseg);
    int64_t a = 0;
    for (int i = i0; i < i1; i++) a += sc.cnt[i];
    part[t] = a;
    __syncthreads();
    for (int o = 1; o < T; o <<= 1) {
        const int64_t y = t >= o ? part[t - o] : 0;
        __syncthreads();
        part[t] += y;
        __syncthreads();
    }
    int64_t run = part[t] - a;
    for (int i = i0; i < i1; i++) {
        const int64_t c = sc.cnt[i];
        sc.cnt[i] = (int32_t)(run < B.cap ? run : B.cap);
        run += c;
    }
    if (t == T - 1) {
        if (part[t] > B.cap || B.n == 0 || B.cap == 0) st.bad = 1;
        st.total = (int32_t)(part[t] < B.cap ? part[t] : B.cap);
    }
}

// the token checks the exact decoder makes (the emit keeps a token only if
// it would run it the same way)
__device__ __forceinline__ bool tok_ok(uint32_t tok, const Tok &t, int32_t n, int32_t op, int32_t cap) {
    // (op <= cap < 2^30 and every length < 2^30 + 2^8: no sum below overflows;
    // the last is evaluated only once op + ll <= cap - 12 holds)
    // literal-length bytes: liblz4 stops reading them (a "loop error" it
    // ignores) once its input position reaches iend-15 after a 255 byte;
    // lenip < iend-14 means the terminator was read before that point
    bool ok = !t.cut && ((tok >> 4) != 15 || t.lenip < n - 14);
    if (t.last) {
        ok = ok && t.lit_end == n && op + t.ll <= cap;
    } else {
        ok = ok && t.lit_end <= n - 8 && op + t.ll <= cap - 12 && t.off >= 1 && t.off <= op + t.ll &&
             ((tok & 15) != 15 || t.mlip < n - 4) && op + t.ll + t.ml <= cap - 5;
    }
    return ok;
}

// One WAVE per segment: the segment's true tokens are parsed wave-uniformly
// and each token's origin run is written by the whole wave (consecutive
// entries per lane: coalesced stores).  (One thread per segment wrote ~2 KB
// of scattered 16-byte stores each: 147 us of a lone 4 MiB block's 426.)
constexpr int EWV = T / 64;  // segments per workgroup
constexpr int ESTG = 1024;   // compressed bytes staged per segment (its tokens' fields, mostly)
constexpr int64_t EMIT_WAVE_MAX = 65536;  // segments (about 4 blocks of 4 MiB text)
__global__ __launch_bounds__(T) void emit_kernel(int nb, int nseg_all, Scratch sc) {
    __shared__ alignas(16) uint8_t stg[EWV][ESTG];
    const int l = lane_id();
    const int g = (int)uniform((uint32_t)(blockIdx.x * EWV + (threadIdx.x >> 6)));
    if (g >= nseg_all) return;
    const int b = (int)uniform((uint32_t)block_of(sc.blk, nb, g));
    BStat &st = sc.st[b];
    if (st.fix[FIX_ROUNDS - 1] || st.bad) return;
    const SBlock B = sc.blk[b];
    const gc_u8 *s = (const gc_u8 *)(((uint64_t)uniform((uint32_t)((uint64_t)(uintptr_t)B.src >> 32)) << 32) |
                                     uniform((uint32_t)(uintptr_t)B.src));
    g_u32 *org = (g_u32 *)(sc.org + B.org_off);
    const int32_t n = (int32_t)uniform((uint32_t)B.n), cap = (int32_t)uniform((uint32_t)B.cap),
                  k = g - (int32_t)uniform((uint32_t)B.seg0);
    const int32_t s0 = k * SEG, s1 = s0 + SEG < n ? s0 + SEG : n;
    int32_t x = (int32_t)uniform((uint32_t)sc.entry[g]), op = (int32_t)uniform((uint32_t)sc.cnt[g]);
    // the parse reads the segment's bytes from LDS (one wave-uniform LDS round
    // trip per field instead of an L2 one); bytes past the staging from HBM
    uint8_t *buf = stg[threadIdx.x >> 6];
    const uintptr_t a0 = ((uintptr_t)(s + s0)) & ~(uintptr_t)15, aend = (uintptr_t)(s + n);
    {
        const uintptr_t a = a0 + 16u * (uint32_t)l;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (a < aend) v = *(const gc_u4 *)a;  // (an aligned chunk holding a valid byte: same page)
        *(uint4 *)(buf + 16 * l) = v;
        __builtin_amdgcn_wave_barrier();
    }
    struct Rd {
        const gc_u8 *s;
        const uint8_t *buf;
        int32_t A;  // stream position of buf[0] (a0 - s: s0 less its misalignment)
        __device__ uint32_t operator[](int32_t p) const {  // (p wave-uniform: scalar branch)
            const uint32_t r = (uint32_t)(p - A);
            uint32_t v;
            if (r < (uint32_t)ESTG) v = buf[r];
            else v = s[p];
            return uniform(v);
        }
    } rd{s, buf, s0 - (int32_t)((uintptr_t)(s + s0) & 15u)};
    while (x < s1) {
        const Tok t = parse_rd(rd, n, x, true);
        const bool ok = tok_ok(t.tok, t, n, op, cap);
        if (!ok) {
            if (l == 0) st.bad = 1;
            return;
        }
        const uint32_t v0 = (uint32_t)(-(t.lenip) - 1);  // literal entry i = v0 - i
        const int32_t ll = t.ll, ml = t.ml;
        for (int32_t i = l; i < ll; i += 64) org[op + i] = v0 - (uint32_t)i;
        op += t.ll;
        if (t.last) {
            if (l == 0) st.last_ok = 1;
            return;
        }
        // match entry i = op - off + (i mod off): overlapped matches point before the match
        const int32_t base = op - t.off;
        const uint32_t off = (uint32_t)t.off;
        if (off >= (uint32_t)ml) {  // no overlap (most matches): no modulo
            for (int32_t i = l; i < ml; i += 64) org[op + i] = (uint32_t)(base + i);
        } else {
            for (int32_t i = l; i < ml; i += 64) {
                const uint32_t ui = (uint32_t)i;
                org[op + i] = (uint32_t)(base + (ui < off ? ui : ui % off));
            }
        }
        op += t.ml;
        x = t.next;
    }
}

// One THREAD per segment (large batches: 64 segments per wave do the most
// work per instruction; the wave form above wins only while the segments are
// too few to fill the GPU -- a 16-block chunk ran 20 % slower in it).
__global__ __launch_bounds__(T) void emit_thread_kernel(int nb, int nseg_all, Scratch sc) {
    const int g = blockIdx.x * T + threadIdx.x;
    if (g >= nseg_all) return;
    const int b = block_of(sc.blk, nb, g);
    BStat &st = sc.st[b];
    if (st.fix[FIX_ROUNDS - 1] || st.bad) return;
    const SBlock B = sc.blk[b];
    const gc_u8 *s = (const gc_u8 *)B.src;
    g_u32 *org = (g_u32 *)(sc.org + B.org_off);
    const int32_t n = B.n, cap = B.cap, k = g - B.seg0;
    const int32_t s0 = k * SEG, s1 = s0 + SEG < n ? s0 + SEG : n;
    int32_t x = sc.entry[g], op = sc.cnt[g];
    while (x < s1) {
        const Tok t = parse(s, n, x, true);
        const bool ok = tok_ok(t.tok, t, n, op, cap);
        if (!ok) {
            st.bad = 1;
            return;
        }
        // origin entries, 16-byte stores where the run is 4-aligned (the
        // area starts 16-byte aligned: org_off is a multiple of 4 entries)
        {
            const uint32_t v0 = (uint32_t)(-(t.lenip) - 1);  // entry i = v0 - i
            int32_t i = 0;
            for (; i < t.ll && ((op + i) & 3); i++) org[op + i] = v0 - (uint32_t)i;
            for (; i + 4 <= t.ll; i += 4) {
                const uint32_t v = v0 - (uint32_t)i;
                *(g_u4 *)(org + op + i) = make_uint4(v, v - 1u, v - 2u, v - 3u);
            }
            for (; i < t.ll; i++) org[op + i] = v0 - (uint32_t)i;
        }
        op += t.ll;
        if (t.last) {
            st.last_ok = 1;
            return;
        }
        {
            const int32_t base = op - t.off;
            const uint32_t off = (uint32_t)t.off;
            uint32_t j = 0;  // entry i = base + (i mod off)
            int32_t i = 0;
            for (; i < t.ml && ((op + i) & 3); i++) {
                org[op + i] = (uint32_t)(base + j);
                j = j + 1 == off ? 0u : j + 1;
            }
            for (; i + 4 <= t.ml; i += 4) {
                uint32_t e[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    e[q] = (uint32_t)(base + j);
                    j = j + 1 == off ? 0u : j + 1;
                }
                *(g_u4 *)(org + op + i) = make_uint4(e[0], e[1], e[2], e[3]);
            }
            for (; i < t.ml; i++) {
                org[op + i] = (uint32_t)(base + j);
                j = j + 1 == off ? 0u : j + 1;
            }
        }
        op += t.ml;
        x = t.next;
    }
}

// grid (x: JX workgroups per block, y: block); each thread strides over its
// block's entries, 4 at a time (a fixed, small grid: the rounds after the
// first mostly find their block settled, and dispatching a workgroup per
// 1,024 entries for them cost more than the hops).
__global__ __launch_bounds__(T) void jump_kernel(Scratch sc, int round) {
    const int b = blockIdx.y;
    BStat &st = sc.st[b];
    if (st.fix[FIX_ROUNDS - 1] || st.bad) return;
    if (round > 0 && !st.jmp[round - 1]) return;
    const int64_t total = st.total;
    const SBlock B = sc.blk[b];
    g_u32 *org = (g_u32 *)(sc.org + B.org_off);
    bool any = false;
    for (int64_t p = ((int64_t)blockIdx.x * T + threadIdx.x) * 4; p < total; p += (int64_t)gridDim.x * T * 4) {
        const int lim = total - p < 4 ? (int)(total - p) : 4;
        uint4 v = *(const g_u4 *)(org + p);
        const uint32_t e0[4] = {v.x, v.y, v.z, v.w};
        int32_t o[4];
#pragma unroll
        for (int i = 0; i < 4; i++) o[i] = i < lim ? (int32_t)e0[i] : -1;
        // the four entries' hops interleaved: four independent loads in flight
        for (int h = 0; h < HOPS; h++) {
            if (o[0] < 0 && o[1] < 0 && o[2] < 0 && o[3] < 0) break;
            int32_t nx[4];
#pragma unroll
            for (int i = 0; i < 4; i++) nx[i] = o[i] >= 0 ? (int32_t)org[o[i]] : o[i];
#pragma unroll
            for (int i = 0; i < 4; i++) o[i] = nx[i];
        }
        uint32_t e[4];
        bool changed = false;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            e[i] = i < lim ? (uint32_t)o[i] : e0[i];
            changed |= e[i] != e0[i];
        }
        if (changed) {
            *(g_u4 *)(org + p) = make_uint4(e[0], e[1], e[2], e[3]);
            any = true;
        }
    }
    if (any) st.jmp[round] = 1;
}

// blocks decoded by this path / handed to the exact kernel (diagnostics)
__device__ unsigned long long g_split_counts[6];

// per block: the verdict (exact path or not) and the result of the good ones
__global__ void verdict_kernel(int nb, Scratch sc, int32_t *__restrict__ ret, int32_t *__restrict__ todo) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nb) return;
    BStat &st = sc.st[b];
    const bool bad = st.bad || !st.last_ok || st.fix[FIX_ROUNDS - 1] || st.unsettled;
    st.todo = bad;
    todo[b] = bad;
    if (!bad) ret[b] = st.total;
    atomicAdd(&g_split_counts[bad ? 1 : 0], 1ull);
    // why a block was handed over: fix-up / jumping did not converge, a token
    // outside the proven cases, no final literal run
    if (st.fix[FIX_ROUNDS - 1]) atomicAdd(&g_split_counts[2], 1ull);
    else if (st.bad) atomicAdd(&g_split_counts[4], 1ull);
    else if (!st.last_ok) atomicAdd(&g_split_counts[5], 1ull);
    else if (st.unsettled) atomicAdd(&g_split_counts[3], 1ull);
}

// (runs before the verdict: an entry that is still not a literal flags its
// block, whose output the exact kernel then rewrites whole)
__global__ __launch_bounds__(T) void gather_kernel(Scratch sc) {
    const int b = blockIdx.y;
    BStat &st = sc.st[b];
    if (st.bad || !st.last_ok || st.fix[FIX_ROUNDS - 1]) return;  // (entries not all written: never read)
    const int64_t p = ((int64_t)blockIdx.x * T + threadIdx.x) * 4;
    const int64_t total = st.total;
    if (p >= total) return;
    const SBlock B = sc.blk[b];
    const gc_u32 *org = (const gc_u32 *)(sc.org + B.org_off);
    const gc_u8 *s = (const gc_u8 *)B.src;
    g_u8 *d = (g_u8 *)B.dst;
    const uint4 v = *(const gc_u4 *)(org + p);
    const uint32_t e[4] = {v.x, v.y, v.z, v.w};
    bool lit = true;
#pragma unroll
    for (int i = 0; i < 4; i++) lit &= p + i >= total || (int32_t)e[i] < 0;
    if (!lit) {
        st.unsettled = 1;
        return;
    }
    if (p + 4 <= total && (((uintptr_t)(d + p)) & 3u) == 0) {
        uint32_t w = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) w |= (uint32_t)s[-(int64_t)(int32_t)e[i] - 1] << (8 * i);
        *(g_u32 *)(d + p) = w;
    } else {
        for (int i = 0; i < 4 && p + i < total; i++) d[p + i] = s[-(int64_t)(int32_t)e[i] - 1];
    }
}

}  // namespace lz4s
}  // namespace jfs

using namespace jfs::lz4s;

// Scratch layout, shared by the planner on the host and the launcher.
static int64_t a256(int64_t x) { return (x + 255) & ~255ll; }

extern "C" int64_t jfs_lz4_split_scratch_bytes(int nb, const int32_t *src_len, const int32_t *cap) {
    int64_t seg = 0, org = 0;
    for (int b = 0; b < nb; b++) {
        const int64_t n = src_len[b] > 0 ? src_len[b] : 0, c = cap[b] > 0 ? cap[b] : 0;
        seg += (n + SEG - 1) / SEG;
        org += (c + 3) & ~3ll;
    }
    return a256(nb * (int64_t)sizeof(SBlock)) + a256(nb * (int64_t)sizeof(BStat)) + 3 * a256(seg * 4) +
           a256(seg * (SEG / 8)) + a256(org * 4) + a256(nb * 4) + 256;
}

// nseg_all / max_cap: Σ segments and the largest dst_cap (grid sizes); the
// host computes both from the same (src_len, cap) it sized the scratch with.
// d_todo (nb int32, optional): 1 for the blocks the exact kernel must redo.
extern "C" int jfs_launch_lz4_split(const jfs_dev_block *d_desc, int nb, int32_t *d_ret, void *d_scratch,
                                    int64_t nseg_all, int64_t max_cap, int64_t norg_all, hipStream_t st) {
    if (nb <= 0) return 0;
    uint8_t *p = (uint8_t *)(((uintptr_t)d_scratch + 255) & ~(uintptr_t)255);
    Scratch sc;
    sc.blk = (SBlock *)p;
    p += a256(nb * (int64_t)sizeof(SBlock));
    sc.st = (BStat *)p;
    p += a256(nb * (int64_t)sizeof(BStat));
    sc.spec_exit = (int32_t *)p;
    p += a256(nseg_all * 4);
    sc.entry = (int32_t *)p;
    p += a256(nseg_all * 4);
    sc.cnt = (int32_t *)p;
    p += a256(nseg_all * 4);
    sc.bits = (uint32_t *)p;
    p += a256(nseg_all * (SEG / 8));
    int32_t *todo = (int32_t *)p;
    p += a256(nb * 4);
    sc.org = (int32_t *)p;
    const int gs = (int)((nseg_all + T - 1) / T);
    const dim3 gp((unsigned)((max_cap / 4 + T) / T), (unsigned)nb);
    hipLaunchKernelGGL(plan_kernel, dim3(1), dim3(T), 0, st, d_desc, nb, sc, nseg_all, max_cap, norg_all);
    if (nseg_all > 0) {
        hipLaunchKernelGGL(spec_kernel, dim3(gs), dim3(T), 0, st, nb, (int)nseg_all, sc);
        for (int r = 0; r < FIX_ROUNDS; r++) hipLaunchKernelGGL(fix_kernel, dim3(gs), dim3(T), 0, st, nb, (int)nseg_all, sc, r);
        hipLaunchKernelGGL(count_kernel, dim3(gs), dim3(T), 0, st, nb, (int)nseg_all, sc);
    }
    hipLaunchKernelGGL(scan_kernel, dim3(nb), dim3(T), 0, st, sc);
    if (nseg_all > 0) {
        // a wave per segment while that leaves the GPU short of waves (a lone
        // block: ~16 k segments), a thread per segment beyond
        if (nseg_all <= EMIT_WAVE_MAX)
            hipLaunchKernelGGL(emit_kernel, dim3((unsigned)((nseg_all + EWV - 1) / EWV)), dim3(T), 0, st, nb, (int)nseg_all, sc);
        else
            hipLaunchKernelGGL(emit_thread_kernel, dim3((unsigned)gs), dim3(T), 0, st, nb, (int)nseg_all, sc);
    }
    // jump grid: about 2,048 workgroups in all (every entry of a 4 MiB block
    // is covered after a few strides), at most one per 1,024 entries
    const unsigned jx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_cap / 4 + T) / T, (2048 + nb - 1) / nb));
    // Rounds: after round r every entry points >= HOPS^r steps up its chain (or
    // to a literal), and a chain is at most one step per token (a step from a
    // token's match lands in an earlier token's output or in its own
    // literals), i.e. <= max_cap / 4 + 1 steps: HOPS^jr above that settles
    // every well-formed block (8 rounds for 4 MiB; each idle launch cost ~6 us
    // of a lone decode).  The gather checks every entry regardless.
    int jr = 1;
    for (double reach = HOPS; reach <= (double)max_cap / 4 + 1 && jr < JUMP_ROUNDS; reach *= HOPS) jr++;
    for (int r = 0; r < jr; r++) hipLaunchKernelGGL(jump_kernel, dim3(jx, (unsigned)nb), dim3(T), 0, st, sc, r);
    hipLaunchKernelGGL(gather_kernel, gp, dim3(T), 0, st, sc);
    hipLaunchKernelGGL(verdict_kernel, dim3((nb + 63) / 64), dim3(64), 0, st, nb, sc, d_ret, todo);
    if (hipGetLastError() != hipSuccess) return -1;
    // the exact one-workgroup kernel for the flagged blocks (the others exit at once)
    return jfs_launch_lz4_decode_todo(d_desc, nb, d_ret, todo, st);
}

// Diagnostics: blocks the small-batch path decoded itself (out[0]) and blocks
// it handed to the exact kernel (out[1]) on the current device since the
// last reset; synchronous.
extern "C" int jfs_lz4_split_counts(uint64_t *out, int reset) {
    unsigned long long v[6] = {0, 0, 0, 0, 0, 0};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_split_counts), sizeof(v)) != hipSuccess) return -1;
    for (int i = 0; i < 6; i++) out[i] = v[i];
    if (reset) {
        unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_split_counts), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
