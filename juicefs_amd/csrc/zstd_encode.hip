// Zstd frame encoder for gfx950 -- one wavefront per input.
//
// Replaces ZSTD_compress(level 1) reached from pkg/compress/compress.go:82-91
// (ZStandard.Compress -> zstd.CompressLevel(dst, src, ZSTD_LEVEL)).  The
// reference pins DataDog/zstd v1.5.6, whose encoder is not available offline,
// so byte parity with it is unpinnable; what this encoder
// guarantees is an RFC 8878 frame that libzstd and the GPU decoder both turn
// back into the input, no larger than ZSTD_COMPRESSBOUND (the capacity the Go
// adapter requires), with the frame layout libzstd uses (FCS always present,
// no checksum, no dictionary, raw blocks for incompressible data, smallest
// literal-header format).
//
// Per 128 KiB block:
//   1. greedy LZ77 parse (4-byte hash of the position, table of 8192 positions
//      in LDS, acceleration skip on misses like LZ4's, forward extension 64
//      bytes per step across the wave, backward catch-up); literals go
//      straight to the output, sequences to a per-input scratch list;
//   2. literals section: Huffman-compressed (Compressed_Literals_Block, 4
//      streams, code lengths <= 11, the tree description FSE-compressed or as
//      direct 4-bit weights), RLE for one repeated byte, else raw -- whichever
//      is smallest, like HUF_compress in libzstd;
//   3. sequences section: Predefined_Mode for all three codes (no table
//      descriptions), FSE-encoded backwards exactly as RFC 8878 section 4.1.2
//      reads it (offsets are sent as offset + 3: no repeat codes);
//   4. if that is not smaller than the block, the block is stored raw.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace zstde {

constexpr int32_t BLK = 128 << 10;          // Block_Maximum_Size
constexpr int64_t SEQ_CAP = BLK / 4 + 64;   // sequences per block (every match is >= 4 bytes)
constexpr int64_t LSTREAM = 36 << 10;       // one Huffman stream (<= 32 KiB of literals) in scratch
constexpr int64_t SCR_PER = SEQ_CAP * 8 + 4 * LSTREAM;  // scratch bytes per input
constexpr int HUF_MAXB = 11;                // code length limit (HUF_TABLELOG_DEFAULT)
constexpr int HUF_MINL = 64;                // fewer literals stay raw
#ifndef JFS_ZE_HBITS
#define JFS_ZE_HBITS 13  // libzstd level 1 for inputs > 256 KiB: hashLog 13
#endif
constexpr int32_t HBITS = JFS_ZE_HBITS;     // hash table: 2^HBITS positions in LDS

#ifdef JFS_PROF
// diagnostic build only: per-phase s_memtime sums of the encoder waves
// (0 parse, 1 literal histogram + Huffman build, 2 Huffman streams, 3 literal
// section writes, 4 sequence tables, 5 sequence bitstream, 6 block header /
// raw fallback; 8 blocks, 9 sequences)
__device__ unsigned long long g_zeprof[12];
#define ZE_DECL uint64_t ze_t = __builtin_amdgcn_s_memtime(), ze_acc[12] = {0};
#define ZE(k) do { const uint64_t x_ = __builtin_amdgcn_s_memtime(); ze_acc[k] += x_ - ze_t; ze_t = x_; } while (0)
#define ZEC(k, n) (ze_acc[k] += (n))
#define ZE_FLUSH() do { if (lane_id() == 0) for (int i_ = 0; i_ < 12; ++i_) atomicAdd(&g_zeprof[i_], (unsigned long long)ze_acc[i_]); } while (0)
#else
#define ZE_DECL
#define ZE(k) do { } while (0)
#define ZEC(k, n) do { } while (0)
#define ZE_FLUSH() do { } while (0)
#endif

// RFC 8878 3.1.1.3.2.1 code tables and 3.1.1.3.2.2 predefined distributions
__constant__ uint32_t LL_BASE[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,   10,  11,  12,   13,   14,   15,    16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t ML_BASE[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  0,  0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// FSE compression table (FSE_buildCTable semantics) of one code type; N =
// state-table capacity (512 for a block's own tables, 64 for the predefined
// and Huffman-weight tables, table log <= 6)
template <int N>
struct CTabN {
    uint16_t st[N];    // state table: tableSize + spread position, by cumulative symbol rank
    int32_t dnb[53];   // deltaNbBits
    int16_t dfs[53];   // deltaFindState (|.| <= 512)
};
typedef CTabN<512> CTab;
typedef CTabN<64> CTab64;
// read view of either size
struct CView {
    const uint16_t *st;
    const int32_t *dnb;
    const int16_t *dfs;
};
template <int N>
__device__ __forceinline__ CView cview(const CTabN<N> &t) { return CView{t.st, t.dnb, t.dfs}; }

// Huffman literal coding state of the current block (lane 0 builds, lanes 0-3 encode)
struct HufSmem {
    uint32_t cnt[256];
    union {
        uint32_t w[512];  // tree node weights (leaves 0..n-1, sorted by count; huf_build)
        struct {          // the tree description's FSE table (huf_describe)
            CTab64 wct;   // Huffman weights (log 6)
            uint8_t tsym[512];
            int32_t cumul[64];
        } d;
    };
    uint16_t par[512];
    uint8_t dep[512];
    uint16_t sym[256];  // leaf -> symbol
    uint16_t code[256];
    uint8_t len[256];
    uint8_t wt[256];    // Huffman weights of symbols 0..maxsym
    int16_t norm[16];   // FSE normalized counts of the weights
    uint8_t hdr[192];   // tree description (header byte first)
    int32_t hsize, maxbits, maxsym, nsym;
    int32_t ssz[4];     // stream sizes
};

// Sequence-table state of the current block (after its literals are written)
struct SeqSmem {
    CTab act[3];           // FSE_Compressed tables (LL, ML, OF)
    uint32_t scnt[3][64];  // code histograms of the block's sequences
    int16_t snorm[3][64];
    uint8_t shdr[3][96];   // their normalized-count headers
    uint8_t tsym[512];     // build_ctab scratch
    int32_t cumul[64];
};

// <= 40 KiB: four inputs (waves) per CU
struct Smem {
    uint32_t table[1 << HBITS];
    CTab64 ct[3];  // 0 LL (log 6), 1 ML (log 6), 2 OF (log 5)
    uint8_t lut_ll[64], lut_ml[128];
    int32_t shsz[3], smode[3], slog[3];
    union {  // a block's literal coding, then its sequence tables
        HufSmem h;
        SeqSmem q;
    };
};
static_assert(sizeof(Smem) <= 40960, "four encoder waves per CU");

__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// Build the encoding table of a predefined distribution (lane 0 writes).
// Spread and state numbering are the decoder's (FSE_buildDTable): -1
// ("less than 1") symbols at the top, the others spread with step
// (size>>1)+(size>>3)+3 skipping the top; state table in symbol order.
template <int N>
__device__ void build_ctab(uint8_t *tsym, int32_t *cumul, CTabN<N> &t, const int16_t *norm, int maxsv, int tlog) {
    if (lane_id() == 0) {
        const int size = 1 << tlog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
        int high = size - 1;
        cumul[0] = 0;
        for (int u = 1; u <= maxsv + 1; u++) {
            if (norm[u - 1] == -1) {
                cumul[u] = cumul[u - 1] + 1;
                tsym[high--] = (uint8_t)(u - 1);
            } else {
                cumul[u] = cumul[u - 1] + norm[u - 1];
            }
        }
        int pos = 0;
        for (int sym = 0; sym <= maxsv; sym++) {
            for (int k = 0; k < norm[sym]; k++) {
                tsym[pos] = (uint8_t)sym;
                do { pos = (pos + step) & mask; } while (pos > high);
            }
        }
        for (int u = 0; u < size; u++) {
            const int sym = tsym[u];
            t.st[cumul[sym]++] = (uint16_t)(size + u);
        }
        int total = 0;
        for (int sym = 0; sym <= maxsv; sym++) {
            const int nc = norm[sym];
            if (nc == 0) {
                t.dnb[sym] = ((tlog + 1) << 16) - size;
                t.dfs[sym] = 0;
            } else if (nc == -1 || nc == 1) {
                t.dnb[sym] = (tlog << 16) - size;
                t.dfs[sym] = total - 1;
                total += 1;
            } else {
                const int mbo = tlog - (int)highbit((uint32_t)(nc - 1));
                t.dnb[sym] = (mbo << 16) - (nc << mbo);
                t.dfs[sym] = total - nc;
                total += nc;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// byte access (the input is read-only; uniform addresses)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld32u(const gc_u8 *p) {
    const uintptr_t a = (uintptr_t)p;
    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = w[0];
    if (sh == 0) return w0;
    return __builtin_amdgcn_alignbyte(w[1], w0, sh);
}

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - HBITS); }
// ZSTD_hash6Ptr: the low 6 bytes of an 8-byte little-endian read
__device__ __forceinline__ uint32_t hash6(uint64_t v) { return (uint32_t)(((v << 16) * 227718039650203ull) >> (64 - HBITS)); }
__device__ __forceinline__ uint64_t ld64u(const gc_u8 *p) {
    const uintptr_t a = (uintptr_t)p;
    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = w[0], w1 = w[1];
    if (sh == 0) return (uint64_t)w0 | ((uint64_t)w1 << 32);
    const uint32_t w2 = w[2];
    return (uint64_t)__builtin_amdgcn_alignbyte(w1, w0, sh) | ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32);
}
#ifndef JFS_ZE_WLOG
#define JFS_ZE_WLOG 19
#endif
#ifndef JFS_ZE_HASH
#define JFS_ZE_HASH 4  // bytes hashed for match candidates (libzstd level 1: 6)
#endif
#ifndef JFS_ZE_PSEARCH
#define JFS_ZE_PSEARCH 1  // lane-parallel search (the serial loop's parse, 64 positions per step)
#endif
#ifndef JFS_ZE_REP
#define JFS_ZE_REP 1   // try the repeat offset one byte ahead first (zstd_fast)
#endif
constexpr int64_t WMAX = 1 << JFS_ZE_WLOG;  // match window (windowLog 19, like level 1)

// ---------------------------------------------------------------------------
// backward bitstream writer (BIT_CStream semantics), uniform; bytes go to HBM
// ---------------------------------------------------------------------------
struct BitW {
    g_u8 *dst;
    int64_t wp, lim;  // next byte position; writes at or beyond lim are refused
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

__device__ __forceinline__ uint32_t fse_init(const CView &t, uint32_t sym) {
    const int32_t dnb = t.dnb[sym];
    const uint32_t nbo = (uint32_t)((dnb + (1 << 15)) >> 16);
    const uint32_t v = (nbo << 16) - (uint32_t)dnb;
    return t.st[(v >> nbo) + (uint32_t)t.dfs[sym]];
}
__device__ __forceinline__ void fse_enc(BitW &w, const CView &t, uint32_t &st, uint32_t sym) {
    const uint32_t nbo = (uint32_t)(((int32_t)st + t.dnb[sym]) >> 16);
    bw_add(w, st, (int)nbo);
    st = t.st[(st >> nbo) + (uint32_t)t.dfs[sym]];
}
__device__ __forceinline__ void fse_fin(BitW &w, uint32_t st, int tlog) {
    bw_add(w, st, tlog);
    bw_flush(w);
}

__device__ __forceinline__ uint32_t ll_code(const Smem &s, uint32_t ll) { return ll < 64 ? s.lut_ll[ll] : highbit(ll) + 19; }
__device__ __forceinline__ uint32_t ml_code(const Smem &s, uint32_t mlb) {
    return mlb < 128 ? s.lut_ml[mlb] : highbit(mlb) + 36;
}

__device__ __forceinline__ void seq_fields(const uint64_t *seq, int64_t i, uint32_t &ll, uint32_t &ml, uint32_t &off) {
    const uint64_t r = seq[i];
    ll = (uint32_t)(r & 0x1FFFFu);
    ml = (uint32_t)((r >> 17) & 0x3FFFFu);
    off = (uint32_t)(r >> 35);
}

// Encode sequences [0, ns) (scratch records: ll | ml << 17 | Offset_Value << 35 as
// u64) as the predefined-mode FSE bitstream at w.wp (ZSTD_encodeSequences
// order: last sequence first, states OF/ML/LL, extra bits LL/ML/OF).
// Per 64 sequences the lanes load the records and look up, in parallel,
// everything that does not depend on the FSE states (codes, extra-bit fields,
// each symbol's deltaNbBits / deltaFindState); the serial loop then only
// steps the three states (one LDS round trip per sequence) and packs bits.
__device__ void encode_sequences(const Smem &s, BitW &w, const uint64_t *seq, int64_t ns) {
    // per table: the block's FSE_Compressed table (mode 2) or the predefined one
    const CView TL = s.smode[0] == 2 ? cview(s.q.act[0]) : cview(s.ct[0]);
    const CView TM = s.smode[1] == 2 ? cview(s.q.act[1]) : cview(s.ct[1]);
    const CView TO = s.smode[2] == 2 ? cview(s.q.act[2]) : cview(s.ct[2]);
    const int l = lane_id();
    uint32_t sML = 0, sOF = 0, sLL = 0;
    for (int64_t c0 = ns - 1; c0 >= 0; c0 -= 64) {
        const int64_t i = c0 - l;
        uint32_t ll = 0, ml = 3, ofv = 1;
        if (i >= 0) seq_fields(seq, i, ll, ml, ofv);
        const uint32_t lc = ll_code(s, ll), mc = ml_code(s, ml - 3), oc = highbit(ofv);
        const int32_t dO = TO.dnb[oc], dM = TM.dnb[mc], dL = TL.dnb[lc];
        const uint32_t fOM = ((uint32_t)(uint16_t)TO.dfs[oc]) | ((uint32_t)(uint16_t)TM.dfs[mc] << 16);
        const int32_t fL = TL.dfs[lc];
        const uint32_t eLL = ll - LL_BASE[lc], eML = ml - ML_BASE[mc], eOF = ofv - (1u << oc);
        const uint32_t nb = (uint32_t)LL_BITS[lc] | ((uint32_t)ML_BITS[mc] << 8) | (oc << 16);
        const int nj = c0 + 1 < 64 ? (int)(c0 + 1) : 64;
        for (int j = 0; j < nj; ++j) {
            const int32_t jdO = (int32_t)readlane((uint32_t)dO, j), jdM = (int32_t)readlane((uint32_t)dM, j),
                          jdL = (int32_t)readlane((uint32_t)dL, j);
            const uint32_t jf = readlane(fOM, j);
            const int32_t jfO = (int16_t)(jf & 0xFFFFu), jfM = (int16_t)(jf >> 16), jfL = (int32_t)readlane((uint32_t)fL, j);
            const uint32_t jnb = readlane(nb, j);
            const uint32_t jeLL = readlane(eLL, j), jeML = readlane(eML, j), jeOF = readlane(eOF, j);
            if (c0 == ns - 1 && j == 0) {
                // FSE_initCState2: the last sequence only sets the states
                const uint32_t nM = (uint32_t)((jdM + (1 << 15)) >> 16), nO = (uint32_t)((jdO + (1 << 15)) >> 16),
                               nL = (uint32_t)((jdL + (1 << 15)) >> 16);
                const uint32_t vM = ((nM << 16) - (uint32_t)jdM) >> nM, vO = ((nO << 16) - (uint32_t)jdO) >> nO,
                               vL = ((nL << 16) - (uint32_t)jdL) >> nL;
                sML = TM.st[vM + (uint32_t)jfM];
                sOF = TO.st[vO + (uint32_t)jfO];
                sLL = TL.st[vL + (uint32_t)jfL];
            } else {
                const uint32_t nO = (uint32_t)(((int32_t)sOF + jdO) >> 16), nM = (uint32_t)(((int32_t)sML + jdM) >> 16),
                               nL = (uint32_t)(((int32_t)sLL + jdL) >> 16);
                bw_add(w, sOF, (int)nO);
                bw_add(w, sML, (int)nM);
                bw_add(w, sLL, (int)nL);
                // the three table reads are independent: one LDS round trip
                const uint32_t tO = TO.st[(sOF >> nO) + (uint32_t)jfO], tM = TM.st[(sML >> nM) + (uint32_t)jfM],
                               tL = TL.st[(sLL >> nL) + (uint32_t)jfL];
                sOF = tO;
                sML = tM;
                sLL = tL;
                bw_flush(w);
            }
            bw_add(w, jeLL, (int)(jnb & 0xFFu));
            bw_add(w, jeML, (int)((jnb >> 8) & 0xFFu));
            bw_flush(w);
            bw_add(w, jeOF, (int)(jnb >> 16));
            bw_flush(w);
        }
    }
    fse_fin(w, sML, s.slog[1]);
    fse_fin(w, sOF, s.slog[2]);
    fse_fin(w, sLL, s.slog[0]);
    bw_add(w, 1, 1);  // end mark
    bw_flush(w);
    if (w.bp > 0) {   // last partial byte
        if (w.wp + 1 > w.lim) w.ovf = true;
        if (!w.ovf && lane_id() == 0) w.dst[w.wp] = (uint8_t)w.bc;
        w.wp++;
        w.bp = 0;
        w.bc = 0;
    }
}


// ---------------------------------------------------------------------------
// Huffman-compressed literals (RFC 8878 4.2.1; the choices of libzstd's
// HUF_compress: code lengths limited to 11, 4 streams, tree description
// FSE-compressed with two interleaved states or as direct 4-bit weights)
// ---------------------------------------------------------------------------
// FSE normalized-count header (RFC 8878 4.1.1; FSE_writeNCount layout).
__device__ int write_ncount(uint8_t *out, const int16_t *norm, int maxsv, int tlog) {
    int o = 0;
    const int tsize = 1 << tlog;
    int remaining = tsize + 1, threshold = tsize, nbits = tlog + 1;
    uint32_t bs = (uint32_t)(tlog - 5);
    int bc = 4;
    int sym = 0, prev0 = 0;
    const int alpha = maxsv + 1;
    while (sym < alpha && remaining > 1) {
        if (prev0) {
            int start = sym;
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
            bs += (uint32_t)(sym - start) << bc;
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

// lane-local backward bitstream into LDS (the tree description)
struct LBits {
    uint8_t *out;
    int o, lim;
    uint64_t bc;
    int bp;
};
__device__ __forceinline__ void lb_add(LBits &b, uint32_t v, int nb) {
    b.bc |= ((uint64_t)v & ((1ull << nb) - 1ull)) << b.bp;
    b.bp += nb;
}
__device__ __forceinline__ void lb_flush(LBits &b) {
    while (b.bp >= 8) {
        if (b.o < b.lim) b.out[b.o] = (uint8_t)b.bc;
        b.o++;
        b.bc >>= 8;
        b.bp -= 8;
    }
}
__device__ __forceinline__ void lb_enc(LBits &b, const CView &t, uint32_t &st, uint32_t sym) {
    const uint32_t nbo = (uint32_t)(((int32_t)st + t.dnb[sym]) >> 16);
    lb_add(b, st, (int)nbo);
    st = t.st[(st >> nbo) + (uint32_t)t.dfs[sym]];
}

// Code lengths (<= HUF_MAXB, complete code) of the counted literals; lane 0.
// Returns max length, 0 when Huffman does not apply (fewer than 2 symbols or
// no exact length limit found).
__device__ int huf_build(HufSmem &h) {
    int n = 0;
    for (int c = 0; c < 256; c++) {
        h.len[c] = 0;
        if (h.cnt[c]) h.sym[n++] = (uint16_t)c;
    }
    h.nsym = n;
    if (n < 2) return 0;
    for (int i = 1; i < n; i++) {  // insertion sort by count (stable in symbol order)
        const uint16_t x = h.sym[i];
        const uint32_t cx = h.cnt[x];
        int j = i - 1;
        while (j >= 0 && h.cnt[h.sym[j]] > cx) {
            h.sym[j + 1] = h.sym[j];
            j--;
        }
        h.sym[j + 1] = x;
    }
    for (int i = 0; i < n; i++) h.w[i] = h.cnt[h.sym[i]];
    int li = 0, qi = n;
    for (int k = n; k < 2 * n - 1; k++) {  // two-queue merge
        int x, y;
        if (li < n && (qi >= k || h.w[li] <= h.w[qi])) x = li++;
        else x = qi++;
        if (li < n && (qi >= k || h.w[li] <= h.w[qi])) y = li++;
        else y = qi++;
        h.w[k] = h.w[x] + h.w[y];
        h.par[x] = h.par[y] = (uint16_t)k;
    }
    const int root = 2 * n - 2;
    h.dep[root] = 0;
    for (int k = root - 1; k >= 0; k--) h.dep[k] = (uint8_t)(h.dep[h.par[k]] + 1);
    // limit to HUF_MAXB: clamp; while the code is over-subscribed lengthen the
    // rarest code still below the limit; then, while under-subscribed, shorten
    // the most frequent codes whose step still fits (Kraft sum in units of
    // 2^-HUF_MAXB; every step is a power of two and codes at the limit step
    // by 1, so the sum lands exactly on 2^HUF_MAXB: a complete prefix code)
    const int64_t full = 1ll << HUF_MAXB;
    int64_t kraft = 0;
    for (int i = 0; i < n; i++) {
        const int d = h.dep[i] > HUF_MAXB ? HUF_MAXB : h.dep[i];
        h.dep[i] = (uint8_t)d;
        kraft += 1ll << (HUF_MAXB - d);
    }
    for (int guard = 0; kraft > full && guard < 4096; guard++) {
        int i = 0;  // leaves are sorted by count: index 0 is the rarest
        while (i < n && h.dep[i] >= HUF_MAXB) i++;
        if (i == n) return 0;
        kraft -= 1ll << (HUF_MAXB - h.dep[i] - 1);
        h.dep[i]++;
    }
    for (int guard = 0; kraft < full && guard < 64; guard++) {
        for (int i = n - 1; i >= 0 && kraft < full; i--) {  // most frequent first
            const int64_t add = h.dep[i] > 1 ? 1ll << (HUF_MAXB - h.dep[i]) : full;
            if (kraft + add <= full) {
                h.dep[i]--;
                kraft += add;
            }
        }
    }
    if (kraft != full) return 0;
    int maxb = 0;
    for (int i = 0; i < n; i++) {
        h.len[h.sym[i]] = h.dep[i];
        maxb = h.dep[i] > maxb ? h.dep[i] : maxb;
    }
    // canonical codes: longest first, symbol order within a length
    uint32_t c = 0;
    for (int nb = maxb; nb >= 1; nb--) {
        for (int v = 0; v < 256; v++)
            if (h.len[v] == nb) h.code[v] = (uint16_t)c++;
        c >>= 1;
    }
    int maxsym = 0;
    for (int v = 0; v < 256; v++) {
        h.wt[v] = h.len[v] ? (uint8_t)(maxb + 1 - h.len[v]) : 0;
        if (h.len[v]) maxsym = v;
    }
    h.maxsym = maxsym;
    return maxb;
}

// Tree description into h.hdr: FSE-compressed weights (2 states, table log
// 6) when that is smaller, else direct 4-bit weights (<= 128 transmitted).
// Returns its size, or -1 when neither applies.  Lane 0 (h.d: table + scratch).
__device__ int huf_describe(Smem &s) {
    HufSmem &h = s.h;
    const int nw = h.maxsym;  // weights of symbols 0..maxsym-1 (the last one is implied)
    int fse = -1;
    if (nw >= 2) {
        int wc[16] = {0};
        int maxsv = 0;
        for (int i = 0; i < nw; i++) {
            wc[h.wt[i]]++;
            maxsv = h.wt[i] > maxsv ? h.wt[i] : maxsv;
        }
        const int tlog = 6, tsize = 1 << tlog;
        int sum = 0, big = 0;
        for (int v = 0; v <= maxsv; v++) {
            h.norm[v] = (int16_t)(wc[v] ? (wc[v] * tsize / nw > 0 ? wc[v] * tsize / nw : 1) : 0);
            sum += h.norm[v];
            if (wc[v] > wc[big]) big = v;
        }
        h.norm[big] = (int16_t)(h.norm[big] + (tsize - sum));
        if (h.norm[big] >= 1) {
            int o = 1 + write_ncount(h.hdr + 1, h.norm, maxsv, tlog);
            build_ctab(h.d.tsym, h.d.cumul, h.d.wct, h.norm, maxsv, tlog);
            LBits b;
            b.out = h.hdr;
            b.o = o;
            b.lim = 128;
            b.bc = 0;
            b.bp = 0;
            // FSE_compress_usingCTable order: two states, last symbols first
            int ip = nw;
            uint32_t s1, s2;
            if (nw & 1) {
                s1 = fse_init(cview(h.d.wct), h.wt[--ip]);
                s2 = fse_init(cview(h.d.wct), h.wt[--ip]);
                lb_enc(b, cview(h.d.wct), s1, h.wt[--ip]);
                lb_flush(b);
            } else {
                s2 = fse_init(cview(h.d.wct), h.wt[--ip]);
                s1 = fse_init(cview(h.d.wct), h.wt[--ip]);
            }
            if ((nw - 2) & 2) {
                lb_enc(b, cview(h.d.wct), s2, h.wt[--ip]);
                lb_enc(b, cview(h.d.wct), s1, h.wt[--ip]);
                lb_flush(b);
            }
            while (ip > 0) {
                lb_enc(b, cview(h.d.wct), s2, h.wt[--ip]);
                lb_enc(b, cview(h.d.wct), s1, h.wt[--ip]);
                lb_enc(b, cview(h.d.wct), s2, h.wt[--ip]);
                lb_enc(b, cview(h.d.wct), s1, h.wt[--ip]);
                lb_flush(b);
            }
            lb_add(b, s2, tlog);
            lb_flush(b);
            lb_add(b, s1, tlog);
            lb_flush(b);
            lb_add(b, 1, 1);  // end mark
            lb_flush(b);
            if (b.bp > 0) {
                if (b.o < b.lim) b.out[b.o] = (uint8_t)b.bc;
                b.o++;
            }
            if (b.o - 1 < 128) {
                h.hdr[0] = (uint8_t)(b.o - 1);
                fse = b.o;
            }
        }
    }
    const int direct = nw <= 128 ? 1 + (nw + 1) / 2 : -1;
    if (fse > 0 && (direct < 0 || fse <= direct)) return fse;
    if (direct < 0) return -1;
    h.hdr[0] = (uint8_t)(127 + nw);
    for (int i = 0; i < nw; i += 2) h.hdr[1 + i / 2] = (uint8_t)((h.wt[i] << 4) | (i + 1 < nw ? h.wt[i + 1] : 0));
    return direct;
}

// Encode literals lit[0, L) as four Huffman streams into the scratch (lanes
// 0-3, one stream each, last symbol first); returns the streams' total size.
__device__ int64_t huf_streams(Smem &s, const gc_u8 *lit, int64_t L, g_u8 *scr) {
    HufSmem &h = s.h;
    const int l = lane_id();
    const int64_t seg = (L + 3) / 4;
    if (l < 4) {
        const int64_t a = l * seg, e = (l + 1) * seg < L ? (l + 1) * seg : L;
        g_u8 *out = scr + l * LSTREAM;
        int64_t o = 0;
        uint64_t bc = 0;
        int bp = 0;
        for (int64_t i = e - 1; i >= a; --i) {
            const uint32_t v = lit[i];
            bc |= (uint64_t)h.code[v] << bp;
            bp += h.len[v];
            if (bp >= 32) {
                out[o] = (uint8_t)bc;
                out[o + 1] = (uint8_t)(bc >> 8);
                out[o + 2] = (uint8_t)(bc >> 16);
                out[o + 3] = (uint8_t)(bc >> 24);
                o += 4;
                bc >>= 32;
                bp -= 32;
            }
        }
        bc |= 1ull << bp;  // end mark
        bp += 1;
        while (bp > 0) {
            out[o++] = (uint8_t)bc;
            bc >>= 8;
            bp -= 8;
        }
        h.ssz[l] = (int32_t)o;
    }
    __syncthreads();
    return (int64_t)h.ssz[0] + h.ssz[1] + h.ssz[2] + h.ssz[3];
}

// Sequence tables of one block (RFC 8878 3.1.1.3.2.1): FSE_Compressed when the
// estimated bits (symbols + table header) beat the predefined distribution.
// All lanes histogram the codes; lane 0 normalizes, writes the headers and
// builds the tables.  Sets s.smode / s.slog / s.shdr / s.shsz.
__device__ void choose_seq_tables(Smem &s, const uint64_t *seq, int64_t ns) {
    const int l = lane_id();
    for (int k = l; k < 3 * 64; k += 64) (&s.q.scnt[0][0])[k] = 0;
    __syncthreads();
    for (int64_t i = l; i < ns; i += 64) {
        uint32_t ll, ml, off;
        seq_fields(seq, i, ll, ml, off);
        atomicAdd(&s.q.scnt[0][ll_code(s, ll)], 1u);
        atomicAdd(&s.q.scnt[1][ml_code(s, ml - 3)], 1u);
        atomicAdd(&s.q.scnt[2][highbit(off)], 1u);
    }
    __syncthreads();
    if (l == 0) {
        const int16_t *pre[3] = {LL_DEF, ML_DEF, OF_DEF};
        const int prelog[3] = {6, 6, 5}, premax[3] = {35, 52, 28}, maxlog[3] = {9, 9, 8}, nsym[3] = {36, 53, 32};
        for (int t = 0; t < 3; t++) {
            s.smode[t] = 0;
            s.slog[t] = prelog[t];
            s.shsz[t] = 0;
            const uint32_t *cnt = s.q.scnt[t];
            int maxsv = 0, distinct = 0;
            for (int v = 0; v < nsym[t]; v++)
                if (cnt[v]) { maxsv = v; distinct++; }
            if (ns < 64 || distinct < 2) continue;
            // predefined cost (bits); a code it cannot express forces mode 2
            float pc = 0.f;
            bool pre_ok = maxsv <= premax[t];
            for (int v = 0; v <= maxsv && pre_ok; v++) {
                if (!cnt[v]) continue;
                const int pn = pre[t][v] == -1 ? 1 : pre[t][v];
                if (pn <= 0) { pre_ok = false; break; }
                pc += (float)cnt[v] * ((float)prelog[t] - __log2f((float)pn));
            }
            int tlog = (int)highbit((uint32_t)(ns - 1)) - 2;
            tlog = tlog < 5 ? 5 : tlog > maxlog[t] ? maxlog[t] : tlog;
            while ((1 << tlog) < 2 * distinct && tlog < maxlog[t]) tlog++;
            const int tsize = 1 << tlog;
            int16_t *norm = s.q.snorm[t];
            int sum = 0, big = 0;
            for (int v = 0; v <= maxsv; v++) {
                int nv = 0;
                if (cnt[v]) {
                    nv = (int)(((uint64_t)cnt[v] * (uint64_t)tsize) / (uint64_t)ns);
                    nv = nv < 1 ? 1 : nv;
                }
                norm[v] = (int16_t)nv;
                sum += nv;
                if (cnt[v] > cnt[big]) big = v;
            }
            norm[big] = (int16_t)(norm[big] + (tsize - sum));
            if (norm[big] < 1) continue;  // (cannot happen with 2 * distinct <= tsize)
            float cc = 0.f;
            for (int v = 0; v <= maxsv; v++)
                if (cnt[v]) cc += (float)cnt[v] * ((float)tlog - __log2f((float)norm[v]));
            const int hs = write_ncount(s.q.shdr[t], norm, maxsv, tlog);
            cc += 8.f * (float)hs;
            if (pre_ok && pc <= cc) continue;
            build_ctab(s.q.tsym, s.q.cumul, s.q.act[t], norm, maxsv, tlog);
            s.smode[t] = 2;
            s.slog[t] = tlog;
            s.shsz[t] = hs;
        }
    }
    __syncthreads();
}

// wave-parallel byte copy src[a, a+len) -> dst[o, o+len)
__device__ __forceinline__ void copy_bytes(g_u8 *dst, int64_t o, const gc_u8 *src, int64_t a, int64_t len) {
    const int l = lane_id();
    for (int64_t k = l; k < len; k += 64) dst[o + k] = src[a + k];
}

__device__ __forceinline__ void put3(g_u8 *dst, int64_t o, uint32_t v) {
    const int l = lane_id();
    if (l < 3) dst[o + l] = (uint8_t)(v >> (8 * l));
}

// Frame header size (magic, FHD, [Window_Descriptor], Frame_Content_Size).
__device__ __forceinline__ int frame_header(int64_t n, bool write, g_u8 *dst) {
    const int l = lane_id();
    const bool single = n <= (1 << 19);
    int fcs_flag, fs;
    if (single) {
        if (n < 256) { fcs_flag = 0; fs = 1; }
        else if (n < 65536 + 256) { fcs_flag = 1; fs = 2; }
        else { fcs_flag = 2; fs = 4; }
    } else {
        fcs_flag = n < (1ll << 32) ? 2 : 3;
        fs = fcs_flag == 2 ? 4 : 8;
    }
    const uint32_t fhd = (uint32_t)((fcs_flag << 6) | (single ? 0x20 : 0));
    const int fpos = single ? 5 : 6;  // FCS position
    const uint64_t fv = (uint64_t)n - (fs == 2 ? 256 : 0);
    const int hn = fpos + fs;
    uint32_t byte = 0;
    if (l < 4) byte = (0xFD2FB528u >> (8 * l)) & 0xFFu;
    else if (l == 4) byte = fhd;
    else if (l == 5 && !single) byte = (19 - 10) << 3;  // windowLog 19 (512 KiB), like level 1
    else if (l >= fpos && l < hn) byte = (uint32_t)(fv >> (8 * (l - fpos))) & 0xFFu;
    if (write && l < hn) dst[l] = (uint8_t)byte;
    return hn;
}

__device__ __forceinline__ int64_t ze_bound(int64_t n) { return n + (n >> 8) + (n < BLK ? (BLK - n) >> 11 : 0); }

// Block-parallel mode (BPAR): one work item = one 128 KiB block of a frame,
// encoded into its slot dst[hn + k * SLOT] (a block and its literal staging
// never exceed SLOT bytes); zstd_compact_kernel then moves the blocks down
// to their frame positions.  The wave's hash table starts from the WARM bytes
// before the block (every position inserted), the repeat offset starts
// unknown (no repeat code before the block's first explicit offset): the
// frames are valid RFC 8878 frames, the window (512 KiB) reaches back into
// earlier blocks.  Without BPAR one wave encodes a whole frame, block after
// block.
constexpr int64_t SLOT = BLK + 16;
#ifndef JFS_ZE_WARM_KB
#define JFS_ZE_WARM_KB 256  // 64: ratio 3.032, 128: 3.049, 256: 3.054 (one wave per frame: 3.052)
#endif
constexpr int64_t WARM = (int64_t)JFS_ZE_WARM_KB << 10;

template <bool BPAR>
__global__ __launch_bounds__(64) void zstd_encode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                        int32_t *__restrict__ ret, uint64_t *__restrict__ scratch,
                                                        const int2 *__restrict__ work, int nwork,
                                                        int32_t *__restrict__ bsize) {
    __shared__ Smem s;
    if (!BPAR && (int)blockIdx.x >= nblk) return;
    const int l = lane_id();
    // per-wave scratch: sequences and Huffman streams of the current block
    const int64_t sidx = (int64_t)blockIdx.x;
    uint64_t *seq = (uint64_t *)((uint8_t *)scratch + sidx * SCR_PER);
    g_u8 *lscr = (g_u8 *)((uint8_t *)scratch + sidx * SCR_PER + SEQ_CAP * 8);
    // tables
    for (int v = l; v < 64; v += 64) {
        int c = 0;
        while (c + 1 < 36 && LL_BASE[c + 1] <= (uint32_t)v) c++;
        s.lut_ll[v] = (uint8_t)c;
    }
    for (int v = l; v < 128; v += 64) {
        int c = 0;
        while (c + 1 < 53 && ML_BASE[c + 1] - 3 <= (uint32_t)v) c++;
        s.lut_ml[v] = (uint8_t)c;
    }
    for (int t = l; t < 3; t += 64) {
        s.smode[t] = 0;
        s.slog[t] = t == 2 ? 5 : 6;
        s.shsz[t] = 0;
    }
    build_ctab(s.q.tsym, s.q.cumul, s.ct[0], LL_DEF, 35, 6);
    __builtin_amdgcn_wave_barrier();
    build_ctab(s.q.tsym, s.q.cumul, s.ct[1], ML_DEF, 52, 6);
    __builtin_amdgcn_wave_barrier();
    build_ctab(s.q.tsym, s.q.cumul, s.ct[2], OF_DEF, 28, 5);
    __syncthreads();
    ZE_DECL

    for (int wi = BPAR ? (int)blockIdx.x : 0; BPAR ? wi < nwork : wi < 1; wi += BPAR ? (int)gridDim.x : 1) {
    const int b = BPAR ? work[wi].x : (int)blockIdx.x;  // the frame (input)
    const int kb = BPAR ? work[wi].y : 0;               // its block (BPAR)
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    const gc_u8 *src = (const gc_u8 *)d.src;
    g_u8 *dst = (g_u8 *)d.dst;
    const int64_t n = d.src_len, cap = d.dst_cap;
    if (n < 0 || cap < ze_bound(n)) {  // compress.go:86-89: cap(dst) < CompressBound -> "buffer too short"
        if (l == 0) {
            if (BPAR) bsize[wi] = -1;
            else ret[b] = -2;
        }
        continue;
    }
    // ---- frame header (BPAR: written by the frame's first block)
    const int hn = frame_header(n, !BPAR || kb == 0, dst);
    const int64_t slot0 = BPAR ? hn + (int64_t)kb * SLOT : hn;
    int64_t op = slot0;
    for (int k = l; k < (1 << HBITS); k += 64) s.table[k] = 0;
    int64_t bs = BPAR ? (int64_t)kb * BLK : 0;
    if (BPAR && bs > 0) {  // warm-up: the positions of the WARM bytes before the block
        __builtin_amdgcn_wave_barrier();
        const int64_t w0 = bs > WARM ? bs - WARM : 0;
        for (int64_t q0 = w0; q0 + 8 <= bs; q0 += 64) {
            const int64_t q = q0 + l;
            if (q + 8 <= bs) {
                const uint64_t v = ld64u(src + q);
                s.table[JFS_ZE_HASH == 6 ? hash6(v) : hash4((uint32_t)v)] = (uint32_t)q;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();

    // ---- blocks (the repeat offsets carry across the frame's blocks, RFC 8878 3.1.1.5)
    uint32_t rep0 = BPAR && bs > 0 ? 0u : 1u;  // Repeated_Offset1 (0: unknown; only it is reused: Offset_Value 1 with LL > 0)
    do {
        const int64_t be = bs + BLK < n ? bs + BLK : n;
        const bool last = be == n;
        const int64_t raw = be - bs;
        const int64_t lit0 = op + 3 + 3;  // block header + largest literals header
        int64_t L = 0, ns = 0;
        bool ok = raw > 0;
        // 1. parse; literals straight to dst[lit0 + L]
        {
            int64_t ip = bs, anchor = bs;
            uint32_t miss = 0;
            while (ok && ip + 8 <= be) {
                // zstd_fast: a repeat-offset match one byte ahead first, else the
                // 6-byte hash candidate (level 1: minMatch 6) within the window
                int64_t cand;
                uint32_t ofv = 0;  // Offset_Value: 1 = repeat offset 1, else offset + 3
#if JFS_ZE_PSEARCH
                // Lane-parallel search: lane j takes the j-th next position of
                // the miss schedule and makes both checks of the serial loop
                // there (repeat offset one byte ahead, then the hash candidate);
                // the first lane with a match ends the search.  Table entries
                // are read before any insert of the batch, which is the serial
                // order while no two positions share a hash: the batch is cut
                // at the first lane of a shared hash (tagged write + read-back),
                // so the parse is the serial loop's exactly.
                {
                    bool done = false;
                    for (;;) {
                        const uint32_t st = 1u + ((miss + (uint32_t)l) >> 6);
                        const uint32_t inc = dpp_scan_add(st);
                        const int64_t P = ip + (int64_t)(inc - st);
                        const uint64_t onm = __ballot(P + 8 <= be);
                        const int nl = ~onm ? (int)__builtin_ctzll(~onm) : 64;
                        if (nl == 0) { done = true; break; }
                        const bool on = l < nl;
                        bool rep = false;
                        uint64_t v = 0;
                        uint32_t h = 0, E = 0;
                        if (on) {
                            const int64_t rp = P + 1;
                            rep = JFS_ZE_REP && rep0 > 0 && rep0 <= rp && ld32u(src + rp) == ld32u(src + rp - rep0);
                            v = ld64u(src + P);
                            h = JFS_ZE_HASH == 6 ? hash6(v) : hash4((uint32_t)v);
                            E = s.table[h];
                        }
                        const uint32_t tag = 0xFFFFFF00u | (uint32_t)l;  // never a position (inputs < 2 GiB)
                        if (on) s.table[h] = tag;
                        __builtin_amdgcn_wave_barrier();
                        uint32_t cm = 64u;
                        if (on) {
                            const uint32_t t = s.table[h];
                            if (t != tag) cm = umin32((uint32_t)l, t & 0xFFu);
                        }
                        const int ncut = (int)dwave_min(cm) + 1;
                        const int nb = ncut < nl ? ncut : nl;  // lanes [0, nb) are exact
                        if (on && l >= nb) s.table[h] = E;
                        const int64_t hc = (int64_t)E;
                        bool hit = l < nb && !rep && hc < P && P - hc <= WMAX;
                        if (__ballot(hit)) {
                            if (hit) hit = ld32u(src + hc) == (uint32_t)v;
                        }
                        const bool got = l < nb && (rep || hit);
                        const uint64_t gm = __ballot(got);
                        const int jm = gm ? (int)__builtin_ctzll(gm) : 64;
                        // inserts: every position before jm, and jm itself unless its repeat check hit
                        if (l < nb) s.table[h] = (l < jm || (l == jm && !rep)) ? (uint32_t)P : E;
                        __builtin_amdgcn_wave_barrier();
                        if (gm) {
                            const int64_t pj = ip + (int64_t)readlane(inc - st, jm);
                            if (readlane(rep ? 1u : 0u, jm)) {
                                ip = pj + 1;
                                cand = ip - rep0;
                                ofv = 1;
                            } else {
                                ip = pj;
                                cand = (int64_t)readlane(E, jm);
                            }
                            break;
                        }
                        ip += (int64_t)readlane(inc, nb - 1);
                        miss += (uint32_t)nb;
                    }
                    if (done) break;
                }
                {
#else
                const int64_t rp = ip + 1;
                if (JFS_ZE_REP && rep0 > 0 && rep0 <= rp && ld32u(src + rp) == ld32u(src + rp - rep0)) {
                    cand = rp - rep0;
                    ip = rp;
                    ofv = 1;
                } else {
                    const uint64_t v = ld64u(src + ip);
                    const uint32_t h = JFS_ZE_HASH == 6 ? hash6(v) : hash4((uint32_t)v);
                    cand = (int64_t)s.table[h];
                    s.table[h] = (uint32_t)ip;
                    bool hit = cand < ip && ip - cand <= WMAX;
                    if (hit) hit = ld32u(src + cand) == (uint32_t)v;
                    if (!hit) {
                        ip += 1 + (miss++ >> 6);
                        continue;
                    }
#endif
                }
                miss = 0;
                // forward extension from +4 (64 bytes per step, up to the block
                // end) and backward catch-up (new offsets only): the first step
                // of both is loaded in one HBM round trip
                int64_t ml = 4;
                int64_t lim = 0;
                if (ofv == 0) {
                    lim = ip - anchor;
                    if (cand < lim) lim = cand;
                }
                const int64_t kk = 1 + l, a0 = ip + 4 + l;
                uint32_t xa = 0, xb = 1, ca = 0, cb = 1;
                if (a0 < be) { xa = src[a0]; xb = src[cand + 4 + l]; }
                if (kk <= lim) { ca = src[ip - kk]; cb = src[cand - kk]; }
                {
                    const uint64_t ne = ~__ballot(a0 < be && xa == xb);
                    const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                    ml += run;
                    bool more = run == 64;
                    while (more) {
                        const int64_t a = ip + ml + l;
                        const bool eq = a < be && src[a] == src[cand + ml + l];
                        const uint64_t ne2 = ~__ballot(eq);
                        const int r2 = ne2 ? (int)__builtin_ctzll(ne2) : 64;
                        ml += r2;
                        more = r2 == 64;
                    }
                }
                int64_t m0 = cand;
                if (ofv == 0) {
                    const uint64_t cne = ~__ballot(kk <= lim && ca == cb);
                    int64_t back = cne ? (int)__builtin_ctzll(cne) : 64;
                    bool cmore = back == 64;
                    while (cmore && back < lim) {
                        const int64_t k = back + 1 + l;
                        const bool eq = k <= lim && src[ip - k] == src[m0 - k];
                        const uint64_t ne = ~__ballot(eq);
                        const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        back += run;
                        cmore = run == 64;
                    }
                    if (back > lim) back = lim;
                    ip -= back;
                    m0 -= back;
                    ml += back;
                }
                const int64_t ll = ip - anchor;
                copy_bytes(dst, lit0 + L, src, anchor, ll);
                L += ll;
                if (ns >= SEQ_CAP) { ok = false; break; }
                if (ofv == 0) {  // a new offset enters the repeat history
                    const uint32_t off = (uint32_t)(ip - m0);
                    ofv = off + 3;
                    rep0 = off;
                }
                if (l == 0) seq[ns] = (uint64_t)ll | ((uint64_t)ml << 17) | ((uint64_t)ofv << 35);
                ns++;
                ip += ml;
                anchor = ip;
                if (ip - 2 >= bs && ip + 6 <= n) {
                    const uint64_t v2 = ld64u(src + ip - 2);
                    s.table[JFS_ZE_HASH == 6 ? hash6(v2) : hash4((uint32_t)v2)] = (uint32_t)(ip - 2);
                }
            }
            if (ok) {  // last literals of the block
                copy_bytes(dst, lit0 + L, src, anchor, be - anchor);
                L += be - anchor;
            }
        }
        __threadfence_block();
        ZE(0);
        ZEC(8, 1);
        ZEC(9, ns);
        // 2./3. headers and the sequences bitstream
        int64_t end = lit0 + L;
        if (ok) {
            // literal section kind: 2 Huffman, 1 RLE, 0 raw -- the smallest
            const int hsz = L < 32 ? 1 : L < 4096 ? 2 : 3;  // raw / RLE header bytes
            int kind = 0;
            int64_t hcs = 0;  // Huffman: Compressed_Size (tree + jump table + streams)
            int hlh = 0;      // Huffman: literal header bytes
            if (L >= HUF_MINL) {
                wait_vm();  // the literals this wave stored are read back
                for (int k = l; k < 256; k += 64) s.h.cnt[k] = 0;
                __syncthreads();
                for (int64_t k = l; k < L; k += 64) atomicAdd(&s.h.cnt[dst[lit0 + k]], 1u);
                __syncthreads();
                if (l == 0) {
                    s.h.maxbits = huf_build(s.h);
                    s.h.hsize = s.h.maxbits > 0 ? huf_describe(s) : -1;
                }
                __syncthreads();
                ZE(1);
                if (s.h.nsym == 1) {
                    kind = 1;
                } else if (s.h.maxbits > 0 && s.h.hsize > 0) {
                    const int64_t ss = huf_streams(s, (const gc_u8 *)dst + lit0, L, lscr);
                    hcs = s.h.hsize + 6 + ss;
                    const int64_t big = L > hcs ? L : hcs;
                    hlh = big < 1024 ? 3 : big < 16384 ? 4 : 5;
                    if (big < (1 << 18) && hlh + hcs < hsz + L) kind = 2;
                }
                wait_vm();
                __syncthreads();
                ZE(2);
            }
            if (kind == 2) {
                const uint64_t sf = hlh == 3 ? 1 : hlh == 4 ? 2 : 3;
                const int sb = hlh == 3 ? 10 : hlh == 4 ? 14 : 18;
                const uint64_t lh = 2u | (sf << 2) | ((uint64_t)L << 4) | ((uint64_t)hcs << (4 + sb));
                int64_t o = op + 3;
                if (l < hlh) dst[o + l] = (uint8_t)(lh >> (8 * l));
                o += hlh;
                for (int k = l; k < s.h.hsize; k += 64) dst[o + k] = s.h.hdr[k];
                o += s.h.hsize;
                if (l < 3) {  // jump table: sizes of streams 1-3
                    dst[o + 2 * l] = (uint8_t)s.h.ssz[l];
                    dst[o + 2 * l + 1] = (uint8_t)(s.h.ssz[l] >> 8);
                }
                o += 6;
                for (int k = 0; k < 4; k++) {
                    copy_bytes(dst, o, (const gc_u8 *)lscr + k * LSTREAM, 0, s.h.ssz[k]);
                    o += s.h.ssz[k];
                }
                end = o;
            } else if (kind == 1) {
                const uint32_t lh = hsz == 1   ? ((uint32_t)L << 3) | 1u
                                    : hsz == 2 ? (1u << 2) | ((uint32_t)L << 4) | 1u
                                               : (3u << 2) | ((uint32_t)L << 4) | 1u;
                const uint8_t v = dst[lit0];
                __builtin_amdgcn_wave_barrier();
                if (l < hsz) dst[op + 3 + l] = (uint8_t)(lh >> (8 * l));
                if (l == 0) dst[op + 3 + hsz] = v;
                end = op + 3 + hsz + 1;
            }
            // Raw_Literals_Block with the smallest Size_Format (1, 2 or 3 header
            // bytes, like libzstd); the literals move down to follow it
            const uint32_t lh = hsz == 1   ? (uint32_t)L << 3
                                : hsz == 2 ? (1u << 2) | ((uint32_t)L << 4)
                                           : (3u << 2) | ((uint32_t)L << 4);
            if (kind == 0 && hsz < 3) {
                const int64_t to = op + 3 + hsz;
                for (int64_t k = 0; k < L; k += 64) {  // dst < src: ascending chunks are safe
                    uint8_t v = 0;
                    if (k + l < L) v = dst[lit0 + k + l];
                    __builtin_amdgcn_wave_barrier();
                    if (k + l < L) dst[to + k + l] = v;
                }
                end = to + L;
            }
            if (kind == 0 && l < hsz) dst[op + 3 + l] = (uint8_t)(lh >> (8 * l));
            __threadfence_block();
            if (ns < 128) {
                if (l == 0) dst[end] = (uint8_t)ns;
                end += 1;
            } else if (ns < 0x7F00) {
                if (l == 0) dst[end] = (uint8_t)((ns >> 8) + 128);
                if (l == 1) dst[end + 1] = (uint8_t)(ns & 255);
                end += 2;
            } else {
                const int64_t r = ns - 0x7F00;
                if (l == 0) dst[end] = 255;
                if (l == 1) dst[end + 1] = (uint8_t)(r & 255);
                if (l == 2) dst[end + 2] = (uint8_t)(r >> 8);
                end += 3;
            }
            ZE(3);
            if (ns > 0) {
                choose_seq_tables(s, seq, ns);
                ZE(4);
                // Symbol_Compression_Modes: LL bits 7-6, OF 5-4, ML 3-2; then the
                // table descriptions in the order LL, OF, ML
                if (l == 0) dst[end] = (uint8_t)((s.smode[0] << 6) | (s.smode[2] << 4) | (s.smode[1] << 2));
                end += 1;
                for (int t : {0, 2, 1}) {
                    for (int k = l; k < s.shsz[t]; k += 64) dst[end + k] = s.q.shdr[t][k];
                    end += s.shsz[t];
                }
                __threadfence_block();
                BitW w;
                w.dst = dst;
                w.wp = end;
                w.lim = op + 3 + raw;  // not smaller than raw -> stored raw anyway
                w.bc = 0;
                w.bp = 0;
                w.ovf = false;
                encode_sequences(s, w, seq, ns);
                end = w.wp;
                if (w.ovf) ok = false;
                ZE(5);
            }
        }
        const int64_t csize = end - (op + 3);
        __threadfence_block();
        if (ok && csize < raw) {
            put3(dst, op, (uint32_t)((csize << 3) | (2u << 1) | (last ? 1u : 0u)));
            op = end;
        } else {
            put3(dst, op, (uint32_t)((raw << 3) | (last ? 1u : 0u)));  // Raw_Block
            copy_bytes(dst, op + 3, src, bs, raw);
            op += 3 + raw;
        }
        __threadfence_block();
        ZE(6);
        bs = be;
    } while (!BPAR && bs < n);
    if (l == 0) {
        if (BPAR) bsize[wi] = (int32_t)(op - slot0);
        else ret[b] = op <= cap ? (int32_t)op : -2;
    }
    }
    ZE_FLUSH();
}

// BPAR: move every frame's blocks from their slots to their places (ascending:
// a block only moves down, over bytes already moved or its own) and report
// the frame size.  One wave per frame; first[f] = index of its first item.
__global__ __launch_bounds__(64) void zstd_compact_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                         int32_t *__restrict__ ret, const int32_t *__restrict__ bsize,
                                                         const int32_t *__restrict__ first) {
    const int f = blockIdx.x;
    if (f >= nblk) return;
    const int l = lane_id();
    const jfs_dev_block d = ((const gc_blk *)blocks)[f];
    g_u8 *dst = (g_u8 *)d.dst;
    const int64_t n = d.src_len, cap = d.dst_cap;
    const int i0 = first[f], i1 = first[f + 1];
    bool bad = n < 0 || cap < ze_bound(n);
    for (int i = i0; i < i1 && !bad; i++) bad = bsize[i] < 0;
    if (bad) {
        if (l == 0) ret[f] = -2;
        return;
    }
    const int hn = frame_header(n, false, dst);
    int64_t out = hn;
    for (int i = i0; i < i1; i++) {
        const int64_t from = hn + (int64_t)(i - i0) * SLOT, sz = bsize[i];
        if (from != out) {
            // dst[out, out + sz) <- dst[from, from + sz): 16-byte stores, the
            // source read as aligned dwords (alignbyte), 1 KiB per wave step
            int64_t x = 0;
            const uint32_t hm = (uint32_t)(((uintptr_t)(dst + out)) & 15u), ha = (16u - hm) & 15u;
            const int64_t head = (int64_t)ha < sz ? (int64_t)ha : sz;
            uint8_t hb = 0;
            if (l < head) hb = dst[from + l];
            __builtin_amdgcn_wave_barrier();
            if (l < head) dst[out + l] = hb;
            x = head;
            for (; x + 16 <= sz; x += 1024) {
                const int64_t y = x + 16 * l;
                uint4 o = make_uint4(0, 0, 0, 0);
                const bool on = y + 16 <= sz;
                if (on) {
                    const uintptr_t a = (uintptr_t)(dst + from + y);
                    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
                    const uint32_t sh = (uint32_t)(a & 3u);
                    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = sh ? w[4] : 0u;
                    o.x = __builtin_amdgcn_alignbyte(w1, w0, sh);
                    o.y = __builtin_amdgcn_alignbyte(w2, w1, sh);
                    o.z = __builtin_amdgcn_alignbyte(w3, w2, sh);
                    o.w = __builtin_amdgcn_alignbyte(w4, w3, sh);
                }
                if (on) *(g_u4 *)(dst + out + y) = o;
            }
            const int64_t xe = head + ((sz - head) & ~(int64_t)15);
            uint8_t tb = 0;
            if (xe + l < sz) tb = dst[from + xe + l];
            if (xe + l < sz) dst[out + xe + l] = tb;
        }
        out += sz;
    }
    if (l == 0) ret[f] = out <= cap ? (int32_t)out : -2;
}

}  // namespace zstde
}  // namespace jfs

namespace {
struct ZEScratch {
    std::mutex mu;
    uint64_t *d = nullptr;
    size_t cap = 0;  // waves
    uint8_t *aux = nullptr;  // BPAR work list, frame starts, block sizes
    size_t aux_cap = 0;
    int waves = 0;   // resident encoder waves on this device (BPAR grid)
    bool grow(size_t w) {
        if (d) (void)hipFree(d);  // hipFree synchronises with work still using it
        d = nullptr;
        cap = 0;
        if (hipMalloc((void **)&d, (size_t)jfs::zstde::SCR_PER * w) != hipSuccess) return false;
        cap = w;
        return true;
    }
};
// JFS_ZSTD_BPAR=0: one wave per frame (blocks in order) instead of one work
// item per 128 KiB block
bool zstd_bpar() {
    static const bool v = [] {
        const char *e = getenv("JFS_ZSTD_BPAR");
        return !(e && atoi(e) == 0);
    }();
    return v;
}
ZEScratch g_zes[16];
}  // namespace

#ifdef JFS_PROF
extern "C" int jfs_zeprof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::zstde::g_zeprof), sizeof(unsigned long long) * 12) == hipSuccess ? 0 : -1;
}
extern "C" int jfs_zeprof_reset() {
    unsigned long long z[12] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::zstde::g_zeprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int jfs_launch_zstd_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    using namespace jfs::zstde;
    if (nblk <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
    ZEScratch &z = g_zes[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (!zstd_bpar()) {
        if (z.cap < (size_t)nblk && !z.grow((size_t)nblk)) return -1;
        hipLaunchKernelGGL(zstd_encode_kernel<false>, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret, z.d,
                           (const int2 *)nullptr, 0, (int32_t *)nullptr);
        if (hipGetLastError() != hipSuccess) return -1;
        // the scratch is shared by every launch on this device: finish before it is reused
        return hipStreamSynchronize(stream) == hipSuccess ? 0 : -1;
    }
    // block-parallel: one work item per 128 KiB block (the descriptors may
    // have been written on this stream: read them after it drains)
    std::vector<jfs_dev_block> h(nblk);
    if (hipMemcpyAsync(h.data(), d_blocks, sizeof(jfs_dev_block) * nblk, hipMemcpyDeviceToHost, stream) != hipSuccess ||
        hipStreamSynchronize(stream) != hipSuccess)
        return -1;
    std::vector<int2> work;
    std::vector<int32_t> first(nblk + 1);
    for (int f = 0; f < nblk; f++) {
        first[f] = (int32_t)work.size();
        const int64_t n = h[f].src_len;
        const int64_t nb = n <= 0 ? 1 : (n + BLK - 1) / BLK;
        for (int64_t k = 0; k < nb; k++) work.push_back(make_int2(f, (int)k));
    }
    first[nblk] = (int32_t)work.size();
    const int nwork = (int)work.size();
    if (z.waves == 0) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, zstd_encode_kernel<true>, 64, 0) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return -1;
        z.waves = std::max(1, per_cu) * std::max(1, cus);
    }
    const int grid = std::min(nwork, z.waves);
    if (z.cap < (size_t)grid && !z.grow((size_t)grid)) return -1;
    const size_t wb = sizeof(int2) * nwork, fb = sizeof(int32_t) * (nblk + 1), sb = sizeof(int32_t) * nwork;
    if (z.aux_cap < wb + fb + sb) {
        if (z.aux) (void)hipFree(z.aux);
        z.aux = nullptr;
        z.aux_cap = 0;
        if (hipMalloc((void **)&z.aux, wb + fb + sb) != hipSuccess) return -1;
        z.aux_cap = wb + fb + sb;
    }
    int2 *d_work = (int2 *)z.aux;
    int32_t *d_first = (int32_t *)(z.aux + wb), *d_bsize = (int32_t *)(z.aux + wb + fb);
    if (hipMemcpyAsync(d_work, work.data(), wb, hipMemcpyHostToDevice, stream) != hipSuccess ||
        hipMemcpyAsync(d_first, first.data(), fb, hipMemcpyHostToDevice, stream) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(zstd_encode_kernel<true>, dim3(grid), dim3(64), 0, stream, d_blocks, nblk, d_ret, z.d,
                       (const int2 *)d_work, nwork, d_bsize);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zstd_compact_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret,
                       (const int32_t *)d_bsize, (const int32_t *)d_first);
    if (hipGetLastError() != hipSuccess) return -1;
    // the scratch and the host work list are shared / local: finish first
    return hipStreamSynchronize(stream) == hipSuccess ? 0 : -1;
}
