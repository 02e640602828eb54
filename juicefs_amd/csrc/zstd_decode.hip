// Zstd frame decoder for gfx950 (RFC 8878; behaviour of ZSTD_decompress as
// reached from pkg/compress/compress.go:94-103 via DataDog/zstd v1.5.6).
//
// Kernels per batch of inputs (one jfs_dev_block = one input buffer, which
// may hold several frames):
//
//  zscan / zplan  one lane per input walks frame/block/literal/sequence
//                 headers and sizes the scratch exactly; device-side scans
//                 place every input's literal, table and item ranges.
//  zlit           one wave per input decodes the literal sections (Huffman 4
//                 streams, two blocks at a time; raw, RLE) into the literal
//                 buffer.
//  zseqa          one wave per input walks the block headers and parks each
//                 compressed block's FSE table descriptions and descriptor.
//  zbuild         one wave per table spreads the FSE tables (position-parallel).
//  zseqb          two workgroups per input (blocks [0, ZNB) and the rest), two
//                 waves each: a decoder wave decodes ZNB blocks' sequence
//                 streams at once (one lane per block) from LDS, a mover wave
//                 keeps their bitstream rings filled; repeat offsets are
//                 symbolic per block and resolved in block order (phase C).
//  zexec          one wave per input replays the items (literal copy + match
//                 copy) through an 8 KiB LDS output ring, streams the output
//                 to HBM, checks content size / checksum, writes the result.
// Batches of at most JFS_ZSTD_SPLIT_MAX inputs take the block-parallel path of
// zstd_split.inc instead (same items, origin-map replay).
//
// Items are 16 bytes {x, y, z, kind}; errors found by the entropy waves are
// placed in stream order so zexec reports the first error libzstd would.
// Result codes match oracle/zstd_oracle.c: size, -1 corrupt, -2 dst too
// small, -3 source size wrong.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace zstdd {

#ifdef JFS_PROF
// diagnostic build only: cycle sums / counts of the sequence wave
__device__ unsigned long long g_zprof[8];
#define ZP_NOW() __builtin_amdgcn_s_memtime()
#define ZP_ADD(i, v) do { if (lane_id() == 0) atomicAdd(&g_zprof[i], (unsigned long long)(v)); } while (0)
#define XP_ADD(i, v) do { x.pacc[i] += (v); } while (0)
// zseq: 0 phase A (walk + tables), 1 table staging, 2 phase B decode, 3 phase C, 4 decoder barrier waits (v2), 5 groups
__device__ unsigned long long g_zsprof[8];
#define ZS_ADD(i, v) do { if (lane_id() == 0) atomicAdd(&g_zsprof[i], (unsigned long long)(v)); } while (0)
#else
#define ZS_ADD(i, v) do { } while (0)
#define XP_ADD(i, v) do { } while (0)
#define ZP_NOW() 0ull
#define ZP_ADD(i, v) do { } while (0)
#endif

enum { E_CORRUPT = -1, E_DSTSMALL = -2, E_SRCSIZE = -3, E_SCRATCH = -4, E_BUG = -100 };
enum { IT_SEQ = 0, IT_FSTART = 1, IT_FEND = 2, IT_BSTART = 3, IT_BEND = 4, IT_ERR = 5, IT_BREP = 6 };
// Offsets of sequence items may be symbolic: bit 31 set, bits 29-30 = j,
// bits 0-28 = d  ->  offset = max(1, rep_j - d) with rep_j the repeat-offset
// state at the start of the block (IT_BREP item).  Composition of libzstd's
// "rep0 - 1, and 0 becomes 1" steps is exactly max(1, x - d).
constexpr uint32_t SYMB = 0x80000000u;
enum { FE_FCS = 1, FE_CHECK = 2, FE_MISSING = 4 };
constexpr uint32_t ZSTD_MAGIC = 0xFD2FB528u;
constexpr int32_t BLOCK_MAX = 128 << 10;

// per-input bookkeeping
struct ZInfo {
    uint64_t item_off;      // first item (host scan)
    uint64_t lit_off;       // first literal byte (host scan)
    uint64_t tab_off;       // first FSE table cell (host scan)
    uint32_t n_items;       // zscan: capacity; zseq: items written
    uint32_t lit_bytes;     // zscan: capacity
    uint32_t n_cblk;        // zscan: compressed blocks (TAB_CELLS table cells each)
    uint32_t lit_err_blk;   // zlit: ordinal of the block whose literals failed
    int32_t lit_err_code;
    uint32_t ovf;           // zplan: the scratch cannot hold this input (ret = E_SCRATCH)
    uint32_t n_sblk;        // zseqa: compressed blocks described (ZDesc after each table area)
    uint32_t n_blk;         // zscan: blocks of every type (small-batch path: one record each)
    int32_t cap;            // zscan: the input's dst_cap
};
constexpr int TAB_CELLS = 1280;  // u16 FSE cells per compressed block: LL 512, OF 256, ML 512
constexpr int TAB_STRIDE = TAB_CELLS + 32;  // table area stride: the cells, then the block's ZDesc (64 B)

// a compressed block's sequence section, written by zseqa after its tables
struct ZDesc {
    uint64_t bs;             // sequence bitstream (absolute address)
    int32_t bsz, nseq;
    uint32_t item;           // BSTART item index (relative to the input)
    uint32_t tll, tof, tml;  // table cells relative to the input's first cell
    uint32_t al;             // al_ll | al_of << 8 | al_ml << 16 | frame-first << 24
    uint32_t rsv;
};
static_assert(sizeof(ZDesc) <= (TAB_STRIDE - TAB_CELLS) * 2, "ZDesc fits after the cells");

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

__host__ __device__ __forceinline__ uint32_t rd8(const gc_u8 *s, int32_t p) { return s[p]; }
__host__ __device__ __forceinline__ uint32_t rd16(const gc_u8 *s, int32_t p) { return s[p] | (s[p + 1] << 8); }
__host__ __device__ __forceinline__ uint32_t rd24(const gc_u8 *s, int32_t p) { return rd16(s, p) | (s[p + 2] << 16); }
__host__ __device__ __forceinline__ uint32_t rd32(const gc_u8 *s, int32_t p) { return rd16(s, p) | (rd16(s, p + 2) << 16); }

// ---------------------------------------------------------------------------
// frame / block walk (ZSTD_decompressMultiFrame + ZSTD_decompressFrame order)
// ---------------------------------------------------------------------------
enum { EV_DONE = 0, EV_ERROR, EV_FSTART, EV_FEND, EV_BLOCK };

struct Walk {
    const gc_u8 *s;
    int32_t n, p;
    int32_t cap;       // dst capacity (stop rule)
    int64_t lb;        // lower bound of the output produced so far
    int32_t phase;     // 0 between frames, 1 in a frame, 2 finished
    int32_t frames_done, after_last;
    int32_t check, has_fcs;
    uint64_t fcs;
    uint32_t ordinal;  // blocks seen
    // current block
    int32_t btype, bsize, bpos;
};

__host__ __device__ __forceinline__ void walk_init(Walk &w, const gc_u8 *s, int32_t n, int32_t cap) {
    w.s = s; w.n = n; w.p = 0; w.cap = cap; w.lb = 0; w.phase = 0; w.frames_done = 0; w.after_last = 0;
    w.check = 0; w.has_fcs = 0; w.fcs = 0; w.ordinal = 0; w.btype = 0; w.bsize = 0; w.bpos = 0;
}

// Next event.  *err for EV_ERROR; for EV_FEND *flags/*chk describe the frame end.
__host__ __device__ __forceinline__ int walk_next(Walk &w, int32_t *err, uint32_t *flags, uint32_t *chk) {
    const gc_u8 *s = w.s;
    if (w.phase == 2) return EV_DONE;
    if (w.phase == 1 && w.after_last) {
        w.after_last = 0;
        uint32_t f = (w.has_fcs ? FE_FCS : 0) | (w.check ? FE_CHECK : 0);
        *chk = 0;
        if (w.check) {
            if (w.n - w.p < 4) { f |= FE_MISSING; w.phase = 2; }
            else { *chk = rd32(s, w.p); w.p += 4; w.phase = 0; }
        } else {
            w.phase = 0;
        }
        w.frames_done = 1;
        *flags = f;
        return EV_FEND;
    }
    if (w.phase == 1) {
        if (w.lb > (int64_t)w.cap) { w.phase = 2; return EV_DONE; }  // zexec fails inside the last block
        if (w.n - w.p < 3) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
        uint32_t bh = rd24(s, w.p);
        w.p += 3;
        int32_t btype = (bh >> 1) & 3, bsize = (int32_t)(bh >> 3);
        if (btype == 3) { *err = E_CORRUPT; w.phase = 2; return EV_ERROR; }
        int32_t csize = btype == 1 ? 1 : bsize;
        if (csize > w.n - w.p) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
        if (btype == 2 && bsize >= BLOCK_MAX) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
        w.btype = btype; w.bsize = bsize; w.bpos = w.p;
        w.p += csize;
        w.after_last = bh & 1;
        w.ordinal++;
        return EV_BLOCK;
    }
    // between frames
    for (;;) {
        int32_t rem = w.n - w.p;
        if (rem < 5) {
            w.phase = 2;
            if (rem > 0) { *err = E_SRCSIZE; return EV_ERROR; }
            return EV_DONE;
        }
        uint32_t magic = rd32(s, w.p);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (rem < 8) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
            uint32_t sz = rd32(s, w.p + 4);
            if ((uint32_t)(rem - 8) < sz) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
            w.p += 8 + (int32_t)sz;
            continue;
        }
        if (rem < 9) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
        uint32_t fhd = rd8(s, w.p + 4);
        int32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
        int32_t did_size = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
        int32_t fcs_size = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        int32_t fhs = 5 + (single ? 0 : 1) + did_size + fcs_size;
        if (rem < fhs + 3) { *err = E_SRCSIZE; w.phase = 2; return EV_ERROR; }
        if (magic != ZSTD_MAGIC) { *err = w.frames_done ? E_SRCSIZE : E_CORRUPT; w.phase = 2; return EV_ERROR; }
        if (fhd & 8) { *err = E_CORRUPT; w.phase = 2; return EV_ERROR; }
        int32_t q = w.p + 5;
        if (!single) {
            if ((rd8(s, q) >> 3) + 10 > 31) { *err = E_CORRUPT; w.phase = 2; return EV_ERROR; }
            q++;
        }
        if (did) {
            uint32_t id = 0;
            for (int i = 0; i < did_size; i++) id |= rd8(s, q + i) << (8 * i);
            q += did_size;
            if (id != 0) { *err = E_CORRUPT; w.phase = 2; return EV_ERROR; }
        }
        w.has_fcs = fcs_size != 0;
        uint64_t v = 0;
        for (int i = 0; i < fcs_size; i++) v |= (uint64_t)rd8(s, q + i) << (8 * i);
        if (fcs_size == 2) v += 256;
        w.fcs = v;
        q += fcs_size;
        w.check = (fhd >> 2) & 1;
        w.p = q;
        w.phase = 1;
        w.after_last = 0;
        return EV_FSTART;
    }
}

// Literal section header (ZSTD_decodeLiteralsBlock size logic).  Returns 0 or
// an error; *sec = total bytes of the literal section.
struct LitHdr {
    int32_t type, regen, csize, hsz, streams, sec;
};
__host__ __device__ __forceinline__ int32_t lit_header(const gc_u8 *s, int32_t bpos, int32_t bsize, LitHdr &h) {
    if (bsize < 3) return E_CORRUPT;  // MIN_CBLOCK_SIZE
    uint32_t b0 = rd8(s, bpos);
    h.type = b0 & 3;
    int32_t sf = (b0 >> 2) & 3;
    h.streams = 1;
    h.csize = 0;
    if (h.type <= 1) {
        if (sf == 0 || sf == 2) { h.regen = b0 >> 3; h.hsz = 1; }
        else if (sf == 1) { h.regen = rd16(s, bpos) >> 4; h.hsz = 2; }
        else { h.regen = rd24(s, bpos) >> 4; h.hsz = 3; }
        if (h.type == 0) {
            if (h.hsz + h.regen > bsize) return E_CORRUPT;
            h.sec = h.hsz + h.regen;
        } else {
            if (h.hsz + 1 > bsize) return E_CORRUPT;
            if (h.regen > BLOCK_MAX) return E_CORRUPT;
            h.sec = h.hsz + 1;
        }
        return 0;
    }
    if (bsize < 5) return E_CORRUPT;
    uint32_t lhc = rd32(s, bpos);
    if (sf <= 1) {
        h.hsz = 3; h.streams = sf == 0 ? 1 : 4;
        h.regen = (lhc >> 4) & 0x3FF; h.csize = (lhc >> 14) & 0x3FF;
    } else if (sf == 2) {
        h.hsz = 4; h.streams = 4;
        h.regen = (lhc >> 4) & 0x3FFF; h.csize = lhc >> 18;
    } else {
        h.hsz = 5; h.streams = 4;
        h.regen = (lhc >> 4) & 0x3FFFF; h.csize = (lhc >> 22) + (rd8(s, bpos + 4) << 10);
    }
    if (h.regen > BLOCK_MAX) return E_CORRUPT;
    if (h.csize + h.hsz > bsize) return E_CORRUPT;
    h.sec = h.hsz + h.csize;
    return 0;
}

// nbSeq field (ZSTD_decodeSeqHeaders prefix).  Returns 0 or error; *nseq, *used.
__host__ __device__ __forceinline__ int32_t nbseq_header(const gc_u8 *s, int32_t ip, int32_t end, int32_t *nseq, int32_t *used) {
    if (ip >= end) return E_SRCSIZE;
    int32_t v = (int32_t)rd8(s, ip);
    int32_t u = 1;
    if (v >= 128) {
        if (v == 255) {
            if (ip + 3 > end) return E_SRCSIZE;
            v = (int32_t)rd16(s, ip + 1) + 0x7F00;
            u = 3;
        } else {
            if (ip + 2 > end) return E_SRCSIZE;
            v = ((v - 128) << 8) + (int32_t)rd8(s, ip + 1);
            u = 2;
        }
    }
    *nseq = v;
    *used = u;
    if (v == 0 && ip + u != end) return E_SRCSIZE;
    return 0;
}

// ---------------------------------------------------------------------------
// backward bit reader with a 2-block (32 B) prefetch queue (per lane)
// ---------------------------------------------------------------------------
// Positions are relative to b16 = the 16-byte aligned address at or below the
// stream start; the stream occupies bytes [m, m + size).  `left` = bit index
// one past the next unread bit.  Bits below 8m read as zero (libzstd
// BIT_DStream semantics for the sequence/Huffman streams).
struct BR {
    const gc_u4 *b16;
    int32_t m;      // stream start within b16
    int32_t lowk;   // lowest 16-byte block that may be loaded
    int32_t left;   // bits
    int32_t cb;     // container covers bytes [cb, cb+8), cb % 4 == 0
    uint64_t c;
    uint4 cur, pre, pre2;  // blocks k, k-1, k-2 where k = (cb - 4) >> 4
    int32_t ck;            // index of `cur`
};

__device__ __forceinline__ uint4 br_blk(const BR &r, int32_t k) {
    if (k < r.lowk) return make_uint4(0, 0, 0, 0);
    return r.b16[k];
}
// dword i of v without dynamic indexing (which would put v in scratch)
__device__ __forceinline__ uint32_t sel4(const uint4 &v, int32_t i) {
    uint32_t m0 = 0u - (uint32_t)(i == 0), m1 = 0u - (uint32_t)(i == 1);
    uint32_t m2 = 0u - (uint32_t)(i == 2), m3 = 0u - (uint32_t)(i == 3);
    return (v.x & m0) | (v.y & m1) | (v.z & m2) | (v.w & m3);
}
// shift dwords up by one (w <- z <- y <- x <- 0)
__device__ __forceinline__ void shup(uint4 &v) {
    v.w = v.z;
    v.z = v.y;
    v.y = v.x;
    v.x = 0;
}

// stream = [p, p + size) of an input that starts at `in` (loads never go below
// the 16-byte block holding `in`).  Returns false when the last byte is 0.
// `cur.w` is always the next dword to shift into the container.
__device__ __forceinline__ bool br_init(BR &r, const gc_u8 *in, const gc_u8 *p, int32_t size) {
    uintptr_t a = (uintptr_t)p;
    r.b16 = (const gc_u4 *)(a & ~(uintptr_t)15);
    r.m = (int32_t)(a & 15);
    r.lowk = -(int32_t)((((uintptr_t)r.b16) - (((uintptr_t)in) & ~(uintptr_t)15)) >> 4);
    if (size <= 0) return false;
    int32_t top = r.m + size;  // exclusive
    uint32_t last = ((const gc_u8 *)r.b16)[top - 1];
    if (last == 0) return false;
    int hb = 31 - __builtin_clz(last);
    r.left = 8 * (top - 1) + hb;
    r.cb = ((top - 1) & ~3) - 4;
    // container bytes [cb, cb+8): dwords at cb and cb+4
    int32_t k0 = r.cb >> 4, k1 = (r.cb + 4) >> 4;
    uint4 B0 = br_blk(r, k0), B1 = k1 == k0 ? B0 : br_blk(r, k1);
    uint32_t lo = sel4(B0, (r.cb >> 2) & 3), hi = sel4(B1, ((r.cb + 4) >> 2) & 3);
    r.c = ((uint64_t)hi << 32) | lo;
    r.ck = (r.cb - 4) >> 4;
    r.cur = r.ck == k0 ? B0 : br_blk(r, r.ck);
    int32_t j = ((r.cb - 4) >> 2) & 3;  // next dword's index in cur
    if (j < 3) shup(r.cur);
    if (j < 2) shup(r.cur);
    if (j < 1) shup(r.cur);
    r.pre = br_blk(r, r.ck - 1);
    r.pre2 = br_blk(r, r.ck - 2);
    return true;
}

__device__ __forceinline__ void br_refill(BR &r) {
    if (r.left - 8 * r.cb >= 32) return;
    int32_t nb = r.cb - 4;
    r.c = (r.c << 32) | r.cur.w;
    r.cb = nb;
    if ((nb & 15) == 0) {  // block exhausted: rotate the queue, prefetch one more
        r.cur = r.pre;
        r.pre = r.pre2;
        r.ck--;
        r.pre2 = br_blk(r, r.ck - 2);
    } else {
        shup(r.cur);
    }
}

__device__ __forceinline__ uint32_t br_peek(const BR &r, int n) {
    int32_t lo = r.left - n;
    uint32_t v = (uint32_t)(r.c >> (uint32_t)(lo - 8 * r.cb)) & ((1u << n) - 1u);
    int32_t d = 8 * r.m - lo;
    if (d > 0) v = d >= n ? 0u : v & ~((1u << d) - 1u);
    return v;
}
__device__ __forceinline__ bool br_done(const BR &r) { return r.left == 8 * r.m; }

// ---------------------------------------------------------------------------
// FSE tables (LDS, one u32 per cell: sym | nb << 8 | base << 16)
// ---------------------------------------------------------------------------
// forward LSB-first bit peek over a staged byte array
__device__ __forceinline__ uint32_t fpeek(const uint8_t *b, int32_t nbytes, int32_t pos, int n) {
    uint32_t v = 0;
    int32_t byte = pos >> 3;
    uint64_t w = 0;
    for (int i = 0; i < 5; i++) {
        int32_t q = byte + i;
        w |= (uint64_t)(q < nbytes ? b[q] : 0u) << (8 * i);
    }
    v = (uint32_t)(w >> (pos & 7)) & ((1u << n) - 1u);
    return v;
}

// FSE_readNCount over `stage` (nbytes valid).  Returns bytes used or -1.
__device__ __forceinline__ int32_t read_ncount(const uint8_t *stage, int32_t nbytes, int16_t *norm, int32_t *maxsym,
                                               int32_t *al, int32_t maxal) {
    if (nbytes < 1) return -1;
    int32_t pos = 0;
    int32_t nbBits = (int32_t)fpeek(stage, nbytes, 0, 4) + 5;
    pos = 4;
    if (nbBits > maxal) return -1;
    *al = nbBits;
    int32_t remaining = (1 << nbBits) + 1, threshold = 1 << nbBits;
    nbBits++;
    int32_t sym = 0, prev0 = 0, ms = *maxsym;
    for (int i = 0; i <= ms; i++) norm[i] = 0;
    const int32_t nbits = nbytes * 8;
    while (remaining > 1 && sym <= ms) {
        if (prev0) {
            int32_t n0 = sym;
            for (;;) {
                uint32_t r2 = fpeek(stage, nbytes, pos, 2);
                pos += 2;
                n0 += (int32_t)r2;
                if (r2 != 3) break;
                if (pos > nbits) return -1;
            }
            if (n0 > ms) return -1;
            while (sym < n0) norm[sym++] = 0;
            if (pos > nbits) return -1;
        }
        int32_t max = (2 * threshold - 1) - remaining;
        uint32_t v = fpeek(stage, nbytes, pos, nbBits);
        int32_t count;
        if ((int32_t)(v & (uint32_t)(threshold - 1)) < max) {
            count = (int32_t)(v & (uint32_t)(threshold - 1));
            pos += nbBits - 1;
        } else {
            count = (int32_t)(v & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= max;
            pos += nbBits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        norm[sym++] = (int16_t)count;
        prev0 = !count;
        while (remaining < threshold) { nbBits--; threshold >>= 1; }
        if (pos > nbits) return -1;
    }
    if (remaining != 1) return -1;
    *maxsym = sym - 1;
    return (pos + 7) >> 3;
}

// FSE decode table build (serial, wave-uniform).  symnext: >= 64 u16 scratch.
__device__ __forceinline__ int32_t build_fse(uint32_t *t, const int16_t *norm, int32_t maxsym, int32_t al,
                                             uint16_t *symnext, uint8_t *symat) {
    const int l = lane_id();
    int32_t size = 1 << al, high = size - 1;
    for (int s = 0; s <= maxsym; s++) {
        if (norm[s] == -1) {
            if (l == 0) symat[high] = (uint8_t)s;
            high--;
            if (l == 0) symnext[s] = 1;
        } else {
            if (l == 0) symnext[s] = (uint16_t)norm[s];
        }
    }
    int32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1, pos = 0;
    for (int s = 0; s <= maxsym; s++) {
        for (int i = 0; i < norm[s]; i++) {
            if (l == 0) symat[pos] = (uint8_t)s;
            do { pos = (pos + step) & mask; } while (pos > high);
        }
    }
    if (pos != 0) return -1;
    __builtin_amdgcn_wave_barrier();
    // baseline: ranks in cell order per symbol (serial; <= 512 cells)
    for (int u = 0; u < size; u++) {
        uint32_t s = symat[u];
        uint32_t ns = symnext[s];
        __builtin_amdgcn_wave_barrier();
        if (l == 0) symnext[s] = (uint16_t)(ns + 1);
        int nb = al - (31 - __builtin_clz(ns));
        if (l == 0) t[u] = s | ((uint32_t)nb << 8) | (((ns << nb) - (uint32_t)size) << 16);
        __builtin_amdgcn_wave_barrier();
    }
    return 0;
}

// ---------------------------------------------------------------------------
// kernel 1: header scan -> scratch sizes
// ---------------------------------------------------------------------------
// Scratch one input needs (exact): items, literal bytes, compressed blocks.
// Host and device: run_batch plans from the host copy of its inputs.
__host__ __device__ inline void zscan_one(const gc_u8 *src, int32_t n, int32_t cap, ZInfo &out) {
    Walk w;
    walk_init(w, src, n, cap);
    uint64_t items = 0, lits = 0;
    uint32_t cblk = 0;
    for (;;) {
        int32_t err = 0;
        uint32_t fl = 0, chk = 0;
        int ev = walk_next(w, &err, &fl, &chk);
        if (ev == EV_DONE) break;
        items++;  // FSTART / FEND / ERROR / BSTART
        if (ev == EV_ERROR) break;
        if (ev == EV_FEND && (fl & FE_MISSING)) break;
        if (ev != EV_BLOCK) continue;
        items++;  // BEND or ERR
        if (w.btype != 2) {
            items++;  // one literal-only item
            int64_t room = (int64_t)w.cap - w.lb;
            if ((int64_t)w.bsize <= room) lits += w.bsize;  // bytes past cap are never read
            w.lb += w.bsize;
            continue;
        }
        LitHdr h;
        if (lit_header(w.s, w.bpos, w.bsize, h)) break;
        lits += (uint64_t)h.regen + (h.type >= 2 ? 4 : 0);  // 4-stream segments may overhang by <= 3
        int32_t nseq = 0, used = 0;
        if (nbseq_header(w.s, w.bpos + h.sec, w.bpos + w.bsize, &nseq, &used)) break;
        items += (uint64_t)nseq + 1;  // sequences + BREP
        cblk++;
        w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
    }
    out.n_items = (uint32_t)(items + 1);
    out.lit_bytes = (uint32_t)(lits + 16);
    out.n_cblk = cblk;
    out.n_blk = w.ordinal;
    out.cap = cap;
}

__global__ void zscan_kernel(const jfs_dev_block *__restrict__ blocks, int nblk, ZInfo *__restrict__ info) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblk) return;
    jfs_dev_block b = blocks[i];
    zscan_one((const gc_u8 *)b.src, b.src_len, b.dst_cap, info[i]);
}

// Offsets of every input's scratch (exclusive prefix sums over the inputs,
// one workgroup), the capacity check, and the totals the launch needed
// (need[0..2] = items, literal bytes, table cells) -- so the host never waits
// for zscan: an input that does not fit the current scratch reports
// E_SCRATCH and the library grows the scratch for the next call.
constexpr int PLAN_T = 1024;
__global__ __launch_bounds__(PLAN_T) void zplan_kernel(ZInfo *__restrict__ info, int nblk, uint64_t cap_items,
                                                       uint64_t cap_lits, uint64_t cap_tabs,
                                                       uint64_t *__restrict__ need) {
    __shared__ uint64_t sh[3][PLAN_T];
    __shared__ unsigned long long xb, xo, xm;  // small-batch path: blocks, origin entries, largest cap
    const int t = threadIdx.x;
    if (t == 0) xb = xo = xm = 0;
    const int per = (nblk + PLAN_T - 1) / PLAN_T;
    const int b0 = t * per, b1 = b0 + per < nblk ? b0 + per : nblk;
    uint64_t a = 0, c = 0, d = 0;
    for (int i = b0; i < b1; i++) {
        a += info[i].n_items;
        c += (info[i].lit_bytes + 15u) & ~15u;
        d += (uint64_t)info[i].n_cblk * TAB_STRIDE;
    }
    uint64_t nbk = 0, norg = 0, mcap = 0;
    for (int i = b0; i < b1; i++) {
        const uint64_t c = info[i].cap > 0 ? (uint64_t)info[i].cap : 0u;
        nbk += info[i].n_blk;
        norg += (c + 3) & ~3ull;
        mcap = c > mcap ? c : mcap;
    }
    __syncthreads();
    if (nbk) atomicAdd(&xb, (unsigned long long)nbk);
    if (norg) atomicAdd(&xo, (unsigned long long)norg);
    if (mcap) atomicMax(&xm, (unsigned long long)mcap);
    sh[0][t] = a;
    sh[1][t] = c;
    sh[2][t] = d;
    __syncthreads();
    for (int o = 1; o < PLAN_T; o <<= 1) {  // inclusive scan (Hillis-Steele)
        uint64_t x0 = 0, x1 = 0, x2 = 0;
        if (t >= o) { x0 = sh[0][t - o]; x1 = sh[1][t - o]; x2 = sh[2][t - o]; }
        __syncthreads();
        sh[0][t] += x0;
        sh[1][t] += x1;
        sh[2][t] += x2;
        __syncthreads();
    }
    uint64_t oi = sh[0][t] - a, ol = sh[1][t] - c, ot = sh[2][t] - d;
    for (int i = b0; i < b1; i++) {
        ZInfo &z = info[i];
        z.item_off = oi;
        z.lit_off = ol;
        z.tab_off = ot;
        z.lit_err_blk = 0xFFFFFFFFu;
        z.lit_err_code = 0;
        oi += z.n_items;
        ol += (z.lit_bytes + 15u) & ~15u;
        ot += (uint64_t)z.n_cblk * TAB_STRIDE;
        z.ovf = (oi + 64 > cap_items || ol + 4096 + 64 > cap_lits || ot + 64 > cap_tabs) ? 1u : 0u;
    }
    if (t == PLAN_T - 1) {
        need[0] = sh[0][t];
        need[1] = sh[1][t];
        need[2] = sh[2][t];
        need[3] = xb;
        need[4] = xo;
        need[5] = xm;
    }
}

// ---------------------------------------------------------------------------
// kernel 2: entropy decode (wave 0 literals, wave 1 sequences)
// ---------------------------------------------------------------------------
struct LitSmem {
    alignas(16) uint16_t huf[4096];  // sym | nb << 8
    uint8_t stage[256];
    uint8_t w[260];
    int16_t norm[256];
    uint8_t symat[64];
    uint16_t symnext[256];
    uint32_t fse[64];    // weight FSE table (al <= 6)
    uint32_t rank[16];
    int32_t cur;     // current Huffman table: -1 none, 0 / 1 cells [0, 2048) / [2048, 4096), 2 all 4096 (12 bits)
    int32_t smb[3];  // max bits of the table in each of those places
};
__device__ __forceinline__ void lit_set_cur(LitSmem &sm, int32_t place, int32_t maxbits) {
    sm.cur = place;  // (uniform stores)
    sm.smb[place] = maxbits;
    __builtin_amdgcn_wave_barrier();
}
// stage `n` (<= 256) bytes starting at s+p into LDS (zero-padded)
__device__ __forceinline__ void stage_bytes(uint8_t *dst, const gc_u8 *s, int32_t p, int32_t n) {
    const int l = lane_id();
    for (int k = l; k < 256; k += 64) dst[k] = k < n ? s[p + k] : 0;
    __builtin_amdgcn_wave_barrier();
}

template <class P>
__device__ __forceinline__ void build_seq_fse_g(P t, const int16_t *norm, int32_t maxsym, int32_t al,
                                                uint8_t *mark, uint8_t *ksym, uint8_t *symat);
// Huffman table description -> sm.huf at cell 2048 * slot (a 12-bit table:
// cell 0, all 4096 cells).  Returns bytes used, -1 (corrupt) or -2 (a 12-bit
// table with narrow_only: nothing written to the table cells).
__device__ __forceinline__ int32_t read_huf(LitSmem &sm, const gc_u8 *in, const gc_u8 *s, int32_t p, int32_t n,
                                           int slot, bool narrow_only, int32_t *maxbits_out) {
    const int l = lane_id();
    if (n < 1) return -1;
    int32_t hb = (int32_t)rd8(s, p);
    int32_t nw = 0, used;
    if (hb < 128) {
        if (hb + 1 > n) return -1;
        stage_bytes(sm.stage, s, p + 1, hb);
        int32_t maxsym = 255, al = 0;
        int32_t c = read_ncount(sm.stage, hb, sm.norm, &maxsym, &al, 6);
        if (c < 0 || c > hb) return -1;
        if (maxsym > 63) {
            // (only a damaged description counts a weight symbol >= 64: the
            // lane-parallel builder holds one symbol per lane, so take the
            // serial spread of oracle/zstd_oracle.c and libzstd)
            if (build_fse(sm.fse, sm.norm, maxsym, al, sm.symnext, sm.symat)) return -1;
        } else {
            // the weight table by the lane-parallel sequence-table builder (u16
            // cells sym | state << 6 into symnext; sm.w is free until the weights
            // are decoded), then expanded to sym | nb << 8 | base << 16
            build_seq_fse_g(sm.symnext, sm.norm, maxsym, al, sm.w, sm.w + 128, sm.symat);
            if (l < (1 << al)) {
                const uint32_t v = sm.symnext[l], ns = v >> 6;
                const int nb = al - (31 - __builtin_clz(ns));
                sm.fse[l] = (v & 63u) | ((uint32_t)nb << 8) | (((ns << nb) - (1u << al)) << 16);
            }
        }
        __builtin_amdgcn_wave_barrier();
        // the weight stream (<= 127 bytes, staged) as dword q in lane q and the
        // weight FSE table (<= 64 cells) as cell i in lane i: the serial
        // decode reads both with readlane, no memory round trip per weight
        const int32_t len = hb - c;
        if (len <= 0) return -1;
        const uint32_t last = sm.stage[hb - 1];
        if (last == 0) return -1;
        uint32_t dv = 0;
        for (int k = 0; k < 4; k++) {
            const int32_t i = c + 4 * l + k;
            if (4 * l + k < len) dv |= (uint32_t)sm.stage[i] << (8 * k);
        }
        const uint32_t fv = l < (1 << al) ? sm.fse[l] : 0u;
        int32_t left = 8 * (len - 1) + (31 - __builtin_clz(last));
        auto bread = [&](uint32_t nb) -> uint32_t {  // bits [left - nb, left), 0 below the stream start
            const int32_t lo = left - (int32_t)nb;
            left = lo;
            if (nb == 0) return 0u;
            const int32_t q = lo >> 5;
            const uint32_t d0 = q >= 0 ? readlane(dv, q) : 0u;
            const uint32_t d1 = q + 1 < 32 ? readlane(dv, q + 1) : 0u;
            const uint64_t w64 = ((uint64_t)d1 << 32) | d0;
            return (uint32_t)(w64 >> (uint32_t)(lo - 32 * q)) & ((1u << nb) - 1u);
        };
        uint32_t s1 = bread((uint32_t)al), s2 = bread((uint32_t)al);
        for (;;) {
            if (nw > 253) return -1;
            const uint32_t e1 = readlane(fv, (int)s1);
            if (l == 0) sm.w[nw] = (uint8_t)(e1 & 0xFF);
            nw++;
            s1 = (e1 >> 16) + bread((e1 >> 8) & 0xFF);
            if (left < 0) { if (l == 0) sm.w[nw] = (uint8_t)(readlane(fv, (int)s2) & 0xFF); nw++; break; }
            if (nw > 253) return -1;
            const uint32_t e2 = readlane(fv, (int)s2);
            if (l == 0) sm.w[nw] = (uint8_t)(e2 & 0xFF);
            nw++;
            s2 = (e2 >> 16) + bread((e2 >> 8) & 0xFF);
            if (left < 0) { if (l == 0) sm.w[nw] = (uint8_t)(readlane(fv, (int)s1) & 0xFF); nw++; break; }
        }
        used = 1 + hb;
    } else {
        nw = hb - 127;
        int32_t bytes = (nw + 1) / 2;
        if (1 + bytes > n) return -1;
        stage_bytes(sm.stage, s, p + 1, bytes);
        for (int i = l; i < nw; i += 64) {
            uint32_t b = sm.stage[i / 2];
            sm.w[i] = (uint8_t)((i & 1) ? (b & 15) : (b >> 4));
        }
        used = 1 + bytes;
    }
    __builtin_amdgcn_wave_barrier();
    // weight statistics (lanes over symbols)
    uint32_t sum = 0, r1 = 0, bad = 0;
    for (int i = l; i < nw; i += 64) {
        uint32_t wi = sm.w[i];
        bad |= wi >= 12;
        sum += wi ? (1u << (wi - 1)) : 0u;
        r1 += wi == 1;
    }
    sum = dwave_sum(sum);
    r1 = dwave_sum(r1);
    bad = dwave_max(bad);
    if (bad || sum == 0) return -1;
    int32_t maxbits = 32 - __builtin_clz(sum);
    if (maxbits > 12) return -1;
    uint32_t rest = (1u << maxbits) - sum;
    if (rest & (rest - 1)) return -1;
    uint32_t lastw = (31 - __builtin_clz(rest)) + 1;
    if (l == 0) sm.w[nw] = (uint8_t)lastw;
    r1 += lastw == 1;
    nw++;
    if (r1 < 2 || (r1 & 1)) return -1;
    if (maxbits == 12 && narrow_only) return -2;
    const uint32_t hbase = maxbits == 12 ? 0u : 2048u * (uint32_t)slot;
    __builtin_amdgcn_wave_barrier();
    // every symbol's ordinal in (weight, symbol) order and its first cell:
    // lanes over symbols (four rounds), one ballot per weight and round
    uint32_t wv[4], ordv[4], posv[4];
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int i = l + 64 * r;
        wv[r] = i < nw ? (uint32_t)sm.w[i] : 0u;
        ordv[r] = posv[r] = 0;
    }
    uint32_t run = 0, done = 0;  // first cell / first ordinal of weight k's symbols
#pragma unroll
    for (uint32_t k = 1; k <= 12; k++) {
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const uint64_t m = __builtin_amdgcn_ballot_w64(wv[r] == k);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (wv[r] == k) {
                ordv[r] = done + c + below;
                posv[r] = run + ((c + below) << (k - 1));
            }
            c += (uint32_t)__builtin_popcountll(m);
        }
        run += c << (k - 1);
        done += c;
    }
    // markers: a symbol's first cell holds its ordinal + 1, the others 0;
    // symnext[ordinal] = the symbol's entry
    const uint32_t size = 1u << maxbits;
    uint16_t *ht = sm.huf + hbase;
    for (uint32_t u = 8u * (uint32_t)l; u < size; u += 512u) *(uint4 *)(ht + u) = make_uint4(0, 0, 0, 0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; r++) {
        if (wv[r]) {
            ht[posv[r]] = (uint16_t)(ordv[r] + 1u);
            sm.symnext[ordv[r]] = (uint16_t)((uint32_t)(l + 64 * r) | ((uint32_t)(maxbits + 1) - wv[r]) << 8);
        }
    }
    __builtin_amdgcn_wave_barrier();
    // every cell: the entry of the last marker at or below it (prefix max,
    // lanes over consecutive pieces)
    const uint32_t per = size >= 64u ? size >> 6 : 1u, q0 = (uint32_t)l * per;
    uint32_t lm = 0;
    for (uint32_t i = 0; i < per; i++)
        if (q0 + i < size) lm = umax32(lm, ht[q0 + i]);
    uint32_t carry = dpp_shift_up(dpp_scan_max(lm), 0u);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = 0; i < per; i++) {
        if (q0 + i < size) {
            carry = umax32(carry, ht[q0 + i]);
            ht[q0 + i] = sm.symnext[carry - 1u];
        }
    }
    __builtin_amdgcn_wave_barrier();
    *maxbits_out = maxbits;
    __builtin_amdgcn_wave_barrier();
    return used;
}

// lane-parallel byte stores into the literal buffer
__device__ __forceinline__ void put_word(g_u8 *lb, int64_t start, int64_t end4, uint32_t acc) {
    // bytes [end4-4, end4) of which those >= start are valid
    if (end4 - 4 >= start) {
        *(g_u32 *)(lb + end4 - 4) = acc;
    } else {
        for (int64_t q = start; q < end4; q++) lb[q] = (uint8_t)(acc >> (8 * (q & 3)));
    }
}

// A Huffman literal section ready to decode: the stream section (jump table
// and streams) and the table it uses.
struct LJob {
    int32_t p, n;          // stream section within s
    int32_t regen, streams;
    int64_t lpos;          // first output byte in the literal buffer
    int32_t hb, mb;        // table cell base, max bits
};

// Lanes 4j..4j+3 decode job j's streams (j < nj <= 2).  Returns bit j set
// when job j is corrupt.
__device__ __forceinline__ uint32_t lit_decode(LitSmem &sm, const gc_u8 *in, const gc_u8 *s, g_u8 *lb,
                                               const LJob &j0, const LJob &j1, int nj) {
    const int l = lane_id();
    const int jj = l >> 2, sl = l & 3;
    const bool mine = jj < nj;
    const int32_t p = jj ? j1.p : j0.p, n = jj ? j1.n : j0.n, regen = jj ? j1.regen : j0.regen;
    const int32_t streams = jj ? j1.streams : j0.streams, hb = jj ? j1.hb : j0.hb;
    const int32_t maxbits = jj ? j1.mb : j0.mb;
    const int64_t lpos = jj ? j1.lpos : j0.lpos;
    // stream geometry (lane sl < streams decodes stream sl)
    int32_t mysp = p, mysn = n, mycnt = regen;
    int64_t o = lpos;
    int32_t bad = 0;
    if (mine && streams == 4) {
        int32_t s4 = 0, s1 = 0, s2 = 0, s3 = 0;
        if (n < 10) {
            bad = 1;
        } else {
            s1 = (int32_t)rd16(s, p); s2 = (int32_t)rd16(s, p + 2); s3 = (int32_t)rd16(s, p + 4);
            s4 = n - 6 - s1 - s2 - s3;
            if (s4 < 1) bad = 1;
        }
        const int32_t seg = (regen + 3) / 4;
        mysp = p + 6 + (sl >= 1 ? s1 : 0) + (sl >= 2 ? s2 : 0) + (sl >= 3 ? s3 : 0);
        mysn = sl == 0 ? s1 : sl == 1 ? s2 : sl == 2 ? s3 : s4;
        const int32_t c4 = regen - 3 * seg;
        mycnt = sl < 3 ? seg : (c4 > 0 ? c4 : 0);
        o = lpos + (int64_t)(sl < 3 ? sl : 3) * seg;
    }
    if (mine && sl < streams && !bad) {
        BR r;
        if (!br_init(r, in, s + mysp, mysn)) {
            bad = 1;
        } else {
            const int64_t start = o, end = o + mycnt;
            uint32_t acc = 0;
            // one symbol: peek, table, consume (no refill: a refill leaves >= 32
            // bits in the container, two symbols take <= 24)
            auto sym = [&]() -> uint32_t {
                const uint32_t e = sm.huf[hb + br_peek(r, maxbits)];
                r.left -= (int32_t)(e >> 8);
                return e & 0xFFu;
            };
            // head: up to the first 4-byte-aligned output position
            for (; o < end && (o & 3); o++) {
                acc |= sym() << (8 * (o & 3));
                br_refill(r);
                if (((o + 1) & 3) == 0) { put_word(lb, start, o + 1, acc); acc = 0; }
            }
            // body: four symbols, two refills and one aligned word store per
            // step; while the stream has 4 x maxbits bits above its start no
            // read can reach below it, and the peek needs no start check
            const int32_t fastlim = 8 * r.m + 4 * maxbits;
            const uint32_t pmask = (1u << maxbits) - 1u;
            auto fsym = [&]() -> uint32_t {
                const int32_t lo = r.left - maxbits;
                const uint32_t e = sm.huf[hb + ((uint32_t)(r.c >> (uint32_t)(lo - 8 * r.cb)) & pmask)];
                r.left -= (int32_t)(e >> 8);
                return e & 0xFFu;
            };
            for (; o + 4 <= end; o += 4) {
                uint32_t w;
                if (r.left >= fastlim) {
                    w = fsym();
                    w |= fsym() << 8;
                    br_refill(r);
                    w |= fsym() << 16;
                    w |= fsym() << 24;
                } else {
                    w = sym();
                    w |= sym() << 8;
                    br_refill(r);
                    w |= sym() << 16;
                    w |= sym() << 24;
                }
                br_refill(r);
                *(g_u32 *)(lb + o) = w;
            }
            for (; o < end; o++) {
                acc |= sym() << (8 * (o & 3));
                br_refill(r);
            }
            if (o & 3) {
                for (int64_t q = (o & ~3LL) > start ? (o & ~3LL) : start; q < o; q++) lb[q] = (uint8_t)(acc >> (8 * (q & 3)));
            }
            if (!br_done(r)) bad = 1;
        }
    }
    const uint64_t bm = __ballot(bad != 0);
    return ((bm & 0xFull) ? 1u : 0u) | ((bm & 0xF0ull) ? 2u : 0u);
}

__device__ __forceinline__ int32_t lit_block(LitSmem &sm, const gc_u8 *in, const gc_u8 *s, const LitHdr &h, int32_t bpos,
                             g_u8 *lb, int64_t lpos) {
    const int l = lane_id();
    if (h.type == 0) {
        for (int32_t k = l; k < h.regen; k += 64) lb[lpos + k] = s[bpos + h.hsz + k];
        return 0;
    }
    if (h.type == 1) {
        uint8_t v = (uint8_t)rd8(s, bpos + h.hsz);
        for (int32_t k = l; k < h.regen; k += 64) lb[lpos + k] = v;
        return 0;
    }
    int32_t p = bpos + h.hsz, n = h.csize;
    LJob j;
    if (h.type == 2) {
        int32_t m = 0;
        int32_t u = read_huf(sm, in, s, p, n, 0, false, &m);
        if (u < 0) return E_CORRUPT;
        if (u >= n) return E_CORRUPT;  // table must leave room for the streams
        lit_set_cur(sm, m == 12 ? 2 : 0, m);
        p += u;
        n -= u;
        j.hb = 0;
        j.mb = m;
    } else {
        const int32_t c = sm.cur;
        if (c < 0) return E_CORRUPT;
        j.hb = c == 1 ? 2048 : 0;
        j.mb = sm.smb[c];
    }
    j.p = p; j.n = n; j.regen = h.regen; j.streams = h.streams; j.lpos = lpos;
    return lit_decode(sm, in, s, lb, j, j, 1) ? E_CORRUPT : 0;
}

// Two Huffman literal sections decoded together (lanes 0-3 and 4-7), their
// tables in the two halves of sm.huf.  Returns 0 (both decoded), 1 / 2 (the
// first / second is corrupt; the first error in block order) or -2: nothing
// decoded and the current table untouched unless the first block brings its
// own -- the caller decodes the two one by one (12-bit tables, errors in a
// table description, a treeless first block without a narrow table).
struct LPend {
    LitHdr h;
    int32_t bpos;
    uint32_t ord;
    int64_t lpos;
};
__device__ __forceinline__ int lit_pair(LitSmem &sm, const gc_u8 *s, g_u8 *lb, const LPend &A, const LPend &B) {
    LJob ja, jb;
    int32_t pa = A.bpos + A.h.hsz, na = A.h.csize, pb = B.bpos + B.h.hsz, nb = B.h.csize;
    int sa, sb;
    if (A.h.type == 2) {
        int32_t m = 0;
        const int32_t u = read_huf(sm, s, s, pa, na, 0, true, &m);
        if (u < 0 || u >= na) return -2;
        pa += u; na -= u; sa = 0; ja.mb = m;
    } else {
        const int32_t c = sm.cur;
        if (c < 0 || c == 2) return -2;
        sa = c; ja.mb = sm.smb[c];
    }
    if (B.h.type == 2) {
        int32_t m = 0;
        const int32_t u = read_huf(sm, s, s, pb, nb, sa ^ 1, true, &m);
        if (u < 0 || u >= nb) return -2;
        pb += u; nb -= u; sb = sa ^ 1; jb.mb = m;
    } else {
        sb = sa; jb.mb = ja.mb;
    }
    lit_set_cur(sm, sb, jb.mb);
    ja.p = pa; ja.n = na; ja.regen = A.h.regen; ja.streams = A.h.streams; ja.lpos = A.lpos; ja.hb = 2048 * sa;
    jb.p = pb; jb.n = nb; jb.regen = B.h.regen; jb.streams = B.h.streams; jb.lpos = B.lpos; jb.hb = 2048 * sb;
    const uint32_t bm = lit_decode(sm, s, s, lb, ja, jb, 2);
    return (bm & 1u) ? 1 : (bm & 2u) ? 2 : 0;
}

// sequence table for one field; returns bytes used or -1
__device__ __forceinline__ void lit_wave(LitSmem &sm, const jfs_dev_block &b, ZInfo &zi, g_u8 *litbuf) {
    const int l = lane_id();
    const gc_u8 *s = (const gc_u8 *)b.src;
    Walk w;
    walk_init(w, s, b.src_len, b.dst_cap);
    int64_t lpos = (int64_t)zi.lit_off;
    const int64_t lend = (int64_t)zi.lit_off + zi.lit_bytes;
    uint32_t err_blk = 0xFFFFFFFFu;
    int32_t err_code = 0;
    if (l == 0) sm.cur = -1;
    __builtin_amdgcn_wave_barrier();
    // a Huffman section waiting for a partner (decoded before anything that
    // could report an error after it)
    LPend pd;
    bool hp = false;
    auto single = [&](const LPend &q) -> bool {
        const int32_t e = lit_block(sm, s, s, q.h, q.bpos, litbuf, q.lpos);
        if (e) { err_blk = q.ord; err_code = e; return false; }
        return true;
    };
    auto flush = [&]() -> bool {
        if (!hp) return true;
        hp = false;
        return single(pd);
    };
    for (;;) {
        int32_t err = 0;
        uint32_t fl = 0, chk = 0;
        int ev = walk_next(w, &err, &fl, &chk);
        if (ev == EV_DONE || ev == EV_ERROR) break;
        if (ev == EV_FSTART) {
            if (!flush()) break;
            if (l == 0) sm.cur = -1;
            __builtin_amdgcn_wave_barrier();
            continue;
        }
        if (ev == EV_FEND) {
            if (fl & FE_MISSING) break;
            continue;
        }
        const uint32_t ord = w.ordinal - 1;
        if (w.btype != 2) {
            int64_t room = (int64_t)w.cap - w.lb;
            if ((int64_t)w.bsize <= room) {
                if (lpos + w.bsize > lend) {
                    if (flush()) { err_blk = ord; err_code = -104; }
                    break;
                }
                if (w.btype == 0) {
                    for (int32_t k = l; k < w.bsize; k += 64) litbuf[lpos + k] = s[w.bpos + k];
                } else {
                    uint8_t v = (uint8_t)rd8(s, w.bpos);
                    for (int32_t k = l; k < w.bsize; k += 64) litbuf[lpos + k] = v;
                }
                lpos += w.bsize;
            }
            w.lb += w.bsize;
            continue;
        }
        LitHdr h;
        int32_t e = lit_header(s, w.bpos, w.bsize, h);
        if (e) {
            if (flush()) { err_blk = ord; err_code = e; }
            break;
        }
        if (lpos + h.regen + 4 > lend) {
            if (flush()) { err_blk = ord; err_code = -104; }
            break;
        }
        LPend q;
        q.h = h; q.bpos = w.bpos; q.ord = ord; q.lpos = lpos;
        if (h.type >= 2) {
            if (hp) {
                hp = false;
                const int r = lit_pair(sm, s, litbuf, pd, q);
                if (r == -2) {
                    if (!single(pd) || !single(q)) break;
                } else if (r) {
                    err_blk = r == 1 ? pd.ord : ord;
                    err_code = E_CORRUPT;
                    break;
                }
            } else {
                pd = q;
                hp = true;
            }
        } else if (!single(q)) {  // raw / RLE literals: no table, no error; never waits
            break;
        }
        lpos += h.regen;
        int32_t nseq = 0, used = 0;
        if (nbseq_header(s, w.bpos + h.sec, w.bpos + w.bsize, &nseq, &used)) break;  // reported by the seq wave
        w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
    }
    flush();
    if (l == 0) {
        zi.lit_err_blk = err_blk;
        zi.lit_err_code = err_code;
    }
}

__global__ __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(4)))
void zlit_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                  ZInfo *__restrict__ info, uint8_t *__restrict__ litbuf) {
    __shared__ LitSmem sm;
    const int bi = blockIdx.x;
    if (bi >= nblk) return;
    const jfs_dev_block b = blocks[bi];
    if (info[bi].ovf) return;
    lit_wave(sm, b, info[bi], (g_u8 *)litbuf);
}

// ---------------------------------------------------------------------------
// kernel 2b: sequences.  Phase A (wave-uniform) walks the headers, builds the
// FSE tables of each compressed block into global scratch and collects up to
// 64 blocks; phase B decodes those blocks' sequence streams one lane per block
// (repeat offsets tracked symbolically from the block's entry state); phase C
// resolves the entry states block by block (IT_BREP items).
// ---------------------------------------------------------------------------
typedef JFS_GLOBAL uint16_t g_u16;
typedef JFS_GLOBAL const uint16_t gc_u16;

struct GBlk {
    const gc_u8 *bs;   // sequence bitstream
    const gc_u8 *in;   // start of the input holding it
    g_u4 *ib;          // the input's item array
    int32_t bsz, nseq;
    uint32_t item;     // BSTART item index (relative to the input)
    uint64_t tll, tof, tml;  // table cells (absolute index into the table scratch)
    uint32_t al;       // al_ll | al_of << 8 | al_ml << 16 | frame-first << 24
};
// Inputs per sequence workgroup: a 4 MiB frame has 32 compressed blocks, so
// two inputs fill the 64 lanes of phase B.
constexpr int ZSEQ_INPUTS = 1;  // zseqb: one input per workgroup packs the CUs better (123.3 vs 125.9 ms)
// Round 3 (default): a workgroup of two waves.  Wave 0 walks the headers and
// builds each block's FSE tables straight into the group's LDS arena (phase
// A), then decodes the group's ZNB blocks (one lane each) with every table
// cell and bitstream byte read from LDS — it never waits on HBM; its item
// stores are fire-and-forget.  Wave 1 (the mover) keeps each lane's
// bitstream ring filled ahead of the decoder, one barrier per period of ZK2
// sequences.
// blocks per group = decoder lanes: 16 fit three workgroups per CU in LDS
// (12 fit four, one decoder wave per SIMD, but measured slower: 161-171 vs
// 152 ms on configs[3])
constexpr int ZNB = 16;
constexpr int ZMQ = 64 / ZNB < 4 ? 64 / ZNB : 4;  // mover lanes per block
constexpr int ZK2 = 8;  // sequences per period
constexpr int ZRB2 = 512;  // bitstream ring bytes per lane (blocks of 16 B)
constexpr int ZMD = 2;
constexpr int ZAHEAD = ZRB2 == 512 ? (ZMD == 2 ? 27 : 24) : ZRB2 / 16 - 2;  // ring blocks the mover keeps below the published position
// <= 89 bits per sequence: a period moves the position down <= 6 blocks and
// a refill window reaches 128 bits below it (one block more).  Loads issued
// in iteration p land during iteration p + ZMD and serve period p + ZMD + 1,
// whose reads reach (ZMD + 1) periods + 1 block below the position the
// target came from; and a landing block must not displace (32 slots) one the
// decoder still reads (<= 1 block above its position).
constexpr int ZPB = (ZK2 * 89 + 127) / 128;
constexpr int ZPRE = ZAHEAD + 3 < ZRB2 / 16 - 2 ? ZAHEAD + 3 : ZRB2 / 16 - 2;  // prefill depth below the top block
static_assert((ZMD + 1) * ZPB + 7 <= ZAHEAD && ZAHEAD <= ZRB2 / 16 - 2 && ZPB + 2 <= 8, "ring budget");
struct ASmem {  // zseqa: table-build scratch
    uint8_t stage[256];
    int16_t norm[64];
    uint8_t symat[512], mark[512], ksym[512];
};
struct SeqSmem {  // zseqb
    alignas(16) uint8_t bring[ZNB][ZRB2 + 16];   // per-lane bitstream rings (+ a mirror of block slot 0)
    alignas(16) uint16_t arena[ZNB][TAB_CELLS];  // the group's tables (LL 0, OF 512, ML 768)
    uint32_t lut_ll[36], lut_ml[53];
    uint8_t xb_ll[64], xb_ml[64];  // extra-bit counts alone (the state pass's chain)
    GBlk g[ZNB];
    int32_t pos[2][ZNB];  // decoder bit positions published at each period's barrier
    int32_t more[2];      // any lane still decoding (per period parity)
    int32_t cmd;          // wave 0 -> wave 1: blocks in the group, 0 = done
    uint2 rec[2][ZK2][ZNB];    // a period's sequences (period parity): bit position, states (sll | sof << 10 | sml << 20)
    uint32_t carry[3][ZNB];    // repeat offsets after the block's sequences so far (symbolic in its entry state)
    int32_t rcnt[2][ZNB];      // sequences recorded in the period
    uint32_t ibase[2][ZNB];    // sequence index of the period's first record
};
static_assert(sizeof(SeqSmem) * (ZNB <= 12 ? 4 : 3) <= 160 * 1024, "sequence workgroups per CU (one decoder wave per SIMD)");
static_assert(ZMQ == 4, "the mover serves each block with four lanes (stride-4 block loads)");

// u16 cell = sym | ns << 6  (nb = al - highbit(ns), next-state base = (ns << nb) - 2^al)
template <class P>
__device__ __forceinline__ void build_seq_fse_g(P t, const int16_t *norm, int32_t maxsym, int32_t al,
                                                uint8_t *mark, uint8_t *ksym, uint8_t *symat) {
    const int l = lane_id();
    const int32_t size = 1 << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    const int32_t nrm = l <= maxsym ? (int32_t)norm[l] : 0;
    const uint32_t cntp = nrm > 0 ? (uint32_t)nrm : 0u, low = nrm == -1 ? 1u : 0u;
    const uint32_t cum_i = dpp_scan_add(cntp), low_i = dpp_scan_add(low);
    const uint32_t cum = cum_i - cntp, lowrank = low_i - low;
    const int32_t nlow = (int32_t)readlane(low_i, 63);
    const int32_t high = size - 1 - nlow;
    const int32_t per = (size + 63) >> 6;
    for (int k = l; k < size; k += 64) mark[k] = 0;
    __builtin_amdgcn_wave_barrier();
    if (cntp > 0) mark[cum] = (uint8_t)(l + 1);
    if (low) symat[size - 1 - (int32_t)lowrank] = (uint8_t)l;
    __builtin_amdgcn_wave_barrier();
    const int32_t q0 = l * per;
    uint32_t lm = 0;
    for (int i = 0; i < per; i++)
        if (q0 + i < size) lm = umax32(lm, mark[q0 + i]);
    uint32_t carry = dpp_shift_up(dpp_scan_max(lm), 0u);
    for (int i = 0; i < per; i++) {
        if (q0 + i < size) {
            carry = umax32(carry, mark[q0 + i]);
            ksym[q0 + i] = (uint8_t)(carry - 1);
        }
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t nv = 0;
    for (int i = 0; i < per; i++) {
        int32_t j = q0 + i;
        if (j < size && ((j * step) & mask) <= high) nv++;
    }
    uint32_t k = dpp_scan_add(nv) - nv;
    for (int i = 0; i < per; i++) {
        int32_t j = q0 + i;
        int32_t pj = (j * step) & mask;
        if (j < size && pj <= high) { symat[pj] = ksym[k]; k++; }
    }
    __builtin_amdgcn_wave_barrier();
    // position-parallel: 64 cells per step; a cell's state is its symbol's
    // counter plus its rank among the step's cells of that symbol (one ballot
    // per distinct symbol in the step); one coalesced store per step
    uint32_t ns = nrm == -1 ? 1u : (uint32_t)nrm;  // lane s: symbol s's next state
    for (int c = 0; c < size; c += 64) {
        const int u = c + l;
        const uint32_t sym = u < size ? (uint32_t)symat[u] : 0xFFu;
        uint32_t cell = 0;
        for (uint64_t todo = __builtin_amdgcn_ballot_w64(u < size); todo;) {
            const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)sym, (int)__builtin_ctzll(todo));
            const uint64_t m = __builtin_amdgcn_ballot_w64(sym == s);
            const uint32_t base = (uint32_t)__builtin_amdgcn_readlane((int)ns, (int)s);
            const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (sym == s) cell = s | ((base + rk) << 6);
            if ((uint32_t)l == s) ns += (uint32_t)__builtin_popcountll(m);
            todo &= ~m;
        }
        if (u < size) t[u] = (uint16_t)cell;
    }
    __builtin_amdgcn_wave_barrier();
}

// one field's table; returns bytes used or -1.  cur/al/have: the field's state.
template <class SM, class P>
__device__ __forceinline__ int32_t seq_table_g(SM &sm, P tabs, uint32_t area, uint32_t *cur, int32_t *al,
                                               int32_t *have, int32_t mode, const gc_u8 *s, int32_t p, int32_t n,
                                               int which) {
    const int16_t *def = which == 0 ? LL_DEF : which == 1 ? OF_DEF : ML_DEF;
    int32_t maxsym = which == 0 ? 35 : which == 1 ? 31 : 52;
    int32_t defal = which == 1 ? 5 : 6, defmax = which == 0 ? 35 : which == 1 ? 28 : 52;
    int32_t maxal = which == 1 ? 8 : 9;
    const int l = lane_id();
    if (mode == 0) {
        for (int i = l; i <= defmax; i += 64) sm.norm[i] = def[i];
        __builtin_amdgcn_wave_barrier();
        build_seq_fse_g(tabs + area, sm.norm, defmax, defal, sm.mark, sm.ksym, sm.symat);
        *cur = area; *al = defal; *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (n < 1) return -1;
        uint32_t v = rd8(s, p);
        if ((int32_t)v > maxsym) return -1;
        if (l == 0) tabs[area] = (uint16_t)(v | (1u << 6));
        *cur = area; *al = 0; *have = 1;
        return 1;
    }
    if (mode == 2) {
        int32_t k = n < 256 ? n : 256;
        stage_bytes(sm.stage, s, p, k);
        int32_t ms = maxsym, a = 0;
        int32_t c = read_ncount(sm.stage, k, sm.norm, &ms, &a, maxal);
        if (c < 0 || c > n) return -1;
        __builtin_amdgcn_wave_barrier();
        build_seq_fse_g(tabs + area, sm.norm, ms, a, sm.mark, sm.ksym, sm.symat);
        *cur = area; *al = a; *have = 1;
        return c;
    }
    return *have ? 0 : -1;
}

// A deferred table's normalized counts wait in the last 64 cells of its own
// region (zbuild reads them into registers before spreading over the region);
// ZDesc.rsv carries per field maxsym (6 bits at 6f) and the build kind
// (2 bits at 18 + 2f: 1 stored counts, 2 predefined).
__device__ __forceinline__ uint32_t zfield_cells(int f) { return f == 1 ? 256u : 512u; }
template <class SM>
__device__ __forceinline__ int32_t seq_table_defer(SM &sm, g_u16 *tabs, uint32_t area, uint32_t *cur, int32_t *al,
                                                   int32_t *have, int32_t mode, const gc_u8 *s, int32_t p, int32_t n,
                                                   int which, uint32_t *rs) {
    int32_t maxsym = which == 0 ? 35 : which == 1 ? 31 : 52;
    int32_t defal = which == 1 ? 5 : 6, defmax = which == 0 ? 35 : which == 1 ? 28 : 52;
    int32_t maxal = which == 1 ? 8 : 9;
    const int l = lane_id();
    if (mode == 0) {
        *rs |= ((uint32_t)defmax << (6 * which)) | (2u << (18 + 2 * which));
        *cur = area; *al = defal; *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (n < 1) return -1;
        uint32_t v = rd8(s, p);
        if ((int32_t)v > maxsym) return -1;
        if (l == 0) tabs[area] = (uint16_t)(v | (1u << 6));
        *cur = area; *al = 0; *have = 1;
        return 1;
    }
    if (mode == 2) {
        int32_t k = n < 256 ? n : 256;
        stage_bytes(sm.stage, s, p, k);
        int32_t ms = maxsym, a = 0;
        int32_t c = read_ncount(sm.stage, k, sm.norm, &ms, &a, maxal);
        if (c < 0 || c > n) return -1;
        __builtin_amdgcn_wave_barrier();
        if (l <= ms) tabs[area + zfield_cells(which) - 64 + l] = (uint16_t)sm.norm[l];
        *rs |= ((uint32_t)ms << (6 * which)) | (1u << (18 + 2 * which));
        *cur = area; *al = a; *have = 1;
        return c;
    }
    return *have ? 0 : -1;
}

__device__ __forceinline__ uint32_t rep_res(uint32_t v, uint32_t e0, uint32_t e1, uint32_t e2) {
    if (!(v & SYMB)) return v;
    uint32_t j = (v >> 29) & 3, d = v & 0x1FFFFFFFu;
    uint32_t e = j == 0 ? e0 : j == 1 ? e1 : e2;
    return e > d + 1 ? e - d : 1u;
}


// LDS-only barrier between the decoder and mover waves (the decoder's item
// stores stay in flight)
__device__ __forceinline__ void zsync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Geometry of a block's sequence bitstream in 16-byte blocks relative to the
// aligned base b16: bytes [m, m + bsz); blocks below lowk precede the input.
struct ZGeo {
    const gc_u4 *b16;
    int32_t m, top, kt, lowk;
};
__device__ __forceinline__ ZGeo zgeo(const GBlk &d) {
    ZGeo g;
    const uintptr_t a = (uintptr_t)d.bs;
    g.b16 = (const gc_u4 *)(a & ~(uintptr_t)15);
    g.m = (int32_t)(a & 15);
    g.top = g.m + d.bsz;
    g.kt = (g.top - 1) >> 4;
    g.lowk = -(int32_t)((((uintptr_t)g.b16) - (((uintptr_t)d.in) & ~(uintptr_t)15)) >> 4);
    return g;
}
// a ring slot write; slot 0 is mirrored after the ring so that a refill's
// four dwords never wrap
__device__ __forceinline__ void zr_put(uint8_t *ring, int32_t k, const uint4 &v) {
    const int32_t sl = k & (ZRB2 / 16 - 1);
    *(uint4 *)(ring + (sl << 4)) = v;
    if (sl == 0) *(uint4 *)(ring + ZRB2) = v;
}
// Refill: bits [left - 96, left) from the ring (one round of four LDS dword
// reads; the mover wrote zeros below the stream start, so bits there read as
// zero, like the bit readers above).  hi = bits [left - 64, left), lo = bits [left - 96, left - 64).
__device__ __forceinline__ void zw_fill(const uint8_t *ring, int32_t left, uint64_t &hi, uint32_t &lo) {
    const int32_t cb = ((left - 96) >> 5) << 2;  // 8 * cb in (left - 128, left - 96]
    const uint32_t *w = (const uint32_t *)(ring + (cb & (ZRB2 - 1)));  // + 16 bytes: the mirror
    const uint32_t d0 = w[0], d1 = w[1], d2 = w[2], d3 = w[3];
    const uint64_t A = ((uint64_t)d1 << 32) | d0, B = ((uint64_t)d3 << 32) | d2;
    const int32_t t = left - 8 * cb - 64;  // [32, 64)
    hi = (A >> t) | (B << (64 - t));
    lo = (uint32_t)(A >> (t - 32));
}
// a ring block as the decoder must see it: blocks before the stream's
// first byte (k < 0, and bytes [0, m) of block 0) read as zero
__device__ __forceinline__ uint4 zclip(uint4 v, int32_t k, int32_t m) {
    if (k < 0) return make_uint4(0, 0, 0, 0);
    if (k == 0 && m > 0) {
        const int32_t b0 = m, b1 = m - 4, b2 = m - 8, b3 = m - 12;
        v.x = b0 >= 4 ? 0u : v.x & (~0u << (8 * b0));
        v.y = b1 >= 4 ? 0u : b1 <= 0 ? v.y : v.y & (~0u << (8 * b1));
        v.z = b2 >= 4 ? 0u : b2 <= 0 ? v.z : v.z & (~0u << (8 * b2));
        v.w = b3 <= 0 ? v.w : v.w & (~0u << (8 * b3));
    }
    return v;
}
// next n (<= 31) bits below the c already consumed from the top of hi
__device__ __forceinline__ uint32_t zw_get(uint64_t hi, int32_t &c, uint32_t n) {
    const uint32_t x = (uint32_t)((hi << c) >> 32);
    c += (int32_t)n;
    return __builtin_amdgcn_ubfe(x, 32u - n, n);
}

__device__ __forceinline__ void zvalues(SeqSmem &sm, int gn, int b);
// Wave 1: stage the group's tables (built in HBM by zseqa) into the arena,
// prefill the rings, then one refill round per period until the decoder
// reports no lane running.
__device__ __forceinline__ void zmover(SeqSmem &sm, int gn, const gc_u16 *tabs) {
    const int l = lane_id();
    [[maybe_unused]] uint64_t zt = ZP_NOW();
    for (int j0 = 0; j0 < gn; j0 += 4) {
        uint4 v[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u;
            const GBlk &d = sm.g[j < gn ? j : 0];
            const uint32_t al = d.al;
            const int32_t n16l = ((2 << (al & 0xFF)) + 15) >> 4, n16o = ((2 << ((al >> 8) & 0xFF)) + 15) >> 4,
                          n16m = ((2 << ((al >> 16) & 0xFF)) + 15) >> 4;
            v[u][0] = v[u][1] = v[u][2] = make_uint4(0, 0, 0, 0);
            if (j < gn && d.nseq > 0) {
                if (l < n16l) v[u][0] = ((const gc_u4 *)(tabs + d.tll))[l];
                if (l < n16o) v[u][1] = ((const gc_u4 *)(tabs + d.tof))[l];
                if (l < n16m) v[u][2] = ((const gc_u4 *)(tabs + d.tml))[l];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int j = j0 + u;
            if (j >= gn) break;
            uint4 *ar = (uint4 *)sm.arena[j];
            const uint32_t al = sm.g[j].al;
            if (l < (((2 << (al & 0xFF)) + 15) >> 4)) ar[l] = v[u][0];
            if (l < (((2 << ((al >> 8) & 0xFF)) + 15) >> 4)) ar[64 + l] = v[u][1];
            if (l < (((2 << ((al >> 16) & 0xFF)) + 15) >> 4)) ar[96 + l] = v[u][2];
        }
    }
    // lanes j, j + 16, j + 32, j + 48 serve block j (q = lane >> 4)
    const int q = l / ZNB, j = l - q * ZNB;  // lanes j + ZNB * q (q < ZMQ) serve block j
    const bool on = q < ZMQ && j < gn && sm.g[j < gn ? j : 0].nseq > 0 && sm.g[j < gn ? j : 0].bsz > 0;
    const ZGeo g = zgeo(sm.g[j < gn ? j : 0]);
    uint8_t *ring = sm.bring[q < ZMQ ? j : 0];
    // blocks below -3 are never read (a lane stops once its position is
    // below the stream start); blocks [-3, 0) are written as zeros
    constexpr int32_t KFLOOR = -3;
    // prefill blocks [kt - ZPRE, kt]
    int32_t lr = g.kt + 1;
    {
        const int32_t lo = g.kt - ZPRE > KFLOOR ? g.kt - ZPRE : KFLOOR;
        uint4 v[(ZAHEAD + 7) / 4];
#pragma unroll
        for (int i = 0; i < (ZAHEAD + 7) / 4; ++i) {
            const int32_t k = g.kt - q - 4 * i;
            v[i] = make_uint4(0, 0, 0, 0);
            if (on && k >= lo && k >= 0) v[i] = g.b16[k];
        }
#pragma unroll
        for (int i = 0; i < (ZAHEAD + 7) / 4; ++i) {
            const int32_t k = g.kt - q - 4 * i;
            if (on && k >= lo) zr_put(ring, k, zclip(v[i], k, g.m));
        }
        if (on) lr = lo;
    }
    { const uint64_t t = ZP_NOW(); ZS_ADD(1, t - zt); }
    zsync();  // tables and rings ready
    // Two sets of pending loads, used alternately: the loads a period issues
    // land (into the ring) two periods later from the same registers.  With
    // one shifting queue the copies between queue slots read registers whose
    // loads were still in flight, so every period waited for the loads it had
    // issued one period before (and, vmcnt counting loads and stores alike, for
    // the item stores in between).  Measured once the decoder's chain was lean:
    // zseqb 39.5 -> 37.3 ms (the state pass alone: 36.9).
    static_assert(ZMD == 2, "two alternating load sets");
    int32_t ka[2] = {0, 0}, kb[2] = {0, 0};
    uint4 va[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)}, vb[2] = {va[0], va[0]};
    bool oa[2] = {false, false}, ob[2] = {false, false};
    int p = 0;
    auto period = [&](int32_t (&kk)[2], uint4 (&vv)[2], bool (&oo)[2]) -> bool {
        // land this set's blocks (loaded two periods ago; a block below the
        // stream start was loaded from a safe address and lands as zeros)
#pragma unroll
        for (int i = 0; i < 2; ++i)
            if (oo[i]) zr_put(ring, kk[i], zclip(kk[i] >= 0 ? vv[i] : make_uint4(0, 0, 0, 0), kk[i], g.m));
        // next loads into this set (ZAHEAD blocks below the position published
        // at the last barrier), issued before this period's item stores: a
        // landing then waits only for its own loads and for stores issued
        // three periods before, not for the last period's stores
        const int32_t left = p == 0 ? 0 : sm.pos[(p - 1) & 1][j];
        const int32_t tgt = p == 0 ? lr : ((left - 1) >> 7) - ZAHEAD;
        int32_t lo = lr - 8;
        if (tgt > lo) lo = tgt;
        if (KFLOOR > lo) lo = KFLOOR;
        if (lo > lr) lo = lr;
        // (every lane loads, unconditionally: a fixed count of loads per
        // period lets the landing wait for exactly its own set)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int32_t k = lr - 1 - q - 4 * i;
            kk[i] = k;
            oo[i] = on && k >= lo;
            vv[i] = *(oo[i] && k >= 0 ? g.b16 + k : (const gc_u4 *)tabs);
        }
        if (on && lo < lr) lr = lo;
        if (p > 0) zvalues(sm, gn, (p - 1) & 1);  // the decoder's previous period
        zsync();
        return sm.more[p & 1] != 0;
    };
    for (;;) {
        if (!period(ka, va, oa)) break;
        ++p;
        if (!period(kb, vb, ob)) break;
        ++p;
    }
    zvalues(sm, gn, p & 1);  // the last period
    zsync();
}

// Phase B for the group (lane = block), tables and bitstreams in LDS, in two
// passes per period.  The STATE pass (wave 0, the decoder) is the serial part:
// per lane and sequence three cells, two extra-bit lookups and one bitstream
// window, only the FSE state updates and the bit position (recorded in LDS,
// double-buffered by period parity).  The VALUE pass (wave 1, the mover, one
// period behind) runs on all 64 lanes over a period's records (lane = block +
// 16 x record): extra bits -> lengths and offset value, and the repeat-offset
// updates as per-sequence transforms of (rep0, rep1, rep2) composed by a
// segmented prefix over the lanes of the same block (terms: constants or
// SYMB | j << 29 | d = max(1, rep_j - d), see rep_res); every block carries
// its composition across periods.  The records of period p-1 lie at most one
// 16-byte block above the position published at the end of period p-2, and
// the blocks the mover lands in period p were targeted from the position
// published at the end of period p-3: they evict ring slots >= 5 blocks
// above it, so the value pass still finds every record's bytes.
__device__ __forceinline__ uint32_t zsub(uint32_t x, uint32_t a0, uint32_t a1, uint32_t a2) {
    if (!(x & SYMB)) return x;
    const uint32_t j = (x >> 29) & 3u, dd = x & 0x1FFFFFFFu;
    const uint32_t y = j == 0 ? a0 : j == 1 ? a1 : a2;
    if (y & SYMB) return y + dd;
    return y > dd ? y - dd : 1u;
}
__device__ __forceinline__ void zvalues(SeqSmem &sm, int gn, int b) {
    const int l = lane_id();
    const int j = l & (ZNB - 1);
    static_assert(ZNB == 16 && ZK2 == 8, "value pass layout: 16 blocks x 4 records per round, two rounds");
    const bool blk = j < gn;
    const GBlk &d = sm.g[blk ? j : 0];
    const uint16_t *tl = sm.arena[j], *to = tl + 512, *tm = tl + 768;
    const uint8_t *ring = sm.bring[j];
    const int32_t cntj = blk ? sm.rcnt[b][j] : 0;
    const uint32_t ib0 = sm.ibase[b][j];
#pragma unroll
    for (int half = 0; half < 2; ++half) {
        const int kk = half * 4 + (l >> 4);
        const bool on = blk && kk < cntj;
        uint32_t ll = 0, ml = 0, ofv = 4;
        if (on) {
            const uint2 r = sm.rec[b][kk][j];
            const uint32_t cl = tl[r.y & 1023u], co = to[(r.y >> 10) & 1023u], cm = tm[r.y >> 20];
            uint64_t hi;
            uint32_t lo;
            zw_fill(ring, (int32_t)r.x, hi, lo);
            const uint32_t lv = sm.lut_ll[cl & 63], mv = sm.lut_ml[cm & 63], ofc = co & 63;
            int32_t c = 0;
            ofv = (1u << ofc) + zw_get(hi, c, ofc);
            ml = (mv & 0xFFFFFFu) + zw_get(hi, c, mv >> 24);
            ll = (lv & 0xFFFFFFu) + zw_get(hi, c, lv >> 24);
        }
        const uint32_t I0 = SYMB, I1 = SYMB | (1u << 29), I2 = SYMB | (2u << 29);
        uint32_t t0 = I0, t1 = I1, t2 = I2;
        if (on) {
            if (ofv > 3) {
                t0 = ofv - 3; t1 = I0; t2 = I1;
            } else {
                const uint32_t k = ofv - 1 + (ll == 0 ? 1u : 0u);
                if (k == 1) { t0 = I1; t1 = I0; }
                else if (k == 2) { t0 = I2; t1 = I0; t2 = I1; }
                else if (k == 3) { t0 = I0 + 1u; t1 = I0; t2 = I1; }
            }
        }
#pragma unroll
        for (int sft = 16; sft < 64; sft <<= 1) {  // prefix over the block's lanes (j, j + 16, ...)
            const uint32_t a0 = (uint32_t)__shfl_up((int)t0, sft, 64), a1 = (uint32_t)__shfl_up((int)t1, sft, 64),
                           a2 = (uint32_t)__shfl_up((int)t2, sft, 64);
            if (l >= sft) {
                const uint32_t n0 = zsub(t0, a0, a1, a2), n1 = zsub(t1, a0, a1, a2), n2 = zsub(t2, a0, a1, a2);
                t0 = n0; t1 = n1; t2 = n2;
            }
        }
        const uint32_t c0 = sm.carry[0][j], c1 = sm.carry[1][j], c2 = sm.carry[2][j];
        if (on) d.ib[d.item + 2 + ib0 + (uint32_t)kk] = make_uint4(ll, ml, zsub(t0, c0, c1, c2), IT_SEQ);
        const int nh = cntj - half * 4;  // records of this round for block j
        __builtin_amdgcn_wave_barrier();
        if (blk && nh > 0 && (l >> 4) == (nh < 4 ? nh : 4) - 1) {
            const uint32_t n0 = zsub(t0, c0, c1, c2), n1 = zsub(t1, c0, c1, c2), n2 = zsub(t2, c0, c1, c2);
            sm.carry[0][j] = n0; sm.carry[1][j] = n1; sm.carry[2][j] = n2;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

__device__ __forceinline__ void zdecode(SeqSmem &sm, int gn, uint32_t &r0, uint32_t &r1, uint32_t &r2,
                                        uint32_t &brep) {
    const int l = lane_id();
    const bool mine = l < gn;
    const GBlk d = sm.g[mine ? l : 0];
    const ZGeo g = zgeo(d);
    const uint8_t *ring = sm.bring[l < ZNB ? l : 0];
    const uint16_t *tl = sm.arena[l < ZNB ? l : 0], *to = tl + 512, *tm = tl + 768;
    const int32_t all = d.al & 0xFF, alof = (d.al >> 8) & 0xFF, alml = (d.al >> 16) & 0xFF;
    const int32_t m8 = 8 * g.m;
    g_u4 *it = d.ib + d.item;
    if (l < ZNB) {
        sm.carry[0][l] = SYMB;
        sm.carry[1][l] = SYMB | (1u << 29);
        sm.carry[2][l] = SYMB | (2u << 29);
    }
    zsync();  // the mover has staged the tables and prefilled the rings
    [[maybe_unused]] uint64_t zt = ZP_NOW();
    bool run = false;
    int32_t left = 0, i = 0;
    uint32_t sll = 0, sof = 0, sml = 0;
    if (mine) {
        if (d.nseq == 0) {
            it[1] = make_uint4(0, 0, 0, IT_BREP);
            it[2] = make_uint4(0, 0, 0, IT_BEND);
            brep = 1;
        } else {
            const uint32_t last = d.bsz > 0 ? ring[(g.top - 1) & (ZRB2 - 1)] : 0u;
            if (last == 0) {
                it[1] = make_uint4(0, 0, (uint32_t)E_CORRUPT, IT_ERR);
            } else {
                brep = 1;
                run = true;
                left = 8 * (g.top - 1) + (31 - __builtin_clz(last));
            }
        }
    }
    if (run) {
        uint64_t hi;
        uint32_t lo;
        zw_fill(ring, left, hi, lo);
        int32_t c = 0;
        sll = zw_get(hi, c, all);
        sof = zw_get(hi, c, alof);
        sml = zw_get(hi, c, alml);
        left -= c;
    }
    const uint32_t szl = 1u << all, szo = 1u << alof, szm = 1u << alml;
    const uint32_t kl31 = (uint32_t)all - 31u, ko31 = (uint32_t)alof - 31u, km31 = (uint32_t)alml - 31u;
    // 0: running or ended before, 1: stream overflow, 2: last sequence with
    // the stream exactly consumed (BEND), 3: last sequence, bits left (ERR);
    // the item is stored once per period, after the unrolled sequences
    uint32_t fin = 0;
    for (int p = 0;; ++p) {
        const int32_t i0 = i;
#pragma unroll
        for (int k = 0; k < ZK2; ++k) {
            if (run) {
                if (left < m8) {  // overflow
                    fin = 1;
                    run = false;
                } else {
                    const uint32_t cl = tl[sll], co = to[sof], cm = tm[sml];
                    const int32_t cbw = ((left - 96) >> 5) << 2;  // as zw_fill
                    const uint32_t *w4 = (const uint32_t *)(ring + (cbw & (ZRB2 - 1)));
                    const uint32_t d0 = w4[0], d1 = w4[1], d2 = w4[2], d3 = w4[3];
                    const int32_t tw = left - 8 * cbw - 64;  // [32, 64)
                    sm.rec[p & 1][k][l] = make_uint2((uint32_t)left, sll | (sof << 10) | (sml << 20));
                    const int32_t c = (int32_t)((uint32_t)sm.xb_ll[cl & 63] + (uint32_t)sm.xb_ml[cm & 63] + (co & 63));
                    int32_t c2 = 0;
                    // (the next states are computed for the last sequence too --
                    // the lane stops right after -- so no branch per sequence)
                    {
                        // the 32 bits below position left - c: bits [u, u + 32) of d0..d3
                        const uint32_t u = (uint32_t)(tw + 32 - c), wsel = u >> 5;
                        const uint32_t lo_d = wsel == 0 ? d0 : wsel == 1 ? d1 : d2;
                        const uint32_t hi_d = wsel == 0 ? d1 : wsel == 1 ? d2 : d3;
                        const uint64_t h2 = (uint64_t)__builtin_amdgcn_alignbit(hi_d, lo_d, u & 31u) << 32;
                        const uint32_t nsl = cl >> 6, nso = co >> 6, nsm = cm >> 6;
                        const uint32_t nbl = kl31 + (uint32_t)__builtin_clz(nsl);
                        const uint32_t nbm = km31 + (uint32_t)__builtin_clz(nsm);
                        const uint32_t nbo = ko31 + (uint32_t)__builtin_clz(nso);
                        // the three state reads (<= 9 + 9 + 8 bits) all lie in the
                        // window's top 32 bits: one extraction, three field reads
                        const uint32_t x = (uint32_t)(h2 >> 32);
                        const uint32_t ol = 32u - nbl, om = ol - nbm, oo = om - nbo;
                        sll = ((nsl << nbl) - szl) + __builtin_amdgcn_ubfe(x, ol, nbl);
                        sml = ((nsm << nbm) - szm) + __builtin_amdgcn_ubfe(x, om, nbm);
                        sof = ((nso << nbo) - szo) + __builtin_amdgcn_ubfe(x, oo, nbo);
                        c2 = i + 1 >= d.nseq ? 0 : (int32_t)(32u - oo);
                    }
                    left -= c + c2;
                    ++i;
                    if (i == d.nseq) {
                        fin = left == m8 ? 2u : 3u;
                        run = false;
                    }
                }
            }
        }
        if (fin) {
            it[2 + i] = fin == 2 ? make_uint4(0, 0, 0, IT_BEND) : make_uint4(0, 0, (uint32_t)E_CORRUPT, IT_ERR);
            fin = 0;
        }
        if (l < ZNB) {
            sm.rcnt[p & 1][l] = i - i0;
            sm.ibase[p & 1][l] = (uint32_t)i0;
            sm.pos[p & 1][l] = left;
        }
        const bool any = __ballot(run) != 0;
        if (l == 0) sm.more[p & 1] = any ? 1 : 0;
        [[maybe_unused]] const uint64_t tw = ZP_NOW();
        zsync();  // the mover takes this period's records (value pass) during the next
        ZS_ADD(4, ZP_NOW() - tw);
        if (!any) break;
    }
    zsync();  // the mover's value pass of the last period
    if (l < ZNB) {
        r0 = sm.carry[0][l];
        r1 = sm.carry[1][l];
        r2 = sm.carry[2][l];
    }
    { const uint64_t t = ZP_NOW(); ZS_ADD(2, t - zt); }
}

// phases B (both waves) and C (wave 0) for the collected group
// carry slot of a split input: 16 bytes after the ZDesc of block ZNB - 1
// (e0, e1, e2, ready); zseqa zeroes it, the first half publishes it
__device__ __forceinline__ uint32_t *zcarry_slot(uint16_t *tabs_in) {
    return (uint32_t *)(tabs_in + (uint64_t)(ZNB - 1) * TAB_STRIDE + TAB_CELLS + 24);
}
static_assert(sizeof(ZDesc) <= 48 && TAB_STRIDE - TAB_CELLS >= 32, "carry slot after the ZDesc");
__device__ __forceinline__ void seq_group2(SeqSmem &sm, int gn, uint32_t *e0, uint32_t *e1, uint32_t *e2,
                                           uint32_t *wait_carry = nullptr) {
    const int l = lane_id();
    ZS_ADD(5, 1);
    uint32_t r0 = SYMB | (0u << 29), r1 = SYMB | (1u << 29), r2 = SYMB | (2u << 29);
    uint32_t brep = 0;
    zdecode(sm, gn, r0, r1, r2, brep);
    bool lost = false;
    if (wait_carry) {  // the second half of a split input: entry offsets from the first half
        // Forward progress (see the zseqb launch): the first half never waits
        // on anything, so this wait ends.  Should that ever break, the wait
        // gives up after ~2^22 sleeps (~1 s) and the input fails with E_BUG
        // (an IT_ERR item where its first block's entry state would go)
        // instead of hanging the GPU.
        for (uint32_t spins = 0;
             __hip_atomic_load(wait_carry + 3, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == 0u; ++spins) {
            if (spins > (1u << 22)) { lost = true; break; }
            __builtin_amdgcn_s_sleep(8);
        }
        *e0 = __hip_atomic_load(wait_carry + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *e1 = __hip_atomic_load(wait_carry + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *e2 = __hip_atomic_load(wait_carry + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    [[maybe_unused]] uint64_t zt = ZP_NOW();
    for (int gi = 0; gi < gn; gi++) {
        const uint32_t al = sm.g[gi].al, item = sm.g[gi].item;
        g_u4 *ib = sm.g[gi].ib;
        if (al >> 24) { *e0 = 1; *e1 = 4; *e2 = 8; }
        const uint32_t x0 = readlane(r0, gi), x1 = readlane(r1, gi), x2 = readlane(r2, gi);
        if (lost && gi == 0) {
            if (l == 0) ib[item + 1] = make_uint4(0, 0, (uint32_t)E_BUG, IT_ERR);
        } else if (readlane(brep, gi) && l == 0) {
            ib[item + 1] = make_uint4(*e0, *e1, *e2, IT_BREP);
        }
        const uint32_t n0 = rep_res(x0, *e0, *e1, *e2), n1 = rep_res(x1, *e0, *e1, *e2), n2 = rep_res(x2, *e0, *e1, *e2);
        *e0 = n0; *e1 = n1; *e2 = n2;
    }
    __builtin_amdgcn_wave_barrier();
    { const uint64_t t = ZP_NOW(); ZS_ADD(3, t - zt); }
}

// zseqa (phase A): one wave per input walks the headers, builds each
// compressed block's FSE tables into its HBM table area and writes the
// block's ZDesc after them; zseqb decodes the sequences.
__global__ __launch_bounds__(64) void zseqa_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                      ZInfo *__restrict__ info, uint16_t *__restrict__ tabs_all,
                                                      uint4 *__restrict__ items_all, int strict_reserved) {
    __shared__ ASmem sm;
    const int l = lane_id();
    [[maybe_unused]] uint64_t za = ZP_NOW();
    {
        const int bi = blockIdx.x;
        if (bi >= nblk) return;
        const jfs_dev_block b = blocks[bi];
        ZInfo &zi = info[bi];
        if (zi.ovf) return;
        const gc_u8 *s = (const gc_u8 *)b.src;
        g_u16 *tabs = (g_u16 *)tabs_all + zi.tab_off;
        g_u4 *items = (g_u4 *)items_all + zi.item_off;
        Walk w;
        walk_init(w, s, b.src_len, b.dst_cap);
        const uint32_t cap_items = zi.n_items, cap_cblk = zi.n_cblk;
        uint32_t cur = 0, cblk = 0, nd = 0;  // next item slot, next table area, descriptors
        int first = 0, bug = 0;
        uint32_t t_ll = 0, t_of = 0, t_ml = 0;
        int32_t al_ll = 0, al_of = 0, al_ml = 0, hv_ll = 0, hv_of = 0, hv_ml = 0;
        auto put = [&](uint32_t x, uint32_t y, uint32_t z, uint32_t kind) {
            if (cur >= cap_items) { bug = 1; return; }
            if (l == 0) items[cur] = make_uint4(x, y, z, kind);
            cur++;
        };
        for (;;) {
            int32_t err = 0;
            uint32_t fl = 0, chk = 0;
            int ev = walk_next(w, &err, &fl, &chk);
            if (ev == EV_DONE) break;
            if (ev == EV_ERROR) { put(0, 0, (uint32_t)err, IT_ERR); break; }
            if (ev == EV_FSTART) {
                hv_ll = hv_of = hv_ml = 0;
                first = 1;
                put(0, 0, 0, IT_FSTART);
                continue;
            }
            if (ev == EV_FEND) {
                put((uint32_t)w.fcs, (uint32_t)(w.fcs >> 32), chk, IT_FEND | (fl << 8));
                if (fl & FE_MISSING) break;
                continue;
            }
            const uint32_t ord = w.ordinal - 1;
            if (w.btype != 2) {
                put(ord, (uint32_t)w.bsize, 0, IT_BSTART);
                put((uint32_t)w.bsize, 0, 0, IT_SEQ);
                put(0, 0, 0, IT_BEND);
                w.lb += w.bsize;
                continue;
            }
            LitHdr h;
            int32_t e = lit_header(s, w.bpos, w.bsize, h);
            const uint32_t slot = cur;
            put(ord, e ? 0u : (uint32_t)h.regen, 0, IT_BSTART);
            if (e) { put(0, 0, (uint32_t)e, IT_ERR); break; }
            const int32_t end = w.bpos + w.bsize;
            int32_t ip = w.bpos + h.sec;
            int32_t nseq = 0, used = 0;
            e = nbseq_header(s, ip, end, &nseq, &used);
            if (e) { put(0, 0, (uint32_t)e, IT_ERR); break; }
            ip += used;
            w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
            if (cblk >= cap_cblk || slot + 3 + (uint32_t)nseq > cap_items) { bug = 1; break; }
            const uint32_t area = cblk * TAB_STRIDE;
            cblk++;
            uint32_t rs = 0;  // deferred table builds (zbuild)
            if (nseq > 0) {
                if (ip + 1 > end) { put(0, 0, (uint32_t)E_SRCSIZE, IT_ERR); break; }
                uint32_t modes = rd8(s, ip++);
                if ((modes & 3) && strict_reserved) { put(0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
                int32_t c = seq_table_defer(sm, tabs, area, &t_ll, &al_ll, &hv_ll, modes >> 6, s, ip, end - ip, 0, &rs);
                if (c >= 0) { ip += c; c = seq_table_defer(sm, tabs, area + 512, &t_of, &al_of, &hv_of, (modes >> 4) & 3, s, ip, end - ip, 1, &rs); }
                if (c >= 0) { ip += c; c = seq_table_defer(sm, tabs, area + 768, &t_ml, &al_ml, &hv_ml, (modes >> 2) & 3, s, ip, end - ip, 2, &rs); }
                if (c < 0) { put(0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
                ip += c;
            }
            if (l == 0) {
                ZDesc d;
                d.bs = (uint64_t)(uintptr_t)(s + ip);
                d.bsz = end - ip;
                d.nseq = nseq;
                d.item = slot;
                d.tll = t_ll; d.tof = t_of; d.tml = t_ml;
                d.al = (uint32_t)al_ll | ((uint32_t)al_of << 8) | ((uint32_t)al_ml << 16) | ((uint32_t)first << 24);
                d.rsv = rs;
                *(JFS_GLOBAL ZDesc *)(tabs + area + TAB_CELLS) = d;
                *(JFS_GLOBAL uint4 *)(tabs + area + TAB_CELLS + 24) = make_uint4(0, 0, 0, 0);  // carry slot
            }
            first = 0;
            cur = slot + 3 + (uint32_t)nseq;
            nd++;
        }
        if (l == 0) {
            zi.n_items = bug ? 0xFFFFFFFFu : cur;
            zi.n_sblk = nd;
        }
    }
    ZS_ADD(0, ZP_NOW() - za);
}

// zbuild: spreads the FSE tables zseqa left described.  Grid (inputs, ZBUILD_Q):
// workgroup (i, q) takes tables q, q + Q, ... of input i (three per block).
constexpr int ZBUILD_Q = 16;
__global__ __launch_bounds__(64) void zbuild_kernel(int nblk, const ZInfo *__restrict__ info,
                                                    uint16_t *__restrict__ tabs_all) {
    __shared__ uint8_t symat[512], mark[512], ksym[512];
    const int l = lane_id();
    const int bi = blockIdx.x;
    if (bi >= nblk) return;
    const ZInfo zi = info[bi];
    if (zi.ovf || zi.n_items == 0xFFFFFFFFu) return;
    g_u16 *tabs = (g_u16 *)tabs_all + zi.tab_off;
    const uint32_t nt = 3 * zi.n_sblk;
    for (uint32_t t = blockIdx.y; t < nt; t += ZBUILD_Q) {
        const uint32_t j = t / 3, f = t - 3 * j;
        g_u16 *area = tabs + (uint64_t)j * TAB_STRIDE;
        const uint32_t rs = ((const JFS_GLOBAL ZDesc *)(area + TAB_CELLS))->rsv;
        const uint32_t kind = (rs >> (18 + 2 * f)) & 3u;
        if (!kind) continue;
        const int32_t ms = (int32_t)((rs >> (6 * f)) & 63u);
        g_u16 *reg = area + (f == 0 ? 0 : f == 1 ? 512 : 768);
        int32_t al;
        if (kind == 2) {
            const int16_t *def = f == 0 ? LL_DEF : f == 1 ? OF_DEF : ML_DEF;
            al = f == 1 ? 5 : 6;
            build_seq_fse_g(reg, def, ms, al, mark, ksym, symat);
        } else {
            const uint32_t a8 = ((const JFS_GLOBAL ZDesc *)(area + TAB_CELLS))->al;
            al = (int32_t)((a8 >> (8 * f)) & 0xFFu);
            build_seq_fse_g(reg, (const int16_t *)(reg + zfield_cells((int)f) - 64), ms, al, mark, ksym, symat);
        }
    }
}

// zseqb (phases B and C): wave 0 gathers ZNB blocks' descriptors at a time
// (in stream order over the workgroup's inputs), decodes their sequences
// with wave 1 keeping the tables and bitstreams in LDS, then resolves the
// symbolic repeat offsets in block order.
__global__ __launch_bounds__(128) void zseqb_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                    ZInfo *__restrict__ info, uint16_t *__restrict__ tabs_all,
                                                    uint4 *__restrict__ items_all) {
    __shared__ SeqSmem sm;
    const int l = lane_id();
    for (int i = l; i < 36; i += 64) sm.lut_ll[i] = LL_BASE[i] | ((uint32_t)LL_BITS[i] << 24);
    for (int i = l; i < 53; i += 64) sm.lut_ml[i] = ML_BASE[i] | ((uint32_t)ML_BITS[i] << 24);
    sm.xb_ll[l] = l < 36 ? LL_BITS[l] : (uint8_t)0;  // (codes past the tables: 0; the stream check catches them)
    sm.xb_ml[l] = l < 53 ? ML_BITS[l] : (uint8_t)0;
    if (threadIdx.x >= 64) {  // the mover wave: one group per command from wave 0
        for (;;) {
            zsync();
            const int gn = sm.cmd;
            if (gn == 0) break;
            zmover(sm, gn, (const gc_u16 *)tabs_all);
        }
        return;
    }
    int gn = 0;
    uint32_t e0 = 1, e1 = 4, e2 = 8;  // repeat offsets carried through phase C (reset at each frame)
    // two workgroups per input: blocks [0, ZNB) and [ZNB, n); the second
    // takes its entry repeat offsets from the first at its first phase C
    const int bi = blockIdx.x >> 1, half = blockIdx.x & 1;
    if (bi < nblk) {
        const ZInfo zi = info[bi];
        if (!(zi.ovf || zi.n_items == 0xFFFFFFFFu) && (!half || zi.n_sblk > (uint32_t)ZNB)) {
            const gc_u16 *tabs = (const gc_u16 *)tabs_all + zi.tab_off;
            uint32_t *carry = zcarry_slot(tabs_all + zi.tab_off);
            g_u4 *items = (g_u4 *)items_all + zi.item_off;
            const uint32_t j1 = half ? zi.n_sblk : umin32((uint32_t)ZNB, zi.n_sblk);
            for (uint32_t j = half ? (uint32_t)ZNB : 0u; j < j1;) {
                const uint32_t take = umin32((uint32_t)ZNB, j1 - j);
                if ((uint32_t)l < take) {
                    const ZDesc d = *(const JFS_GLOBAL ZDesc *)(tabs + (uint64_t)(j + l) * TAB_STRIDE + TAB_CELLS);
                    GBlk &g = sm.g[l];
                    g.bs = (const gc_u8 *)(uintptr_t)d.bs;
                    g.in = g.bs;
                    g.ib = items;
                    g.bsz = d.bsz;
                    g.nseq = d.nseq;
                    g.item = d.item;
                    g.tll = zi.tab_off + d.tll; g.tof = zi.tab_off + d.tof; g.tml = zi.tab_off + d.tml;
                    g.al = d.al;
                }
                __builtin_amdgcn_wave_barrier();
                if (l == 0) sm.cmd = (int)take;
                zsync();
                seq_group2(sm, (int)take, &e0, &e1, &e2, half && j == (uint32_t)ZNB ? carry : nullptr);
                j += take;
            }
            if (!half && zi.n_sblk > (uint32_t)ZNB && l == 0) {
                __hip_atomic_store(carry + 0, e0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(carry + 1, e1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(carry + 2, e2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(carry + 3, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (l == 0) sm.cmd = 0;
    zsync();  // releases the mover
}

// ---------------------------------------------------------------------------
// kernel 3: execute items
// ---------------------------------------------------------------------------
// V2 needs no far-source buffer: the ring takes its 4 KiB (sources up to 8 KiB
// back stay in LDS; fewer far matches, rarer waits for flushed output)
constexpr int R = 8192;
constexpr int RMASK = R - 1;
constexpr int LW = 2048;          // literal staging window
constexpr int FLUSH_T = 1024;

constexpr int BSPAN = 2048;      // max output span of one lane-parallel batch
static_assert(BSPAN <= R / 2, "a batch span and the unflushed tail fit the ring");
constexpr int LONGI = 64;  // items with a literal run or match longer than this go whole-wave

// 10,240 bytes: 16 workgroups (one per frame of a 4,096-frame launch) fit a
// CU's 160 KiB, so a launch is one round (at 10,304 bytes it was 15 per CU and
// the 256 leftover frames ran as a second round).  Over-reads past lw and
// farbuf (dword/alignbyte tails) only fetch bytes that are never used.
struct XSmem {
    alignas(16) uint8_t ring[R];
    union {
        alignas(16) uint8_t lw[LW];  // literal window (x.lw0 is reset after a checksum)
        uint64_t xxh[4];             // frame checksum (between batches)
    };
};
static_assert(sizeof(XSmem) * 16 <= 160 * 1024, "16 zexec workgroups per CU");

struct X {
#ifdef JFS_PROF
    uint64_t pacc[8];
#endif
    int32_t bug;
    g_u8 *dst;
    const gc_u8 *lit;      // literal buffer of this input
    int64_t lw0;           // literal index of lw[0]
    int32_t cap, op, F, Fw, fstart;
    uint32_t dmis;
};

__device__ __forceinline__ uint32_t slot(const X &x, int32_t pos) { return (uint32_t)(pos + (int32_t)x.dmis) & RMASK; }

__device__ __forceinline__ void xflush(XSmem &s, X &x, int32_t to, bool wait = true) {
    const int l = lane_id();
    if (wait) {
        wait_vm();
        x.Fw = x.F;
    }
    int32_t F = x.F;
    if (to <= F) return;
    int32_t a = F + (int32_t)((16u - ((x.dmis + (uint32_t)F) & 15u)) & 15u);
    if (a > to) a = to;
    if (l < a - F) x.dst[F + l] = s.ring[slot(x, F + l)];
    int32_t bb = a + ((to - a) & ~15);
    for (int32_t q = a + 16 * l; q < bb; q += 1024) *(g_u4 *)(x.dst + q) = *(const uint4 *)(s.ring + slot(x, q));
    if (l < to - bb) x.dst[bb + l] = s.ring[slot(x, bb + l)];
    x.F = to;
}
__device__ __forceinline__ void xflush_line(XSmem &s, X &x, int32_t hi, bool wait = true) {
    int32_t to = (int32_t)(((uint32_t)hi + x.dmis) & ~127u) - (int32_t)x.dmis;
    if (to > x.F) xflush(s, x, to, wait);
}

// make lit[lp, lp+need) resident in the staging window
__device__ __forceinline__ void lit_window(XSmem &s, X &x, int64_t lp, int32_t need = 64) {
    if (lp >= x.lw0 && lp + need <= x.lw0 + LW) return;
    const int l = lane_id();
    int64_t base = lp & ~15LL;
    for (int k = l; k < LW / 16; k += 64) {
        uint4 v = *(const gc_u4 *)(x.lit + base + 16 * k);
        *(uint4 *)(s.lw + 16 * k) = v;
    }
    x.lw0 = base;
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ void x_lit(XSmem &s, X &x, int64_t lp, int32_t len) {
    const int l = lane_id();
    for (int32_t k = 0; k < len; k += 64) {
        if (x.op + k - x.F >= FLUSH_T) xflush_line(s, x, x.op + k);
        lit_window(s, x, lp + k);
        int32_t i = k + l;
        if (i < len) s.ring[slot(x, x.op + i)] = s.lw[lp + i - x.lw0];
        __builtin_amdgcn_wave_barrier();
    }
    x.op += len;
}

// XXH64 of dst[a, b) (already in HBM), one wave
__device__ __forceinline__ uint64_t xxh64_dev(XSmem &s, const gc_u8 *p, int64_t len) {
    const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                   P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
    auto rotl = [](uint64_t v, int r) { return (v << r) | (v >> (64 - r)); };
    auto rd64 = [&](int64_t q) {
        uint64_t v = 0;
        for (int i = 0; i < 8; i++) v |= (uint64_t)p[q + i] << (8 * i);
        return v;
    };
    const int l = lane_id();
    uint64_t h;
    int64_t pos = 0;
    if (len >= 32) {
        uint64_t acc = l == 0 ? P1 + P2 : l == 1 ? P2 : l == 2 ? 0 : (uint64_t)0 - P1;
        int64_t nst = len / 32;
        if (l < 4) {
            for (int64_t k = 0; k < nst; k++) {
                acc += rd64(32 * k + 8 * l) * P2;
                acc = rotl(acc, 31) * P1;
            }
            s.xxh[l] = acc;
        }
        __builtin_amdgcn_wave_barrier();
        uint64_t v1 = s.xxh[0], v2 = s.xxh[1], v3 = s.xxh[2], v4 = s.xxh[3];
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        auto merge = [&](uint64_t a, uint64_t v) { v *= P2; v = rotl(v, 31) * P1; a ^= v; return a * P1 + P4; };
        h = merge(h, v1); h = merge(h, v2); h = merge(h, v3); h = merge(h, v4);
        pos = nst * 32;
    } else {
        h = P5;
    }
    h += (uint64_t)len;
    while (pos + 8 <= len) {
        uint64_t k1 = rd64(pos) * P2;
        k1 = rotl(k1, 31) * P1;
        h ^= k1;
        h = rotl(h, 27) * P1 + P4;
        pos += 8;
    }
    if (pos + 4 <= len) {
        uint64_t v = (uint64_t)p[pos] | ((uint64_t)p[pos + 1] << 8) | ((uint64_t)p[pos + 2] << 16) | ((uint64_t)p[pos + 3] << 24);
        h ^= v * P1;
        h = rotl(h, 23) * P2 + P3;
        pos += 4;
    }
    while (pos < len) {
        h ^= (uint64_t)p[pos] * P5;
        h = rotl(h, 11) * P1;
        pos++;
    }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

// ---------------------------------------------------------------------------
// V2 batch: the LZ4 copier's scheme (lz4_decode.hip batch()).
// The batch's ring span is zeroed, then every write is an LDS atomic OR of
// whole dwords (lanes sharing a boundary dword cannot clobber each other), in
// fixed 16-byte steps: literal runs from the staged literal window, far matches
// from HBM (24 bytes loaded per 16-byte step), then near matches: source
// substitution (a match whose source lies inside another pending match of the
// batch reads that match's source), one lane-parallel round for matches whose
// source is final (before the batch, or inside one literal run of it), and the
// rest by the whole wave in lane (= output) order.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t zbal(bool b) { return __builtin_amdgcn_ballot_w64(b); }

__device__ __forceinline__ void zor(XSmem &s, uint32_t a, uint32_t v) {  // a % 4 == 0
    __hip_atomic_fetch_or(reinterpret_cast<uint32_t *>(s.ring) + (a >> 2), v, __ATOMIC_RELAXED,
                          __HIP_MEMORY_SCOPE_WORKGROUP);
}
// bytes [ha, ha + m) (1 <= m <= 16, ha = da & 3) of the 20-byte span w0..w4 to ring slot da
__device__ __forceinline__ void zput16(XSmem &s, uint32_t da, int32_t m, uint32_t w0, uint32_t w1, uint32_t w2,
                                       uint32_t w3, uint32_t w4) {
    const int32_t ha = (int32_t)(da & 3u), e8 = 8 * (ha + m);
    const uint32_t D0 = da & ~3u;
    auto lm = [](int32_t b) -> uint32_t {  // low min(max(b, 0), 32) bits
        const uint32_t sh = (uint32_t)(b < 0 ? 0 : b > 32 ? 32 : b);
        return (uint32_t)((0xFFFFFFFFull << sh) >> 32);
    };
    zor(s, D0, w0 & lm(e8) & ~lm(8 * ha));
    zor(s, (D0 + 4) & RMASK, w1 & lm(e8 - 32));
    zor(s, (D0 + 8) & RMASK, w2 & lm(e8 - 64));
    zor(s, (D0 + 12) & RMASK, w3 & lm(e8 - 96));
    zor(s, (D0 + 16) & RMASK, w4 & lm(e8 - 128));
}
// m (1..16) bytes from LDS byte address sa (RING: ring slot space) to ring slot da
template <bool RING>
__device__ __forceinline__ void zcopy16(XSmem &s, uint32_t sa, uint32_t da, int32_t m) {
    const uint8_t *lds = (const uint8_t *)&s;
    const uint32_t ha = da & 3u;
    const uint32_t sb = sa - ha, S0 = sb & ~3u, sh = sb & 3u;
    uint32_t r[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t a = RING ? ((S0 + 4 * j) & RMASK) : (S0 + 4 * j);
        r[j] = *(const uint32_t *)(lds + a);
    }
    zput16(s, da, m, __builtin_amdgcn_alignbyte(r[1], r[0], sh), __builtin_amdgcn_alignbyte(r[2], r[1], sh),
           __builtin_amdgcn_alignbyte(r[3], r[2], sh), __builtin_amdgcn_alignbyte(r[4], r[3], sh),
           __builtin_amdgcn_alignbyte(r[5], r[4], sh));
}
// zero ring bytes of output [O0, O1) (bytes below O0 in the first dword are kept)
__device__ __forceinline__ void zzero_span(XSmem &s, const X &x, int32_t O0, int32_t O1) {
    const int l = lane_id();
    const uint32_t a = slot(x, O0), h = a & 3u;
    const int32_t A = O0 + (int32_t)((4u - h) & 3u);
    if (l == 0 && h) {
        const uint32_t keep = (1u << (8 * h)) - 1u;
        __hip_atomic_fetch_and(reinterpret_cast<uint32_t *>(s.ring) + (a >> 2), keep, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    for (int32_t q = A + 4 * l; q < O1; q += 256) *(uint32_t *)(s.ring + slot(x, q)) = 0u;
}
typedef uint32_t zu32x4 __attribute__((ext_vector_type(4), aligned(4)));
typedef uint32_t zu32x2 __attribute__((ext_vector_type(2), aligned(4)));
// far source: the 6 dwords from the dword holding HBM address a.  A dword
// wholly below the output's first dword (lo) holds no source byte (only bytes
// the write mask drops) and is not read: it reads as 0.
__device__ __forceinline__ void zfar_load(uintptr_t a, uintptr_t lo, uint32_t (&d)[6]) {
    const uintptr_t b = a & ~(uintptr_t)3;
    lo &= ~(uintptr_t)3;
    const bool under = b < lo;
    const uintptr_t q = under ? lo : b;
    const zu32x4 v = *(JFS_GLOBAL const zu32x4 *)q;
    const zu32x2 w = *(JFS_GLOBAL const zu32x2 *)(q + 16);
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w; d[4] = w.x; d[5] = w.y;
    if (zbal(under)) {
        if (under) { d[5] = d[4]; d[4] = d[3]; d[3] = d[2]; d[2] = d[1]; d[1] = d[0]; d[0] = 0; }
    }
}
// whole-wave copy of len bytes to output op from op - D (all inside the ring),
// in chunks of at most D bytes so that self-overlapping matches repeat their period
__device__ __forceinline__ void zwave_near(XSmem &s, const X &x, int32_t op, int32_t D, int32_t len) {
    const int l = lane_id();
    const int32_t step = D < 64 ? D : 64;
    for (int32_t k = 0; k < len; k += step) {
        const int32_t i = k + l;
        if (l < step && i < len) s.ring[slot(x, op + i)] = s.ring[slot(x, op + i - D)];
    }
}

__device__ __forceinline__ void x_batch2(XSmem &s, X &x, bool act, int32_t o, uint32_t ll, uint32_t ml, uint32_t off,
                                         int32_t lit, int32_t O0, int32_t O1) {
    // sources below hz come from HBM: the ring slots of [hz, O1) are intact
    // (zzero_span may clear up to 3 bytes past O1)
    const int32_t hz = O1 + 4 - R;
    uint64_t tq0 = ZP_NOW();
    if (O0 - x.F >= FLUSH_T) xflush_line(s, x, O0, false);
    zzero_span(s, x, O0, O1);
    const int32_t ms = o + (int32_t)ll, msrc = ms - (int32_t)off;
    const bool hasm = act && ml > 0;
    const bool far = hasm && msrc < hz;
    // a far source (< hz + LONGI) must be flushed and its stores complete
    if (zbal(far) && hz + LONGI > x.Fw) {
        wait_vm();
        x.Fw = x.F;
        if (hz + LONGI > x.Fw) x.bug = 105;
    }
    uint32_t fd[6] = {0, 0, 0, 0, 0, 0};
    const uint32_t fha = slot(x, ms) & 3u;
    if (zbal(far)) {
        if (far) zfar_load((uintptr_t)(x.dst + msrc) - fha, (uintptr_t)x.dst, fd);
    }
    uint64_t tq1 = ZP_NOW();
    // literal runs (source: the staged literal window)
    const uint32_t lwoff = (uint32_t)((const uint8_t *)s.lw - (const uint8_t *)&s) + (uint32_t)(lit - (int32_t)x.lw0);
    for (uint32_t k = 0; zbal(act && k < ll); k += 16) {
        if (act && k < ll) {
            const int32_t m = ll - k < 16u ? (int32_t)(ll - k) : 16;
            zcopy16<false>(s, lwoff + k, slot(x, o + (int32_t)k), m);
        }
    }
    uint64_t tq2 = ZP_NOW();
    // far matches
    if (zbal(far)) {
        for (uint32_t k = 0; zbal(far && k < ml); k += 16) {
            if (far && k < ml) {
                const int32_t m = ml - k < 16u ? (int32_t)(ml - k) : 16;
                const uint32_t da = slot(x, ms + (int32_t)k);  // da & 3 == fha
                const uint32_t sh = (uint32_t)((uintptr_t)(x.dst + msrc + (int32_t)k) - fha) & 3u;
                zput16(s, da, m, __builtin_amdgcn_alignbyte(fd[1], fd[0], sh), __builtin_amdgcn_alignbyte(fd[2], fd[1], sh),
                       __builtin_amdgcn_alignbyte(fd[3], fd[2], sh), __builtin_amdgcn_alignbyte(fd[4], fd[3], sh),
                       __builtin_amdgcn_alignbyte(fd[5], fd[4], sh));
            }
            const bool more = far && k + 16 < ml;
            if (zbal(more)) {
                if (more) zfar_load((uintptr_t)(x.dst + msrc + (int32_t)k + 16) - fha, (uintptr_t)x.dst, fd);
            }
        }
    }
    uint64_t tq3 = ZP_NOW();
    XP_ADD(1, tq1 - tq0);
    XP_ADD(2, tq2 - tq1);
    XP_ADD(3, tq3 - tq2);
    XP_ADD(5, 1);
    // source substitution: out[x] == out[x - off_i] for every byte a match i
    // writes, so a pending match whose whole source lies inside another
    // pending match of this batch can read that match's source instead
    bool pend = hasm && !far;
    int32_t src = msrc;
    const uint64_t am = zbal(act);
    const int first = am ? (int)__builtin_ctzll(am) : 0;
    const uint32_t key = act ? (uint32_t)ms : ((int)lane_id() < first ? 0u : 0xFFFFFFFFu);  // non-decreasing
    bool litsrc = false;  // the source lies wholly inside one literal run of this batch (written above)
    {
        const uint32_t mek = pend ? (uint32_t)(ms + (int32_t)ml) : 0u;
        const bool want = pend && off >= ml && src >= O0;
        if (zbal(want)) {
            int lo = 0;  // last lane with key <= src
#pragma unroll
            for (int stp = 32; stp; stp >>= 1) {
                const uint32_t v = (uint32_t)__shfl((int)key, lo + stp, 64);
                lo = v <= (uint32_t)src ? lo + stp : lo;
            }
            const uint32_t vms = (uint32_t)__shfl((int)key, lo, 64);
            const uint32_t vme = (uint32_t)__shfl((int)mek, lo, 64);
            const int32_t voff = __shfl((int)off, lo, 64);
            const uint32_t nms = (uint32_t)__shfl((int)key, lo + 1 < 64 ? lo + 1 : 63, 64);
            const bool ok = want && vms <= (uint32_t)src && (uint32_t)(src + (int32_t)ml) <= vme && voff > 0 &&
                            src - voff >= hz;
            // past the end of lane lo's match and before the next lane's match:
            // inside the next item's literal run, already in the ring
            litsrc = want && vms <= (uint32_t)src && (uint32_t)src >= vme && lo < 63 &&
                     (uint32_t)(src + (int32_t)ml) <= nms;
            src = ok ? src - voff : src;
        }
    }
    int32_t pos = ms, rem = (int32_t)ml, D = ms - src;
    const int32_t send = src + (int32_t)ml < ms ? src + (int32_t)ml : ms;
    {
        // one round: every ready lane copies its first (<= 16 byte) step; what
        // is left is copied by the whole wave in lane order (= output order,
        // so every source is complete when its match's turn comes)
        const bool go = pend && (send <= O0 || litsrc);
        if (zbal(go)) {
            if (go) {
                const int32_t m = rem < 16 ? (rem < D ? rem : D) : (D < 16 ? D : 16);
                zcopy16<true>(s, slot(x, pos - D), slot(x, pos), m);
                pos += m;
                rem -= m;
                if (rem <= 0) pend = false;
            }
        }
        for (uint64_t pmk = zbal(pend); pmk; pmk &= pmk - 1) {
            const int j = (int)__builtin_ctzll(pmk);
            zwave_near(s, x, (int32_t)readlane((uint32_t)pos, j), (int32_t)readlane((uint32_t)D, j),
                       (int32_t)readlane((uint32_t)rem, j));
        }
    }
    XP_ADD(4, ZP_NOW() - tq3);
}

// whole-wave copy of one long match (ring or HBM sources)
__device__ __forceinline__ void x_match(XSmem &s, X &x, uint32_t off, int32_t len) {
    const int l = lane_id();
    int32_t m = 0, step = 0;
    if (off < 64) { m = l % (int32_t)off; step = 64 % (int32_t)off; }
    for (int32_t k = 0; k < len; k += 64) {
        int32_t hi = x.op + k;
        if (hi - x.F >= FLUSH_T) xflush_line(s, x, hi);
        int32_t ringfloor = hi + 64 - R;
        int32_t i = k + l;
        int32_t src = off >= 64 ? x.op - (int32_t)off + i : x.op - (int32_t)off + m;
        bool needg = (i < len) && src < ringfloor;
        if (__ballot(needg)) {
            if (ringfloor > x.Fw) { wait_vm(); x.Fw = x.F; }
        }
        if (i < len) {
            uint32_t v = src >= ringfloor ? s.ring[slot(x, src)] : x.dst[src];
            s.ring[slot(x, x.op + i)] = (uint8_t)v;
        }
        __builtin_amdgcn_wave_barrier();
        if (off < 64) { m += step; if (m >= (int32_t)off) m -= (int32_t)off; }
    }
    x.op += len;
}

// Execute items [0, n) of a checked run (lane j holds item j): split into
// lane-parallel batches; long items are copied by the whole wave.
// (incl / lincl: inclusive prefix sums over the lanes of len and lln as
// below, computed by the caller)
__device__ __forceinline__ void x_run(XSmem &s, X &x, uint32_t n, uint32_t ll, uint32_t ml, uint32_t off,
                                      int64_t *lp, uint32_t incl, uint32_t lincl) {
    const int l = lane_id();
    const bool in = (uint32_t)l < n;
    const uint32_t len = in ? ll + ml : 0u, lln = in ? ll : 0u;
    const int32_t O0run = x.op;
    const int32_t o = O0run + (int32_t)(incl - len);
    const int32_t lit = (int32_t)*lp + (int32_t)(lincl - lln);
    const bool lng = in && (ll > (uint32_t)LONGI || ml > (uint32_t)LONGI);
    uint32_t j = 0;
    while (j < n) {
        const int32_t oj = (int32_t)readlane((uint32_t)o, (int)j), lj = (int32_t)readlane((uint32_t)lit, (int)j);
        if (readlane(lng ? 1u : 0u, (int)j)) {  // one long item, whole wave
            const uint64_t tl0 = ZP_NOW();
            const uint32_t jll = readlane(ll, (int)j), jml = readlane(ml, (int)j), joff = readlane(off, (int)j);
            x.op = oj;
            x_lit(s, x, lj, (int32_t)jll);
            if (jml) x_match(s, x, joff, (int32_t)jml);
            j++;
            XP_ADD(6, ZP_NOW() - tl0);
            continue;
        }
        // maximal batch from j: span, literal window and no long item
        const int32_t endo = o + (int32_t)len, endl = lit + (int32_t)ll;
        const bool ok = (uint32_t)l >= j && in && !lng && endo - oj <= BSPAN && endl - lj <= LW - 64;
        const uint64_t stop = __ballot(!ok) & (~0ull << j);
        const uint32_t e = stop ? (uint32_t)__builtin_ctzll(stop) : 64u;
        const uint32_t eb = e > n ? n : e;
        const bool act = (uint32_t)l >= j && (uint32_t)l < eb;
        const int32_t O1 = (int32_t)readlane((uint32_t)endo, (int)eb - 1);
        const int32_t L1 = (int32_t)readlane((uint32_t)endl, (int)eb - 1);
        const uint64_t tw0 = ZP_NOW();
        if (L1 > lj) lit_window(s, x, lj, L1 - lj);
        XP_ADD(0, ZP_NOW() - tw0);
        x_batch2(s, x, act, o, ll, ml, off, lit, oj, O1);
        x.op = O1;
        j = eb;
    }
    x.op = O0run + (int32_t)readlane(incl, 63);
    *lp += readlane(lincl, 63);
}

__global__ __launch_bounds__(64) void zexec_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                   const ZInfo *__restrict__ info, const uint8_t *__restrict__ litbuf,
                                                   const uint4 *__restrict__ items, int32_t *__restrict__ ret,
                                                   const int32_t *__restrict__ todo) {
    __shared__ XSmem s;
    const int bi = blockIdx.x;
    if (bi >= nblk) return;
    if (todo && !todo[bi]) return;  // small-batch path: replayed by the origin map
    const int l = lane_id();
    const jfs_dev_block b = blocks[bi];
    const ZInfo zi = info[bi];
    X x;
    x.dst = (g_u8 *)b.dst;
    x.lit = (const gc_u8 *)litbuf + zi.lit_off;
    x.lw0 = -(1LL << 40);
    x.cap = b.dst_cap;
    x.op = 0; x.F = 0; x.Fw = 0; x.fstart = 0; x.bug = 0;
#ifdef JFS_PROF
    for (int i = 0; i < 8; i++) x.pacc[i] = 0;
#endif
    const uint64_t tz0 = ZP_NOW();
    __builtin_amdgcn_wave_barrier();
    x.dmis = (uint32_t)((uintptr_t)b.dst & 15u);
    int32_t result = E_BUG;
    if (zi.ovf) { if (l == 0) ret[bi] = E_SCRATCH; return; }
    if (zi.n_items == 0xFFFFFFFFu) { if (l == 0) ret[bi] = -103; return; }
    const gc_u4 *it = (const gc_u4 *)items + zi.item_off;
    const uint32_t nit = zi.n_items;
    int64_t lp = 0;            // literal index
    int32_t regen = 0, lused = 0;
    uint32_t rin0 = 1, rin1 = 4, rin2 = 8;  // repeat offsets at the start of the current block
    bool done = false;
    // items one chunk ahead: the next 64 are loaded while this chunk runs
    uint4 ahead = make_uint4(0, 0, 0, 0);
    if ((uint32_t)l < nit) ahead = it[l];
    for (uint32_t base = 0; base < nit && !done; base += 64) {
        uint64_t tb0 = ZP_NOW();
        const uint4 mine = ahead;
        ahead = make_uint4(0, 0, 0, 0);
        if (base + 64 + l < nit) ahead = it[base + 64 + l];
        XP_ADD(0, ZP_NOW() - tb0);
        uint32_t cnt = nit - base < 64 ? nit - base : 64;
        const uint64_t nonseq = __ballot((uint32_t)l >= cnt || (mine.w & 0xFF) != IT_SEQ);
        for (uint32_t k = 0; k < cnt; k++) {
            uint32_t ix = readlane(mine.x, k), iy = readlane(mine.y, k), iz = readlane(mine.z, k), iw = readlane(mine.w, k);
            uint32_t kind = iw & 0xFF;
            if (kind == IT_SEQ) {
                // a run of consecutive sequence items: checks and copies in parallel
                const uint64_t rest = nonseq & (~0ull << k);
                const uint32_t r = (rest ? (uint32_t)__builtin_ctzll(rest) : 64u) - k;
                const uint32_t src_lane = k + (uint32_t)l < 64 ? k + (uint32_t)l : 63u;
                const uint32_t ll = (uint32_t)__shfl((int)mine.x, (int)src_lane, 64);
                const uint32_t ml = (uint32_t)__shfl((int)mine.y, (int)src_lane, 64);
                const uint32_t off = rep_res((uint32_t)__shfl((int)mine.z, (int)src_lane, 64), rin0, rin1, rin2);
                const bool in = (uint32_t)l < r;
                const uint32_t len = in ? ll + ml : 0u, lln = in ? ll : 0u;
                const uint32_t incl = dpp_scan_add(len), lincl = dpp_scan_add(lln);
                const int64_t o = (int64_t)x.op + (incl - len);
                const bool fdst = o + len > (int64_t)x.cap;
                const bool flit = (int64_t)lused + lincl > (int64_t)regen;
                const bool foff = ml > 0 && (int64_t)off > o + ll - x.fstart;
                const uint64_t bad = __ballot(in && (fdst || flit || foff));
                const uint32_t nexec = bad ? (uint32_t)__builtin_ctzll(bad) : r;
                const int32_t code = (int32_t)readlane(fdst ? (uint32_t)E_DSTSMALL : (uint32_t)E_CORRUPT, (int)(nexec & 63));
                // the run's prefix sums serve the copies too; only a run cut
                // short by a bad item needs them again over its first nexec lanes
                uint32_t xincl = incl, xlincl = lincl;
                if (nexec < r) {
                    const uint32_t el = (uint32_t)l < nexec ? len : 0u, ell = (uint32_t)l < nexec ? lln : 0u;
                    xincl = dpp_scan_add(el);
                    xlincl = dpp_scan_add(ell);
                }
                const uint32_t totll = readlane(xlincl, 63);
                if (nexec) x_run(s, x, nexec, ll, ml, off, &lp, xincl, xlincl);
                lused += (int32_t)totll;
                if (bad) { result = code; done = true; break; }
                k += r - 1;
            } else if (kind == IT_BSTART) {
                if (zi.lit_err_blk == ix) { result = zi.lit_err_code; done = true; break; }
                regen = (int32_t)iy;
                lused = 0;
            } else if (kind == IT_BEND) {
                int32_t rest = regen - lused;
                if ((int64_t)x.op + rest > (int64_t)x.cap) { result = E_DSTSMALL; done = true; break; }
                x_lit(s, x, lp, rest);
                lp += rest;
                lused = regen;
            } else if (kind == IT_BREP) {
                rin0 = ix; rin1 = iy; rin2 = iz;
            } else if (kind == IT_FSTART) {
                x.fstart = x.op;
            } else if (kind == IT_FEND) {
                uint32_t fl = iw >> 8;
                uint64_t fcs = (uint64_t)ix | ((uint64_t)iy << 32);
                if ((fl & FE_FCS) && (uint64_t)(x.op - x.fstart) != fcs) { result = E_CORRUPT; done = true; break; }
                if (fl & FE_MISSING) { result = E_CORRUPT; done = true; break; }
                if (fl & FE_CHECK) {
                    xflush(s, x, x.op);
                    wait_vm();
                    x.Fw = x.F;
                    uint64_t h = xxh64_dev(s, (const gc_u8 *)x.dst + x.fstart, x.op - x.fstart);
                    x.lw0 = -(1LL << 40);  // s.xxh shares the literal window's bytes
                    if ((uint32_t)h != iz) { result = E_CORRUPT; done = true; break; }
                }
            } else if (kind == IT_ERR) {
                result = (int32_t)iz;
                done = true;
                break;
            } else {
                result = -102;
                done = true;
                break;
            }
        }
    }
    if (!done) result = x.op;
    if (x.bug) result = -x.bug;
    XP_ADD(7, ZP_NOW() - tz0);
#ifdef JFS_PROF
    for (int i = 0; i < 8; i++) ZP_ADD(i, x.pacc[i]);
#endif
    xflush(s, x, x.op);
    wait_vm();
    if (l == 0) ret[bi] = result;
}

#include "zstd_split.inc"

}  // namespace zstdd
}  // namespace jfs

// ---------------------------------------------------------------------------
// host launcher: scan -> size scratch -> entropy -> execute
// ---------------------------------------------------------------------------
namespace {
// Scratch of one stream of launches: the entropy decoders' outputs (items,
// literal bytes, FSE table cells) and the per-input plan.
struct ZScratch {
    jfs::zstdd::ZInfo *d_info = nullptr;
    size_t info_cap = 0;
    uint8_t *d_lit = nullptr;
    size_t lit_cap = 0;
    uint4 *d_items = nullptr;
    size_t items_cap = 0;
    uint16_t *d_tabs = nullptr;
    size_t tabs_cap = 0;
    // device API only: the totals a launch needs (zplan -> pinned record), and
    // the event that orders launches sharing this scratch on different streams
    uint64_t *d_need = nullptr, *h_need = nullptr;
    hipEvent_t ev_need = nullptr, ev_done = nullptr;
    // small-batch path scratch (zstd_split.inc)
    uint8_t *d_split = nullptr;
    size_t split_cap = 0;
    std::mutex mu;
};
ZScratch g_scr[16];

template <class T>
bool grow_dev(T **p, size_t *cap, size_t need) {
    if (*cap >= need) return true;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    size_t n = need + need / 4;
    if (hipMalloc((void **)p, n * sizeof(T)) != hipSuccess) { *cap = 0; return false; }
    *cap = n;
    return true;
}
// Symbol_Compression_Modes reserved bits: rejected, like zstd >= 1.5 (the
// reference pins 1.5.6); see oracle/zstd_oracle.c.
constexpr int g_strict_reserved = 1;

int launch_entropy_exec(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, jfs::zstdd::ZInfo *d_info,
                        uint8_t *d_lit, uint16_t *d_tabs, uint4 *d_items, hipStream_t stream) {
    using namespace jfs::zstdd;
    hipLaunchKernelGGL(zlit_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_info, d_lit);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zseqa_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_info, d_tabs, d_items,
                       g_strict_reserved);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zbuild_kernel, dim3(nblk, ZBUILD_Q), dim3(64), 0, stream, nblk, d_info, d_tabs);
    if (hipGetLastError() != hipSuccess) return -1;
    // Workgroup 2 bi decodes input bi's blocks [0, ZNB) and never waits on
    // anything; 2 bi + 1 decodes the rest and, at its first phase C, waits for
    // the repeat offsets 2 bi publishes.  Only second halves wait, and only on
    // first halves, which always run to completion once dispatched: with the
    // round-robin XCD dispatch the first halves even land on other XCDs than
    // the waiting second halves, so those cannot crowd them out.  The wait is
    // bounded anyway (seq_group2).
    static_assert(ZSEQ_INPUTS == 1, "split inputs: one input per workgroup pair");
    hipLaunchKernelGGL(zseqb_kernel, dim3(2 * nblk), dim3(128), 0, stream, d_blocks, nblk, d_info, d_tabs, d_items);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zexec_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_info, d_lit, d_items, d_ret,
                       (const int32_t *)nullptr);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

namespace {
// Batches of at most this many inputs take the small-batch path
// (zstd_split.inc: one workgroup per block, origin-map replay);
// JFS_ZSTD_SPLIT_MAX overrides (0 = never).
int zsplit_max() {
    static int v = [] {
        const char *e = getenv("JFS_ZSTD_SPLIT_MAX");
        return e ? std::max(0, atoi(e)) : 128;
    }();
    return v;
}

int64_t a256(int64_t x) { return (x + 255) & ~255ll; }

// The small-batch path's scratch grows with the blocks (one record each) and
// the output capacity (one origin entry per byte): inputs made of very many
// tiny blocks, or huge capacities, take the one-wave path instead.
bool split_ok(int nblk, const uint64_t *tot) {
    return nblk <= zsplit_max() && tot[3] <= (uint64_t)nblk * 512 + 4096 && tot[4] <= (1ull << 30);
}

// tot: the plan totals (zplan need[] / jfs_zstd_plan_host): [3] blocks,
// [4] origin entries, [5] largest dst_cap
int64_t split_bytes(int nblk, const uint64_t *tot) {
    using namespace jfs::zstdd;
    return a256((int64_t)nblk * (int64_t)sizeof(SIn)) + a256((int64_t)tot[3] * (int64_t)sizeof(SBlk)) +
           a256((int64_t)nblk * 4) + a256((int64_t)tot[4] * 4) + 256;
}

int launch_split(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, jfs::zstdd::ZInfo *d_info, uint8_t *d_lit,
                 uint4 *d_items, void *d_split, const uint64_t *tot, hipStream_t st) {
    using namespace jfs::zstdd;
    uint8_t *p = (uint8_t *)(((uintptr_t)d_split + 255) & ~(uintptr_t)255);
    SScr sc;
    sc.in = (SIn *)p;
    p += a256((int64_t)nblk * (int64_t)sizeof(SIn));
    sc.blk = (SBlk *)p;
    p += a256((int64_t)tot[3] * (int64_t)sizeof(SBlk));
    sc.todo = (int32_t *)p;
    p += a256((int64_t)nblk * 4);
    sc.org = (int32_t *)p;
    const int64_t nbk = (int64_t)tot[3], max_cap = (int64_t)tot[5];
    hipLaunchKernelGGL(zsplan_kernel, dim3(1), dim3(64), 0, st, d_info, nblk, sc);
    hipLaunchKernelGGL(zswalk_kernel, dim3(nblk), dim3(64), 0, st, d_blocks, nblk, d_info, d_items, sc,
                       g_strict_reserved);
    if (nbk > 0)
        hipLaunchKernelGGL(zsblk_kernel, dim3((unsigned)nbk), dim3(128), 0, st, d_blocks, nblk, d_info, d_lit, d_items,
                           sc);
    hipLaunchKernelGGL(zsfix_kernel, dim3(nblk), dim3(64), 0, st, d_blocks, nblk, d_info, d_items, sc);
    if (nbk > 0)
        hipLaunchKernelGGL(zsemit_kernel, dim3((unsigned)nbk, ZSE_PARTS), dim3(ST), 0, st, nblk, (const ZInfo *)d_info,
                           (const uint4 *)d_items, sc);
    const unsigned jx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((max_cap / 4 + ST) / ST, (2048 + nblk - 1) / nblk));
    // Rounds: after round r every entry points >= SJ_HOPS^r steps up its chain
    // (or to a literal), and a step from a match byte lands in an earlier
    // sequence's output (overlaps point before their match), so a chain has
    // at most one step per sequence, <= max_cap / 3 + 1 (matches are >= 3
    // bytes): SJ_HOPS^jr above that settles every well-formed input (8 rounds
    // for 4 MiB).  The gather checks every entry regardless.
    int jr = 1;
    for (double reach = SJ_HOPS; reach <= (double)max_cap / 3 + 1 && jr < SJ_ROUNDS; reach *= SJ_HOPS) jr++;
    for (int r = 0; r < jr; r++) hipLaunchKernelGGL(zsjump_kernel, dim3(jx, (unsigned)nblk), dim3(ST), 0, st, sc, r);
    hipLaunchKernelGGL(zsgather_kernel, dim3((unsigned)((max_cap / 4 + ST) / ST), (unsigned)nblk), dim3(ST), 0, st,
                       d_blocks, (const ZInfo *)d_info, (const uint8_t *)d_lit, sc);
    hipLaunchKernelGGL(zsverd_kernel, dim3((nblk + 63) / 64), dim3(64), 0, st, nblk, sc, d_ret);
    hipLaunchKernelGGL(zexec_kernel, dim3(nblk), dim3(64), 0, st, d_blocks, nblk, (const ZInfo *)d_info,
                       (const uint8_t *)d_lit, (const uint4 *)d_items, d_ret, (const int32_t *)sc.todo);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
}  // namespace

extern "C" int jfs_zstd_split_ok(int nblk, const uint64_t *tot) { return split_ok(nblk, tot) ? 1 : 0; }
extern "C" int64_t jfs_zstd_split_bytes(int nblk, const uint64_t *tot) { return split_bytes(nblk, tot); }

// Diagnostics: inputs the small-batch path replayed itself (out[0]) and
// inputs it handed to the exact replay (out[1]) on the current device since
// the last reset; synchronous.
extern "C" int jfs_zstd_split_counts(uint64_t *out, int reset) {
    unsigned long long v[2] = {0, 0};
    if (hipMemcpyFromSymbol(v, HIP_SYMBOL(jfs::zstdd::g_zsplit_counts), sizeof(v)) != hipSuccess) return -1;
    out[0] = v[0];
    out[1] = v[1];
    if (reset) {
        unsigned long long z[2] = {0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(jfs::zstdd::g_zsplit_counts), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}

// Device API: zscan -> zplan -> entropy -> execute on `stream`.  The call
// waits once on the host for zscan/zplan (the inputs' frame headers: a few
// microseconds of kernel time after whatever `stream` already holds) to learn
// the scratch the launch needs, grows the device's scratch if it is short and
// re-plans, then enqueues the entropy and execute kernels without waiting.
// So every input fits its scratch and ret is never E_SCRATCH.
extern "C" int jfs_launch_zstd_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, uint8_t *,
                                      hipStream_t stream) {
    using namespace jfs::zstdd;
    if (nblk <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
    ZScratch &z = g_scr[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (!z.d_need) {
        if (hipMalloc((void **)&z.d_need, 6 * sizeof(uint64_t)) != hipSuccess) return -1;
        if (hipHostMalloc((void **)&z.h_need, 6 * sizeof(uint64_t), hipHostMallocDefault) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&z.ev_need, hipEventDisableTiming) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&z.ev_done, hipEventDisableTiming) != hipSuccess) return -1;
        for (int i = 0; i < 6; i++) z.h_need[i] = 0;
    }
    if ((size_t)nblk > z.info_cap) {
        // earlier launches (any stream) may still read the old scratch
        if (hipEventSynchronize(z.ev_done) != hipSuccess) return -1;
        if (!grow_dev(&z.d_info, &z.info_cap, (size_t)nblk)) return -1;
    }
    // launches that share the scratch run in call order across streams
    if (hipStreamWaitEvent(stream, z.ev_done, 0) != hipSuccess) return -1;
    hipLaunchKernelGGL(zscan_kernel, dim3((nblk + 63) / 64), dim3(64), 0, stream, d_blocks, nblk, z.d_info);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zplan_kernel, dim3(1), dim3(PLAN_T), 0, stream, z.d_info, nblk, (uint64_t)z.items_cap,
                       (uint64_t)z.lit_cap, (uint64_t)z.tabs_cap, z.d_need);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipMemcpyAsync(z.h_need, z.d_need, 6 * sizeof(uint64_t), hipMemcpyDeviceToHost, stream) != hipSuccess)
        return -1;
    if (hipEventRecord(z.ev_need, stream) != hipSuccess) return -1;
    if (hipEventSynchronize(z.ev_need) != hipSuccess) return -1;
    // zplan's overflow test: total + 64 items, + 4160 literal bytes, + 64 cells
    const uint64_t want_items = z.h_need[0] + 64, want_lits = z.h_need[1] + 4096 + 64, want_tabs = z.h_need[2] + 64;
    if (want_items > z.items_cap || want_lits > z.lit_cap || want_tabs > z.tabs_cap) {
        // every earlier launch on the scratch is done: ev_done was waited for
        // on `stream` ahead of ev_need
        if (!grow_dev(&z.d_items, &z.items_cap, want_items)) return -1;
        if (!grow_dev(&z.d_lit, &z.lit_cap, want_lits)) return -1;
        if (!grow_dev(&z.d_tabs, &z.tabs_cap, want_tabs)) return -1;
        hipLaunchKernelGGL(zplan_kernel, dim3(1), dim3(PLAN_T), 0, stream, z.d_info, nblk, (uint64_t)z.items_cap,
                           (uint64_t)z.lit_cap, (uint64_t)z.tabs_cap, z.d_need);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    uint64_t tot[6];
    for (int i = 0; i < 6; i++) tot[i] = z.h_need[i];
    if (split_ok(nblk, tot)) {
        if (!grow_dev(&z.d_split, &z.split_cap, (size_t)split_bytes(nblk, tot))) return -1;
        if (launch_split(d_blocks, nblk, d_ret, z.d_info, z.d_lit, z.d_items, z.d_split, tot, stream) != 0) return -1;
    } else if (launch_entropy_exec(d_blocks, nblk, d_ret, z.d_info, z.d_lit, z.d_tabs, z.d_items, stream) != 0) {
        return -1;
    }
    return hipEventRecord(z.ev_done, stream) == hipSuccess ? 0 : -1;
}

// Batch path (capi.hip run_batch): the caller planned the scratch on the host
// from its host copy of the inputs (jfs_zstd_plan_host) and owns the scratch
// (one per staging slot), so nothing is shared and nothing waits.
extern "C" int jfs_launch_zstd_decode_planned(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *d_info,
                                              uint8_t *d_lit, uint16_t *d_tabs, void *d_items, void *d_split,
                                              const uint64_t *tot, hipStream_t stream) {
    if (nblk <= 0) return 0;
    if (d_split && split_ok(nblk, tot))
        return launch_split(d_blocks, nblk, d_ret, (jfs::zstdd::ZInfo *)d_info, d_lit, (uint4 *)d_items, d_split, tot,
                            stream);
    return launch_entropy_exec(d_blocks, nblk, d_ret, (jfs::zstdd::ZInfo *)d_info, d_lit, d_tabs, (uint4 *)d_items,
                               stream);
}

// Host plan of a batch: info[i] (ZInfo, 64 bytes each) from the host copy of
// input i; returns the scratch totals (items, literal bytes, table cells) and
// the small-batch path's (blocks, origin entries, largest dst_cap).
extern "C" size_t jfs_zstd_info_bytes(void) { return sizeof(jfs::zstdd::ZInfo); }
extern "C" void jfs_zstd_plan_host(const uint8_t *const *srcs, const int32_t *lens, const int32_t *caps, int nblk,
                                   void *info_out, uint64_t *totals) {
    using namespace jfs::zstdd;
    ZInfo *info = (ZInfo *)info_out;
    uint64_t oi = 0, ol = 0, ot = 0, ob = 0, oo = 0, mc = 0;
    for (int i = 0; i < nblk; i++) {
        ZInfo &z = info[i];
        z = ZInfo{};
        zscan_one((const gc_u8 *)srcs[i], lens[i], caps[i], z);
        z.item_off = oi;
        z.lit_off = ol;
        z.tab_off = ot;
        z.lit_err_blk = 0xFFFFFFFFu;
        z.lit_err_code = 0;
        z.ovf = 0;
        oi += z.n_items;
        ol += (z.lit_bytes + 15u) & ~15u;
        ot += (uint64_t)z.n_cblk * TAB_STRIDE;
        const uint64_t c = caps[i] > 0 ? (uint64_t)caps[i] : 0u;
        ob += z.n_blk;
        oo += (c + 3) & ~3ull;
        mc = std::max(mc, c);
    }
    totals[0] = oi + 64;
    totals[1] = ol + 4096 + 64;
    totals[2] = ot + 64;
    totals[3] = ob;
    totals[4] = oo;
    totals[5] = mc;
}

#ifdef JFS_PROF
extern "C" int jfs_zprof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::zstdd::g_zprof), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -1;
}extern "C" int jfs_zsprof_read(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(jfs::zstdd::g_zsprof), sizeof(unsigned long long) * 8) == hipSuccess ? 0 : -1;
}
extern "C" int jfs_zsprof_reset() {
    unsigned long long z[8] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::zstdd::g_zsprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}

extern "C" int jfs_zprof_reset(void) {
    unsigned long long z[8] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(jfs::zstdd::g_zprof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif
