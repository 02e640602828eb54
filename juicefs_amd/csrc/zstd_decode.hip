// Zstd frame decoder for gfx950 (RFC 8878; behaviour of ZSTD_decompress as
// reached from pkg/compress/compress.go:94-103 via DataDog/zstd v1.5.6).
//
// Three launches per batch of inputs (one jfs_dev_block = one input buffer,
// which may hold several frames):
//
//  1. zscan     one lane per input walks frame/block/literal/sequence headers
//               and sizes the scratch exactly (literal bytes, item count).
//  2. zentropy  one 128-thread workgroup per input: wave 0 decodes literal
//               sections (Huffman 4 streams on 4 lanes, raw, RLE) into the
//               literal buffer; wave 1 decodes FSE sequence streams and
//               resolves repeat offsets into a flat item list.  The two waves
//               walk the frame independently.
//  3. zexec     one wave per input replays the items (literal copy + match
//               copy) through an 8 KiB LDS output ring, streams the output to
//               HBM, checks content size / checksum, and writes the result.
//
// Items are 16 bytes {x, y, z, kind}; errors found by the entropy waves are
// placed in stream order so zexec reports the first error libzstd would.
// Result codes match oracle/zstd_oracle.c: size, -1 corrupt, -2 dst too
// small, -3 source size wrong.
#include <hip/hip_runtime.h>

#include <mutex>
#include <vector>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace zstdd {

enum { E_CORRUPT = -1, E_DSTSMALL = -2, E_SRCSIZE = -3, E_BUG = -100 };
enum { IT_SEQ = 0, IT_FSTART = 1, IT_FEND = 2, IT_BSTART = 3, IT_BEND = 4, IT_ERR = 5 };
enum { FE_FCS = 1, FE_CHECK = 2, FE_MISSING = 4 };
constexpr uint32_t ZSTD_MAGIC = 0xFD2FB528u;
constexpr int32_t BLOCK_MAX = 128 << 10;

// per-input bookkeeping (32 bytes)
struct ZInfo {
    uint64_t item_off;      // first item (host scan)
    uint64_t lit_off;       // first literal byte (host scan)
    uint32_t n_items;       // zscan: capacity
    uint32_t lit_bytes;     // zscan: capacity
    uint32_t lit_err_blk;   // zentropy wave 0: ordinal of the block whose literals failed
    int32_t lit_err_code;
};

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

__device__ __forceinline__ uint32_t rd8(const gc_u8 *s, int32_t p) { return s[p]; }
__device__ __forceinline__ uint32_t rd16(const gc_u8 *s, int32_t p) { return s[p] | (s[p + 1] << 8); }
__device__ __forceinline__ uint32_t rd24(const gc_u8 *s, int32_t p) { return rd16(s, p) | (s[p + 2] << 16); }
__device__ __forceinline__ uint32_t rd32(const gc_u8 *s, int32_t p) { return rd16(s, p) | (rd16(s, p + 2) << 16); }

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

__device__ __forceinline__ void walk_init(Walk &w, const gc_u8 *s, int32_t n, int32_t cap) {
    w.s = s; w.n = n; w.p = 0; w.cap = cap; w.lb = 0; w.phase = 0; w.frames_done = 0; w.after_last = 0;
    w.check = 0; w.has_fcs = 0; w.fcs = 0; w.ordinal = 0; w.btype = 0; w.bsize = 0; w.bpos = 0;
}

// Next event.  *err for EV_ERROR; for EV_FEND *flags/*chk describe the frame end.
__device__ __forceinline__ int walk_next(Walk &w, int32_t *err, uint32_t *flags, uint32_t *chk) {
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
__device__ __forceinline__ int32_t lit_header(const gc_u8 *s, int32_t bpos, int32_t bsize, LitHdr &h) {
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
__device__ __forceinline__ int32_t nbseq_header(const gc_u8 *s, int32_t ip, int32_t end, int32_t *nseq, int32_t *used) {
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

// read n (0..32) bits MSB-first
__device__ __forceinline__ uint32_t br_read(BR &r, int n) {
    if (n == 0) return 0u;
    int32_t lo = r.left - n;
    uint64_t v64 = r.c >> (uint32_t)(lo - 8 * r.cb);
    uint32_t v = (uint32_t)v64 & (uint32_t)(0xFFFFFFFFull >> (32 - n));
    int32_t d = 8 * r.m - lo;
    if (d > 0) v = d >= n ? 0u : v & ~((1u << d) - 1u);
    r.left = lo;
    br_refill(r);
    return v;
}
__device__ __forceinline__ uint32_t br_peek(const BR &r, int n) {
    int32_t lo = r.left - n;
    uint32_t v = (uint32_t)(r.c >> (uint32_t)(lo - 8 * r.cb)) & ((1u << n) - 1u);
    int32_t d = 8 * r.m - lo;
    if (d > 0) v = d >= n ? 0u : v & ~((1u << d) - 1u);
    return v;
}
__device__ __forceinline__ void br_skip(BR &r, int n) {
    r.left -= n;
    br_refill(r);
}
__device__ __forceinline__ bool br_overflow(const BR &r) { return r.left < 8 * r.m; }
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

__device__ __forceinline__ void build_rle(uint32_t *t, uint32_t sym) {
    if (lane_id() == 0) t[0] = sym;
}

// ---------------------------------------------------------------------------
// kernel 1: header scan -> scratch sizes
// ---------------------------------------------------------------------------
__global__ void zscan_kernel(const jfs_dev_block *__restrict__ blocks, int nblk, ZInfo *__restrict__ info) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nblk) return;
    jfs_dev_block b = blocks[i];
    Walk w;
    walk_init(w, (const gc_u8 *)b.src, b.src_len, b.dst_cap);
    uint64_t items = 0, lits = 0;
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
        items += (uint64_t)nseq;
        w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
    }
    info[i].n_items = (uint32_t)(items + 1);
    info[i].lit_bytes = (uint32_t)(lits + 16);
}

// ---------------------------------------------------------------------------
// kernel 2: entropy decode (wave 0 literals, wave 1 sequences)
// ---------------------------------------------------------------------------
struct LitSmem {
    uint16_t huf[4096];  // sym | nb << 8
    uint8_t stage[256];
    uint8_t w[260];
    int16_t norm[256];
    uint8_t symat[64];
    uint16_t symnext[256];
    uint32_t fse[64];    // weight FSE table (al <= 6)
    uint32_t rank[16];
    int32_t maxbits, valid;
};
struct SeqSmem {
    uint32_t ll[512], of[256], ml[512];
    uint8_t stage[256];
    int16_t norm[64];
    uint8_t symat[512];
    uint16_t symnext[64];
    int32_t al_ll, al_of, al_ml, have_ll, have_of, have_ml;
};
struct ZASmem {
    LitSmem lit;
    SeqSmem seq;
};

// stage `n` (<= 256) bytes starting at s+p into LDS (zero-padded)
__device__ __forceinline__ void stage_bytes(uint8_t *dst, const gc_u8 *s, int32_t p, int32_t n) {
    const int l = lane_id();
    for (int k = l; k < 256; k += 64) dst[k] = k < n ? s[p + k] : 0;
    __builtin_amdgcn_wave_barrier();
}

// Huffman table description -> sm.huf.  Returns bytes used or -1.
__device__ __forceinline__ int32_t read_huf(LitSmem &sm, const gc_u8 *in, const gc_u8 *s, int32_t p, int32_t n) {
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
        if (build_fse(sm.fse, sm.norm, maxsym, al, sm.symnext, sm.symat)) return -1;
        __builtin_amdgcn_wave_barrier();
        BR r;
        if (!br_init(r, in, s + p + 1 + c, hb - c)) return -1;
        uint32_t s1 = br_read(r, al), s2 = br_read(r, al);
        for (;;) {
            if (nw > 253) return -1;
            uint32_t e1 = sm.fse[s1];
            if (l == 0) sm.w[nw] = (uint8_t)(e1 & 0xFF);
            nw++;
            s1 = (e1 >> 16) + br_read(r, (e1 >> 8) & 0xFF);
            if (br_overflow(r)) { if (l == 0) sm.w[nw] = (uint8_t)(sm.fse[s2] & 0xFF); nw++; break; }
            if (nw > 253) return -1;
            uint32_t e2 = sm.fse[s2];
            if (l == 0) sm.w[nw] = (uint8_t)(e2 & 0xFF);
            nw++;
            s2 = (e2 >> 16) + br_read(r, (e2 >> 8) & 0xFF);
            if (br_overflow(r)) { if (l == 0) sm.w[nw] = (uint8_t)(sm.fse[s1] & 0xFF); nw++; break; }
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
    __builtin_amdgcn_wave_barrier();
    // rank starts (weight ascending, then symbol order)
    uint32_t cnt = 0;
    for (int i = 0; i < nw; i++) cnt += (sm.w[i] == (uint32_t)l) ? 1u : 0u;  // lane k counts weight k
    uint32_t span = (l >= 1 && l <= 12) ? (cnt << (l - 1)) : 0u;
    uint32_t incl = dpp_scan_add(span);
    uint32_t start = incl - span;
    if (l < 16) sm.rank[l] = start;
    __builtin_amdgcn_wave_barrier();
    // fill: symbol by symbol, lanes over its 2^(w-1) cells
    for (int i = 0; i < nw; i++) {
        uint32_t wi = sm.w[i];
        if (!wi) continue;
        uint32_t len = 1u << (wi - 1);
        uint32_t st = sm.rank[wi];
        uint16_t e = (uint16_t)(i | ((maxbits + 1 - wi) << 8));
        for (uint32_t u = l; u < len; u += 64) sm.huf[st + u] = e;
        __builtin_amdgcn_wave_barrier();
        if (l == 0) sm.rank[wi] = st + len;
        __builtin_amdgcn_wave_barrier();
    }
    sm.maxbits = maxbits;  // (uniform store)
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
    if (h.type == 2) {
        int32_t u = read_huf(sm, in, s, p, n);
        if (u < 0) return E_CORRUPT;
        if (u >= n) return E_CORRUPT;  // table must leave room for the streams
        if (l == 0) sm.valid = 1;
        p += u;
        n -= u;
    } else if (!sm.valid) {
        return E_CORRUPT;
    }
    const int32_t maxbits = sm.maxbits;
    // stream geometry (lane k < streams decodes stream k)
    int32_t mysp = p, mysn = n, mycnt = h.regen;
    int64_t o = lpos;
    if (h.streams == 4) {
        if (n < 10) return E_CORRUPT;
        int32_t s1 = (int32_t)rd16(s, p), s2 = (int32_t)rd16(s, p + 2), s3 = (int32_t)rd16(s, p + 4);
        int32_t s4 = n - 6 - s1 - s2 - s3;
        if (s4 < 1) return E_CORRUPT;
        int32_t seg = (h.regen + 3) / 4;
        mysp = p + 6 + (l >= 1 ? s1 : 0) + (l >= 2 ? s2 : 0) + (l >= 3 ? s3 : 0);
        mysn = l == 0 ? s1 : l == 1 ? s2 : l == 2 ? s3 : s4;
        int32_t c4 = h.regen - 3 * seg;
        mycnt = l < 3 ? seg : (c4 > 0 ? c4 : 0);
        o = lpos + (int64_t)(l < 3 ? l : 3) * seg;
    }
    // lanes 0..3 decode one stream each
    int32_t bad = 0;
    if (l < h.streams) {
        BR r;
        if (!br_init(r, in, s + mysp, mysn)) {
            bad = 1;
        } else {
            const int64_t start = o, end = o + mycnt;
            uint32_t acc = 0;
            for (; o < end; o++) {
                uint32_t v = br_peek(r, maxbits);
                uint32_t e = sm.huf[v];
                acc |= (e & 0xFF) << (8 * (o & 3));
                br_skip(r, (int)(e >> 8));
                if (((o + 1) & 3) == 0) { put_word(lb, start, o + 1, acc); acc = 0; }
            }
            if (o & 3) {
                for (int64_t q = (o & ~3LL) > start ? (o & ~3LL) : start; q < o; q++) lb[q] = (uint8_t)(acc >> (8 * (q & 3)));
            }
            if (!br_done(r)) bad = 1;
        }
    }
    bad = (int32_t)dwave_max((uint32_t)bad);
    return bad ? E_CORRUPT : 0;
}

// one item into the wave's 64-entry store buffer
struct ItemBuf {
    uint4 v;
    int32_t cnt;
    uint64_t pos;    // next item index (absolute in the item buffer)
    uint64_t limit;  // capacity end
    int32_t bug;
};
__device__ __forceinline__ void item_flush(ItemBuf &b, g_u4 *items) {
    const int l = lane_id();
    if (b.cnt == 0) return;
    if (b.pos + (uint64_t)b.cnt > b.limit) { b.bug = 1; b.cnt = 0; return; }
    if (l < b.cnt) items[b.pos + l] = b.v;
    b.pos += b.cnt;
    b.cnt = 0;
}
__device__ __forceinline__ void item_put(ItemBuf &b, g_u4 *items, uint32_t x, uint32_t y, uint32_t z, uint32_t kind) {
    if (lane_id() == b.cnt) b.v = make_uint4(x, y, z, kind);
    b.cnt++;
    if (b.cnt == 64) item_flush(b, items);
}

// sequence table for one field; returns bytes used or -1
__device__ __forceinline__ int32_t seq_table(SeqSmem &sm, uint32_t *t, int32_t *al, int32_t *have, int32_t mode,
                                             const gc_u8 *s, int32_t p, int32_t n, int which) {
    const int16_t *def = which == 0 ? LL_DEF : which == 1 ? OF_DEF : ML_DEF;
    int32_t maxsym = which == 0 ? 35 : which == 1 ? 31 : 52;
    int32_t defal = which == 1 ? 5 : 6, defmax = which == 0 ? 35 : which == 1 ? 28 : 52;
    int32_t maxal = which == 1 ? 8 : 9;
    const int l = lane_id();
    if (mode == 0) {
        for (int i = l; i <= defmax; i += 64) sm.norm[i] = def[i];
        __builtin_amdgcn_wave_barrier();
        if (build_fse(t, sm.norm, defmax, defal, sm.symnext, sm.symat)) return -1;
        *al = defal; *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (n < 1) return -1;
        uint32_t v = rd8(s, p);
        if ((int32_t)v > maxsym) return -1;
        build_rle(t, v);
        *al = 0; *have = 1;
        return 1;
    }
    if (mode == 2) {
        int32_t k = n < 256 ? n : 256;
        stage_bytes(sm.stage, s, p, k);
        int32_t ms = maxsym, a = 0;
        int32_t c = read_ncount(sm.stage, k, sm.norm, &ms, &a, maxal);
        if (c < 0 || c > n) return -1;
        __builtin_amdgcn_wave_barrier();
        if (build_fse(t, sm.norm, ms, a, sm.symnext, sm.symat)) return -1;
        *al = a; *have = 1;
        return c;
    }
    return *have ? 0 : -1;
}

__device__ __forceinline__ void seq_wave(SeqSmem &sm, const jfs_dev_block &b, ZInfo &zi, g_u4 *items, int strict_reserved) {
    const int l = lane_id();
    const gc_u8 *s = (const gc_u8 *)b.src;
    Walk w;
    walk_init(w, s, b.src_len, b.dst_cap);
    ItemBuf ib;
    ib.cnt = 0; ib.pos = zi.item_off; ib.limit = zi.item_off + zi.n_items; ib.bug = 0; ib.v = make_uint4(0, 0, 0, 0);
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    for (;;) {
        int32_t err = 0;
        uint32_t fl = 0, chk = 0;
        int ev = walk_next(w, &err, &fl, &chk);
        if (ev == EV_DONE) break;
        if (ev == EV_ERROR) { item_put(ib, items, 0, 0, (uint32_t)err, IT_ERR); break; }
        if (ev == EV_FSTART) {
            rep0 = 1; rep1 = 4; rep2 = 8;
            if (l == 0) { sm.have_ll = 0; sm.have_of = 0; sm.have_ml = 0; }
            __builtin_amdgcn_wave_barrier();
            item_put(ib, items, 0, 0, 0, IT_FSTART);
            continue;
        }
        if (ev == EV_FEND) {
            item_put(ib, items, (uint32_t)w.fcs, (uint32_t)(w.fcs >> 32), chk, IT_FEND | (fl << 8));
            if (fl & FE_MISSING) break;
            continue;
        }
        // block
        const uint32_t ord = w.ordinal - 1;
        if (w.btype != 2) {
            item_put(ib, items, ord, (uint32_t)w.bsize, 0, IT_BSTART);
            item_put(ib, items, (uint32_t)w.bsize, 0, 0, IT_SEQ);
            item_put(ib, items, 0, 0, 0, IT_BEND);
            w.lb += w.bsize;
            continue;
        }
        LitHdr h;
        int32_t e = lit_header(s, w.bpos, w.bsize, h);
        item_put(ib, items, ord, e ? 0u : (uint32_t)h.regen, 0, IT_BSTART);
        if (e) { item_put(ib, items, 0, 0, (uint32_t)e, IT_ERR); break; }
        const int32_t end = w.bpos + w.bsize;
        int32_t ip = w.bpos + h.sec;
        int32_t nseq = 0, used = 0;
        e = nbseq_header(s, ip, end, &nseq, &used);
        if (e) { item_put(ib, items, 0, 0, (uint32_t)e, IT_ERR); break; }
        ip += used;
        w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
        if (nseq == 0) {
            item_put(ib, items, 0, 0, 0, IT_BEND);
            continue;
        }
        if (ip + 1 > end) { item_put(ib, items, 0, 0, (uint32_t)E_SRCSIZE, IT_ERR); break; }
        uint32_t modes = rd8(s, ip++);
        if ((modes & 3) && strict_reserved) { item_put(ib, items, 0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
        int32_t al_ll = sm.al_ll, al_of = sm.al_of, al_ml = sm.al_ml;
        int32_t hv_ll = sm.have_ll, hv_of = sm.have_of, hv_ml = sm.have_ml;
        int32_t c = seq_table(sm, sm.ll, &al_ll, &hv_ll, modes >> 6, s, ip, end - ip, 0);
        if (c >= 0) { ip += c; c = seq_table(sm, sm.of, &al_of, &hv_of, (modes >> 4) & 3, s, ip, end - ip, 1); }
        if (c >= 0) { ip += c; c = seq_table(sm, sm.ml, &al_ml, &hv_ml, (modes >> 2) & 3, s, ip, end - ip, 2); }
        if (c < 0) { item_put(ib, items, 0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
        ip += c;
        if (l == 0) {
            sm.al_ll = al_ll; sm.al_of = al_of; sm.al_ml = al_ml;
            sm.have_ll = hv_ll; sm.have_of = hv_of; sm.have_ml = hv_ml;
        }
        __builtin_amdgcn_wave_barrier();
        BR r;
        if (!br_init(r, s, s + ip, end - ip)) { item_put(ib, items, 0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
        uint32_t sll = br_read(r, al_ll), sof = br_read(r, al_of), sml = br_read(r, al_ml);
        bool failed = false;
        for (int32_t i = 0; i < nseq; i++) {
            if (br_overflow(r)) { failed = true; break; }
            uint32_t el = sm.ll[sll], eo = sm.of[sof], em = sm.ml[sml];
            uint32_t llc = el & 0xFF, ofc = eo & 0xFF, mlc = em & 0xFF;
            uint32_t ofv = (1u << ofc) + br_read(r, (int)ofc);  // offset bits first
            uint32_t ml = ML_BASE[mlc] + br_read(r, ML_BITS[mlc]);
            uint32_t ll = LL_BASE[llc] + br_read(r, LL_BITS[llc]);
            uint32_t off;
            if (ofv > 3) {
                off = ofv - 3;
                rep2 = rep1; rep1 = rep0; rep0 = off;
            } else {
                uint32_t k = ofv - 1 + (ll == 0 ? 1u : 0u);
                if (k == 0) {
                    off = rep0;
                } else {
                    uint32_t t = k == 3 ? rep0 - 1 : (k == 1 ? rep1 : rep2);
                    if (t == 0) t = 1;
                    if (k != 1) rep2 = rep1;
                    rep1 = rep0;
                    rep0 = t;
                    off = t;
                }
            }
            if (i + 1 < nseq) {
                sll = (el >> 16) + br_read(r, (int)((el >> 8) & 0xFF));
                sml = (em >> 16) + br_read(r, (int)((em >> 8) & 0xFF));
                sof = (eo >> 16) + br_read(r, (int)((eo >> 8) & 0xFF));
            }
            item_put(ib, items, ll, ml, off, IT_SEQ);
        }
        if (failed || !br_done(r)) { item_put(ib, items, 0, 0, (uint32_t)E_CORRUPT, IT_ERR); break; }
        item_put(ib, items, 0, 0, 0, IT_BEND);
    }
    item_flush(ib, items);
    if (ib.bug) item_flush(ib, items);
    // item count for zexec (the buffer ends with at least one terminator: DONE)
    if (l == 0) zi.n_items = ib.bug ? 0xFFFFFFFFu : (uint32_t)(ib.pos - zi.item_off);
}

__device__ __forceinline__ void lit_wave(LitSmem &sm, const jfs_dev_block &b, ZInfo &zi, g_u8 *litbuf) {
    const int l = lane_id();
    const gc_u8 *s = (const gc_u8 *)b.src;
    Walk w;
    walk_init(w, s, b.src_len, b.dst_cap);
    int64_t lpos = (int64_t)zi.lit_off;
    const int64_t lend = (int64_t)zi.lit_off + zi.lit_bytes;
    uint32_t err_blk = 0xFFFFFFFFu;
    int32_t err_code = 0;
    if (l == 0) sm.valid = 0;
    __builtin_amdgcn_wave_barrier();
    for (;;) {
        int32_t err = 0;
        uint32_t fl = 0, chk = 0;
        int ev = walk_next(w, &err, &fl, &chk);
        if (ev == EV_DONE || ev == EV_ERROR) break;
        if (ev == EV_FSTART) {
            if (l == 0) sm.valid = 0;
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
                if (lpos + w.bsize > lend) { err_blk = ord; err_code = E_BUG; break; }
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
        if (e) { err_blk = ord; err_code = e; break; }
        if (lpos + h.regen + 4 > lend) { err_blk = ord; err_code = E_BUG; break; }
        e = lit_block(sm, s, s, h, w.bpos, litbuf, lpos);
        if (e) { err_blk = ord; err_code = e; break; }
        lpos += h.regen;
        int32_t nseq = 0, used = 0;
        if (nbseq_header(s, w.bpos + h.sec, w.bpos + w.bsize, &nseq, &used)) break;  // reported by the seq wave
        w.lb += (int64_t)h.regen + 3 * (int64_t)nseq;
    }
    if (l == 0) {
        zi.lit_err_blk = err_blk;
        zi.lit_err_code = err_code;
    }
}

__global__ __launch_bounds__(128) void zentropy_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                       ZInfo *__restrict__ info, uint8_t *__restrict__ litbuf,
                                                       uint4 *__restrict__ items, int strict_reserved) {
    __shared__ ZASmem sm;
    const int bi = blockIdx.x;
    if (bi >= nblk) return;
    const jfs_dev_block b = blocks[bi];
    ZInfo &zi = info[bi];
    if (threadIdx.x < 64) lit_wave(sm.lit, b, zi, (g_u8 *)litbuf);
    else seq_wave(sm.seq, b, zi, (g_u4 *)items, strict_reserved);
}

// ---------------------------------------------------------------------------
// kernel 3: execute items
// ---------------------------------------------------------------------------
constexpr int R = 8192;
constexpr int RMASK = R - 1;
constexpr int LW = 4096;          // literal staging window
constexpr int FLUSH_T = 1024;

struct XSmem {
    alignas(16) uint8_t ring[R];
    alignas(16) uint8_t lw[LW];
    uint64_t xxh[4];
};

struct X {
    g_u8 *dst;
    const gc_u8 *lit;      // literal buffer of this input
    int64_t lw0;           // literal index of lw[0]
    int32_t cap, op, F, Fw, fstart;
    uint32_t dmis;
};

__device__ __forceinline__ uint32_t slot(const X &x, int32_t pos) { return (uint32_t)(pos + (int32_t)x.dmis) & RMASK; }

__device__ __forceinline__ void xflush(XSmem &s, X &x, int32_t to) {
    const int l = lane_id();
    wait_vm();
    x.Fw = x.F;
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
__device__ __forceinline__ void xflush_line(XSmem &s, X &x, int32_t hi) {
    int32_t to = (int32_t)(((uint32_t)hi + x.dmis) & ~127u) - (int32_t)x.dmis;
    if (to > x.F) xflush(s, x, to);
}

// make lit[lp, lp+64) resident in the staging window
__device__ __forceinline__ void lit_window(XSmem &s, X &x, int64_t lp) {
    if (lp >= x.lw0 && lp + 64 <= x.lw0 + LW) return;
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

__global__ __launch_bounds__(64) void zexec_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                   const ZInfo *__restrict__ info, const uint8_t *__restrict__ litbuf,
                                                   const uint4 *__restrict__ items, int32_t *__restrict__ ret) {
    __shared__ XSmem s;
    const int bi = blockIdx.x;
    if (bi >= nblk) return;
    const int l = lane_id();
    const jfs_dev_block b = blocks[bi];
    const ZInfo zi = info[bi];
    X x;
    x.dst = (g_u8 *)b.dst;
    x.lit = (const gc_u8 *)litbuf + zi.lit_off;
    x.lw0 = -(1LL << 40);
    x.cap = b.dst_cap;
    x.op = 0; x.F = 0; x.Fw = 0; x.fstart = 0;
    x.dmis = (uint32_t)((uintptr_t)b.dst & 15u);
    int32_t result = E_BUG;
    if (zi.n_items == 0xFFFFFFFFu) { if (l == 0) ret[bi] = E_BUG; return; }
    const gc_u4 *it = (const gc_u4 *)items + zi.item_off;
    const uint32_t nit = zi.n_items;
    int64_t lp = 0;            // literal index
    int32_t regen = 0, lused = 0;
    bool done = false;
    for (uint32_t base = 0; base < nit && !done; base += 64) {
        uint4 mine = make_uint4(0, 0, 0, 0);
        if (base + l < nit) mine = it[base + l];
        uint32_t cnt = nit - base < 64 ? nit - base : 64;
        for (uint32_t k = 0; k < cnt; k++) {
            uint32_t ix = readlane(mine.x, k), iy = readlane(mine.y, k), iz = readlane(mine.z, k), iw = readlane(mine.w, k);
            uint32_t kind = iw & 0xFF;
            if (kind == IT_SEQ) {
                int64_t ll = ix, ml = iy;
                if ((int64_t)x.op + ll + ml > (int64_t)x.cap) { result = E_DSTSMALL; done = true; break; }
                if ((int64_t)lused + ll > (int64_t)regen) { result = E_CORRUPT; done = true; break; }
                x_lit(s, x, lp, (int32_t)ll);
                lp += ll;
                lused += (int32_t)ll;
                if (ml) {
                    if ((int64_t)iz > (int64_t)(x.op - x.fstart)) { result = E_CORRUPT; done = true; break; }
                    x_match(s, x, iz, (int32_t)ml);
                }
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
                    if ((uint32_t)h != iz) { result = E_CORRUPT; done = true; break; }
                }
            } else if (kind == IT_ERR) {
                result = (int32_t)iz;
                done = true;
                break;
            } else {
                result = E_BUG;
                done = true;
                break;
            }
        }
    }
    if (!done) result = x.op;
    xflush(s, x, x.op);
    wait_vm();
    if (l == 0) ret[bi] = result;
}

}  // namespace zstdd
}  // namespace jfs

// ---------------------------------------------------------------------------
// host launcher: scan -> size scratch -> entropy -> execute
// ---------------------------------------------------------------------------
namespace {
struct ZScratch {
    int dev = -1;
    jfs::zstdd::ZInfo *d_info = nullptr, *h_info = nullptr;
    size_t info_cap = 0;
    uint8_t *d_lit = nullptr;
    size_t lit_cap = 0;
    uint4 *d_items = nullptr;
    size_t items_cap = 0;
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
}  // namespace

extern "C" int jfs_launch_zstd_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, uint8_t *,
                                      hipStream_t stream) {
    using namespace jfs::zstdd;
    if (nblk <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
    ZScratch &z = g_scr[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (z.info_cap < (size_t)nblk) {
        if (z.d_info) (void)hipFree(z.d_info);
        if (z.h_info) (void)hipHostFree(z.h_info);
        z.d_info = nullptr; z.h_info = nullptr; z.info_cap = 0;
        if (hipMalloc((void **)&z.d_info, sizeof(ZInfo) * nblk) != hipSuccess) return -1;
        if (hipHostMalloc((void **)&z.h_info, sizeof(ZInfo) * nblk, hipHostMallocDefault) != hipSuccess) return -1;
        z.info_cap = nblk;
    }
    hipLaunchKernelGGL(zscan_kernel, dim3((nblk + 63) / 64), dim3(64), 0, stream, d_blocks, nblk, z.d_info);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipMemcpyAsync(z.h_info, z.d_info, sizeof(ZInfo) * nblk, hipMemcpyDeviceToHost, stream) != hipSuccess)
        return -1;
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    uint64_t items = 0, lits = 0;
    for (int i = 0; i < nblk; i++) {
        z.h_info[i].item_off = items;
        z.h_info[i].lit_off = lits;
        items += z.h_info[i].n_items;
        lits += (z.h_info[i].lit_bytes + 15) & ~15u;
        z.h_info[i].lit_err_blk = 0xFFFFFFFFu;
        z.h_info[i].lit_err_code = 0;
    }
    if (!grow_dev(&z.d_items, &z.items_cap, items + 64)) return -1;
    if (!grow_dev(&z.d_lit, &z.lit_cap, lits + 4096 + 64)) return -1;
    if (hipMemcpyAsync(z.d_info, z.h_info, sizeof(ZInfo) * nblk, hipMemcpyHostToDevice, stream) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(zentropy_kernel, dim3(nblk), dim3(128), 0, stream, d_blocks, nblk, z.d_info, z.d_lit,
                       z.d_items, g_strict_reserved);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(zexec_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, z.d_info, z.d_lit, z.d_items,
                       d_ret);
    if (hipGetLastError() != hipSuccess) return -1;
    // keep the pinned mirror alive until the H2D copy has run
    if (hipStreamSynchronize(stream) != hipSuccess) return -1;
    return 0;
}
