/* CPU oracle (TEST INFRASTRUCTURE ONLY -- never linked into the product):
 * a restatement of ZSTD_compress(dst, cap, src, n, 1) of libzstd 1.4.9, the
 * encoder behind pkg/compress/compress.go:82-91 (ZStandard.Compress ->
 * zstd.CompressLevel(dst, src, 1) of github.com/DataDog/zstd; the reference
 * pins v1.5.6, which is not available offline).  Pinned by
 * tests/test_zstd_l1_oracle.py against the level-1 frames of
 * tests/golden/zstd_golden.json (generated from /opt/conda/lib/libzstd 1.4.9
 * by tests/golden/make_golden.py) and, where that library loads, against
 * ZSTD_compress itself on seeded inputs of every size class.
 *
 * What it restates (libzstd 1.4.9 file:function):
 *   compress/zstd_compress.c   ZSTD_getCParams (level 1 rows) +
 *                              ZSTD_adjustCParams_internal, ZSTD_writeFrameHeader,
 *                              ZSTD_compress_frameChunk, ZSTD_compressBlock_internal
 *                              (raw / RLE block rules, repcode + entropy
 *                              confirmation), ZSTD_entropyCompressSequences(_internal),
 *                              ZSTD_seqToCodes, ZSTD_buildCTable,
 *                              ZSTD_selectEncodingType (strategy < lazy),
 *                              ZSTD_encodeSequences, ZSTD_writeEpilogue
 *   compress/zstd_fast.c       ZSTD_compressBlock_fast_generic (ip0/ip1 loop)
 *   compress/zstd_compress_literals.c  ZSTD_compressLiterals
 *   compress/huf_compress.c    HUF_compress_internal, HUF_buildCTable_wksp
 *                              (HUF_sort, HUF_setMaxHeight), HUF_writeCTable,
 *                              HUF_compressWeights, HUF_compress{1X,4X}_usingCTable
 *   compress/fse_compress.c    FSE_optimalTableLog, FSE_normalizeCount (+M2),
 *                              FSE_writeNCount, FSE_buildCTable_wksp,
 *                              FSE_compress_usingCTable
 * The code is written from the format (RFC 8878) and those functions' rules;
 * it is structured for checking, not speed.
 */
/*  Third-party notice.  Byte parity with libzstd forces its exact heuristics,
 * so the following routines are transliterated from Zstandard (libzstd 1.4.9,
 * https://github.com/facebook/zstd), Copyright (c) 2016-present, Yann Collet,
 * Facebook, Inc.  All rights reserved.  Used under the BSD licence of that
 * source tree:
 *   FSE_normalizeCount and FSE_normalizeM2 (fse_compress.c), including its
 *   rtbTable constants; FSE_writeNCount (fse_compress.c); HUF_setMaxHeight
 *   and HUF_buildCTable_wksp (huf_compress.c).
 * Redistribution and use in source and binary forms, with or without
 * modification, are permitted provided that the following conditions are met:
 *  * Redistributions of source code must retain the above copyright notice,
 *    this list of conditions and the following disclaimer.
 *  * Redistributions in binary form must reproduce the above copyright notice,
 *    this list of conditions and the following disclaimer in the documentation
 *    and/or other materials provided with the distribution.
 *  * Neither the name Facebook nor the names of its contributors may be used to
 *    endorse or promote products derived from this software without specific
 *    prior written permission.
 * THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS"
 * AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
 * IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE
 * DISCLAIMED.  IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE
 * FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL
 * DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
 * SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER
 * CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY,
 * OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE
 * OF THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* gcc cannot see that FSE_compress_usingCTable's parity steps never read
 * before the weights array; silence its -Warray-bounds guess */
#pragma GCC diagnostic ignored "-Warray-bounds"

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;

static unsigned hb32(u32 v) { return 31u - (unsigned)__builtin_clz(v); }
static u32 rd32(const u8 *p) { u32 v; memcpy(&v, p, 4); return v; }
static u64 rd64(const u8 *p) { u64 v; memcpy(&v, p, 8); return v; }

/* ---------------------------------------------------------------- params */
typedef struct {
    unsigned wlog, hlog, mls;
} zl1_params;

/* ZSTD_getCParams(1, n, 0): row "level 1" of the size tier, then
 * ZSTD_adjustCParams_internal (window shrunk to the input, hashLog <= wlog+1,
 * windowLog >= 10). */
zl1_params zl1_get_params(u64 n) {
    zl1_params p;
    /* tiers: > 256 KiB, <= 256 KiB, <= 128 KiB, <= 16 KiB (W, H, minMatch) */
    if (n > (256u << 10)) { p.wlog = 19; p.hlog = 14; p.mls = 7; }
    else if (n > (128u << 10)) { p.wlog = 18; p.hlog = 14; p.mls = 6; }
    else if (n > (16u << 10)) { p.wlog = 17; p.hlog = 13; p.mls = 6; }
    else { p.wlog = 14; p.hlog = 15; p.mls = 5; }
    {
        const u32 t = (u32)n;
        const unsigned srclog = t < 64 ? 6 : hb32(t - 1) + 1;
        if (p.wlog > srclog) p.wlog = srclog;
    }
    if (p.hlog > p.wlog + 1) p.hlog = p.wlog + 1;
    if (p.wlog < 10) p.wlog = 10;
    return p;
}

int oracle_zstd_l1_params(int64_t n, int32_t *out3) {
    zl1_params p = zl1_get_params((u64)n);
    out3[0] = (int32_t)p.wlog;
    out3[1] = (int32_t)p.hlog;
    out3[2] = (int32_t)p.mls;
    return 0;
}

static u32 zhash(const u8 *p, unsigned h, unsigned mls) {
    switch (mls) {
    case 5: return (u32)(((rd64(p) << 24) * 889523592379ull) >> (64 - h));
    case 6: return (u32)(((rd64(p) << 16) * 227718039650203ull) >> (64 - h));
    case 7: return (u32)(((rd64(p) << 8) * 58295818150454627ull) >> (64 - h));
    case 8: return (u32)((rd64(p) * 0xCF1BBCDCB7A56463ull) >> (64 - h));
    default: return (rd32(p) * 2654435761u) >> (32 - h);
    }
}

/* ---------------------------------------------------------------- sequences */
typedef struct {
    u32 ll, mlb, ofv; /* literal length, match length - 3, Offset_Value (1..3 repeat, else offset + 3) */
} zseq;

typedef struct {
    zseq *seq;
    size_t ns;
    u8 *lit;
    size_t nl;
} zseqstore;

static void store_seq(zseqstore *s, size_t ll, const u8 *lits, u32 offcode, size_t mlb) {
    memcpy(s->lit + s->nl, lits, ll);
    s->nl += ll;
    s->seq[s->ns].ll = (u32)ll;
    s->seq[s->ns].mlb = (u32)mlb;
    s->seq[s->ns].ofv = offcode + 1;
    s->ns++;
}

static size_t zcount(const u8 *a, const u8 *b, const u8 *aend) {
    const u8 *a0 = a;
    while (a < aend && *a == *b) { a++; b++; }
    return (size_t)(a - a0);
}

/* ZSTD_compressBlock_fast_generic (1.4.9): frame-relative positions, the hash
 * table holds index = position + 1 (0 = empty: the window's dictLimit is 1).
 * Returns the number of last literals; rep[0..1] in/out. */
static size_t fast_block(u32 *T, const zl1_params *P, const u8 *base, size_t bs, size_t be, u32 rep[2],
                         zseqstore *ss) {
    const unsigned hlog = P->hlog, mls = P->mls;
    const size_t stepSize = 2; /* targetLength 0: 0 + !0 + 1 */
    const u64 maxDist = 1ull << P->wlog;
    const u8 *const istart = base + bs;
    const u8 *const iend = base + be;
    const size_t prefixPos = be > maxDist ? (size_t)(be - maxDist) : 0; /* ZSTD_getLowestPrefixIndex(endIndex) */
    const u32 prefixIdx = (u32)prefixPos + 1;
    const u8 *const prefixStart = base + prefixPos;
    const u8 *const ilimit = iend - 8; /* HASH_READ_SIZE */
    const u8 *ip0 = istart, *ip1, *anchor = istart;
    u32 offset_1 = rep[0], offset_2 = rep[1], offsetSaved = 0;

    ip0 += (ip0 == prefixStart);
    ip1 = ip0 + 1;
    {
        const size_t cur = (size_t)(ip0 - base);
        const u32 maxRep = (u32)(cur > maxDist ? maxDist : cur);
        if (offset_2 > maxRep) offsetSaved = offset_2, offset_2 = 0;
        if (offset_1 > maxRep) offsetSaved = offset_1, offset_1 = 0;
    }
    while (ip1 < ilimit) {
        size_t mLength;
        const u8 *ip2 = ip0 + 2;
        const u32 h0 = zhash(ip0, hlog, mls), h1 = zhash(ip1, hlog, mls);
        const u32 val0 = rd32(ip0), val1 = rd32(ip1);
        const u32 current0 = (u32)(ip0 - base) + 1, current1 = (u32)(ip1 - base) + 1;
        const u32 mi0 = T[h0], mi1 = T[h1];
        const u8 *repMatch = ip2 - offset_1;
        const u8 *match0 = base + mi0 - 1, *match1 = base + mi1 - 1;
        u32 offcode;
        T[h0] = current0;
        T[h1] = current1;
        if ((offset_1 > 0) && rd32(repMatch) == rd32(ip2)) {
            mLength = (ip2[-1] == repMatch[-1]) ? 1 : 0;
            ip0 = ip2 - mLength;
            match0 = repMatch - mLength;
            mLength += 4;
            offcode = 0;
            goto match;
        }
        if (mi0 > prefixIdx && rd32(match0) == val0) goto offset;
        if (mi1 > prefixIdx && rd32(match1) == val1) {
            ip0 = ip1;
            match0 = match1;
            goto offset;
        }
        {
            const size_t step = ((size_t)(ip0 - anchor) >> 7) + stepSize; /* kSearchStrength 8 */
            ip0 += step;
            ip1 += step;
            continue;
        }
    offset:
        offset_2 = offset_1;
        offset_1 = (u32)(ip0 - match0);
        offcode = offset_1 + 2; /* ZSTD_REP_MOVE */
        mLength = 4;
        while (ip0 > anchor && match0 > prefixStart && ip0[-1] == match0[-1]) {
            ip0--;
            match0--;
            mLength++;
        }
    match:
        mLength += zcount(ip0 + mLength, match0 + mLength, iend);
        store_seq(ss, (size_t)(ip0 - anchor), anchor, offcode, mLength - 3);
        ip0 += mLength;
        anchor = ip0;
        if (ip0 <= ilimit) {
            T[zhash(base + current0 - 1 + 2, hlog, mls)] = current0 + 2;
            T[zhash(ip0 - 2, hlog, mls)] = (u32)(ip0 - 2 - base) + 1;
            if (offset_2 > 0) {
                while (ip0 <= ilimit && rd32(ip0) == rd32(ip0 - offset_2)) {
                    const size_t rLength = zcount(ip0 + 4, ip0 + 4 - offset_2, iend) + 4;
                    const u32 t = offset_2;
                    offset_2 = offset_1;
                    offset_1 = t;
                    T[zhash(ip0, hlog, mls)] = (u32)(ip0 - base) + 1;
                    ip0 += rLength;
                    store_seq(ss, 0, anchor, 0, rLength - 3);
                    anchor = ip0;
                }
            }
        }
        ip1 = ip0 + 1;
    }
    rep[0] = offset_1 ? offset_1 : offsetSaved;
    rep[1] = offset_2 ? offset_2 : offsetSaved;
    return (size_t)(iend - anchor);
}

/* ---------------------------------------------------------------- bit writer */
typedef struct {
    u8 *start, *ptr, *end;
    u64 bc;
    unsigned bp;
} bitw;

static void bw_init(bitw *b, u8 *dst, size_t cap) {
    b->start = b->ptr = dst;
    b->end = dst + cap;
    b->bc = 0;
    b->bp = 0;
}
static void bw_add(bitw *b, u64 v, unsigned nb) {
    if (nb == 0) return;
    b->bc |= (v & ((nb >= 64) ? ~0ull : ((1ull << nb) - 1))) << b->bp;
    b->bp += nb;
}
static void bw_flush(bitw *b) {
    while (b->bp >= 8) {
        if (b->ptr < b->end) *b->ptr = (u8)b->bc;
        b->ptr++;
        b->bc >>= 8;
        b->bp -= 8;
    }
}
/* BIT_closeCStream: end mark, last partial byte; 0 when it did not fit */
static size_t bw_close(bitw *b) {
    bw_add(b, 1, 1);
    bw_flush(b);
    if (b->bp > 0) {
        if (b->ptr < b->end) *b->ptr = (u8)b->bc;
        b->ptr++;
    }
    if (b->ptr > b->end) return 0;
    return (size_t)(b->ptr - b->start);
}

/* ---------------------------------------------------------------- FSE */
#define FSE_MIN_TLOG 5
#define FSE_MAX_TLOG 12

static unsigned fse_min_tlog(size_t src, unsigned maxsv) {
    const unsigned a = hb32((u32)src) + 1, b = hb32(maxsv) + 2;
    return a < b ? a : b;
}
static unsigned fse_opt_tlog_internal(unsigned maxtl, size_t src, unsigned maxsv, unsigned minus) {
    const unsigned maxBitsSrc = hb32((u32)(src - 1)) - minus;
    unsigned tl = maxtl;
    const unsigned minBits = fse_min_tlog(src, maxsv);
    if (tl == 0) tl = 11;
    if (maxBitsSrc < tl) tl = maxBitsSrc;
    if (minBits > tl) tl = minBits;
    if (tl < FSE_MIN_TLOG) tl = FSE_MIN_TLOG;
    if (tl > FSE_MAX_TLOG) tl = FSE_MAX_TLOG;
    return tl;
}
static unsigned fse_opt_tlog(unsigned maxtl, size_t src, unsigned maxsv) { return fse_opt_tlog_internal(maxtl, src, maxsv, 2); }

static int fse_norm_m2(short *norm, unsigned tlog, const unsigned *count, size_t total, unsigned maxsv, short lowProb) {
    const short NYA = -2;
    unsigned s, distributed = 0, toDist;
    const u32 lowThreshold = (u32)(total >> tlog);
    u32 lowOne = (u32)((total * 3) >> (tlog + 1));
    for (s = 0; s <= maxsv; s++) {
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) { norm[s] = lowProb; distributed++; total -= count[s]; continue; }
        if (count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
        norm[s] = NYA;
    }
    toDist = (1u << tlog) - distributed;
    if (toDist == 0) return 0;
    if ((total / toDist) > lowOne) {
        lowOne = (u32)((total * 3) / (toDist * 2));
        for (s = 0; s <= maxsv; s++) {
            if (norm[s] == NYA && count[s] <= lowOne) { norm[s] = 1; distributed++; total -= count[s]; continue; }
        }
        toDist = (1u << tlog) - distributed;
    }
    if (distributed == maxsv + 1) {
        unsigned maxV = 0, maxC = 0;
        for (s = 0; s <= maxsv; s++)
            if (count[s] > maxC) { maxV = s; maxC = count[s]; }
        norm[maxV] += (short)toDist;
        return 0;
    }
    if (total == 0) {
        for (s = 0; toDist > 0; s = (s + 1) % (maxsv + 1))
            if (norm[s] > 0) { toDist--; norm[s]++; }
        return 0;
    }
    {
        const u64 vStepLog = 62 - tlog;
        const u64 mid = (1ull << (vStepLog - 1)) - 1;
        const u64 rStep = ((((u64)1 << vStepLog) * toDist) + mid) / (u32)total;
        u64 tmpTotal = mid;
        for (s = 0; s <= maxsv; s++) {
            if (norm[s] == NYA) {
                const u64 end = tmpTotal + (count[s] * rStep);
                const u32 sStart = (u32)(tmpTotal >> vStepLog), sEnd = (u32)(end >> vStepLog);
                const u32 weight = sEnd - sStart;
                if (weight < 1) return -1;
                norm[s] = (short)weight;
                tmpTotal = end;
            }
        }
    }
    return 0;
}

/* FSE_normalizeCount (1.4.9, with useLowProbCount) */
static int fse_normalize(short *norm, unsigned tlog, const unsigned *count, size_t total, unsigned maxsv, int lowprob) {
    static const u32 rtb[] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    const short lowProbCount = lowprob ? -1 : 1;
    const u64 scale = 62 - tlog;
    const u64 step = ((u64)1 << 62) / (u32)total;
    const u64 vStep = 1ull << (scale - 20);
    int still = 1 << tlog;
    unsigned s, largest = 0;
    short largestP = 0;
    const u32 lowThreshold = (u32)(total >> tlog);
    if (tlog < fse_min_tlog(total, maxsv)) return -1;
    for (s = 0; s <= maxsv; s++) {
        if (count[s] == total) return 0; /* rle */
        if (count[s] == 0) { norm[s] = 0; continue; }
        if (count[s] <= lowThreshold) {
            norm[s] = lowProbCount;
            still--;
        } else {
            short proba = (short)((count[s] * step) >> scale);
            if (proba < 8) {
                const u64 restToBeat = vStep * rtb[proba];
                proba += (count[s] * step) - ((u64)proba << scale) > restToBeat;
            }
            if (proba > largestP) { largestP = proba; largest = s; }
            norm[s] = proba;
            still -= proba;
        }
    }
    if (-still >= (norm[largest] >> 1)) {
        if (fse_norm_m2(norm, tlog, count, total, maxsv, lowProbCount) < 0) return -1;
    } else {
        norm[largest] += (short)still;
    }
    return (int)tlog;
}

/* FSE_writeNCount */
static size_t fse_write_ncount(u8 *out0, const short *norm, unsigned maxsv, unsigned tlog) {
    u8 *out = out0;
    const int tsize = 1 << tlog;
    int nbBits = (int)tlog + 1, remaining = tsize + 1, threshold = tsize;
    u32 bs = 0;
    int bc = 0;
    unsigned sym = 0;
    const unsigned alpha = maxsv + 1;
    int prev0 = 0;
    bs += (tlog - FSE_MIN_TLOG) << bc;
    bc += 4;
    while (sym < alpha && remaining > 1) {
        if (prev0) {
            unsigned start = sym;
            while (sym < alpha && !norm[sym]) sym++;
            if (sym == alpha) break;
            while (sym >= start + 24) {
                start += 24;
                bs += 0xFFFFu << bc;
                out[0] = (u8)bs;
                out[1] = (u8)(bs >> 8);
                out += 2;
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
                out[0] = (u8)bs;
                out[1] = (u8)(bs >> 8);
                out += 2;
                bs >>= 16;
                bc -= 16;
            }
        }
        {
            int count = norm[sym++];
            const int max = (2 * threshold - 1) - remaining;
            remaining -= count < 0 ? -count : count;
            count++;
            if (count >= threshold) count += max;
            bs += (u32)count << bc;
            bc += nbBits;
            bc -= (count < max);
            prev0 = (count == 1);
            while (remaining < threshold) { nbBits--; threshold >>= 1; }
        }
        if (bc > 16) {
            out[0] = (u8)bs;
            out[1] = (u8)(bs >> 8);
            out += 2;
            bs >>= 16;
            bc -= 16;
        }
    }
    out[0] = (u8)bs;
    out[1] = (u8)(bs >> 8);
    out += (bc + 7) / 8;
    return (size_t)(out - out0);
}

typedef struct {
    unsigned tlog;
    u16 st[1 << FSE_MAX_TLOG];
    int32_t dnb[256];
    int32_t dfs[256];
} fse_ctab;

/* FSE_buildCTable_wksp */
static void fse_build(fse_ctab *ct, const short *norm, unsigned maxsv, unsigned tlog) {
    const u32 size = 1u << tlog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    u32 cumul[257];
    u8 tsym[1 << FSE_MAX_TLOG];
    u32 high = size - 1, u, s;
    ct->tlog = tlog;
    cumul[0] = 0;
    for (u = 1; u <= maxsv + 1; u++) {
        if (norm[u - 1] == -1) {
            cumul[u] = cumul[u - 1] + 1;
            tsym[high--] = (u8)(u - 1);
        } else {
            cumul[u] = cumul[u - 1] + (u32)norm[u - 1];
        }
    }
    {
        u32 pos = 0;
        for (s = 0; s <= maxsv; s++) {
            int k;
            for (k = 0; k < norm[s]; k++) {
                tsym[pos] = (u8)s;
                pos = (pos + step) & mask;
                while (pos > high) pos = (pos + step) & mask;
            }
        }
    }
    for (u = 0; u < size; u++) ct->st[cumul[tsym[u]]++] = (u16)(size + u);
    {
        u32 total = 0;
        for (s = 0; s <= maxsv; s++) {
            switch (norm[s]) {
            case 0: ct->dnb[s] = (int32_t)(((tlog + 1) << 16) - (1u << tlog)); ct->dfs[s] = 0; break;
            case -1:
            case 1:
                ct->dnb[s] = (int32_t)((tlog << 16) - (1u << tlog));
                ct->dfs[s] = (int32_t)total - 1;
                total++;
                break;
            default: {
                const u32 mbo = tlog - hb32((u32)norm[s] - 1);
                const u32 msp = (u32)norm[s] << mbo;
                ct->dnb[s] = (int32_t)((mbo << 16) - msp);
                ct->dfs[s] = (int32_t)total - norm[s];
                total += (u32)norm[s];
            }
            }
        }
    }
}
static void fse_build_rle(fse_ctab *ct, unsigned sym) {
    ct->tlog = 0;
    ct->st[0] = 0;
    ct->st[1] = 0;
    ct->dnb[sym] = 0;
    ct->dfs[sym] = 0;
}

typedef struct {
    u32 value;
    const fse_ctab *ct;
} fse_state;

static void fse_init2(fse_state *s, const fse_ctab *ct, unsigned sym) {
    const u32 nbo = (u32)((ct->dnb[sym] + (1 << 15)) >> 16);
    u32 v = (nbo << 16) - (u32)ct->dnb[sym];
    s->ct = ct;
    s->value = ct->st[(v >> nbo) + (u32)ct->dfs[sym]];
}
static void fse_enc(bitw *b, fse_state *s, unsigned sym) {
    const u32 nbo = (u32)(((int32_t)s->value + s->ct->dnb[sym]) >> 16);
    bw_add(b, s->value, nbo);
    s->value = s->ct->st[(s->value >> nbo) + (u32)s->ct->dfs[sym]];
}
static void fse_flush_state(bitw *b, const fse_state *s) {
    bw_add(b, s->value, s->ct->tlog);
    bw_flush(b);
}

/* FSE_compress_usingCTable (HUF weights) */
static size_t fse_compress_ct(u8 *dst, size_t cap, const u8 *src, size_t n, const fse_ctab *ct) {
    const u8 *ip = src + n;
    bitw b;
    fse_state s1, s2;
    if (n <= 2) return 0;
    bw_init(&b, dst, cap);
    if (n & 1) {
        fse_init2(&s1, ct, *--ip);
        fse_init2(&s2, ct, *--ip);
        fse_enc(&b, &s1, *--ip);
        bw_flush(&b);
    } else {
        fse_init2(&s2, ct, *--ip);
        fse_init2(&s1, ct, *--ip);
    }
    n -= 2;
    if (n & 2) {
        fse_enc(&b, &s2, *--ip);
        fse_enc(&b, &s1, *--ip);
        bw_flush(&b);
    }
    while (ip > src) {
        fse_enc(&b, &s2, *--ip);
        fse_enc(&b, &s1, *--ip);
        fse_enc(&b, &s2, *--ip);
        fse_enc(&b, &s1, *--ip);
        bw_flush(&b);
    }
    fse_flush_state(&b, &s2);
    fse_flush_state(&b, &s1);
    return bw_close(&b);
}

/* ---------------------------------------------------------------- Huffman */
#define HUF_TLOG_MAX 12
#define HUF_TLOG_DEFAULT 11

typedef struct {
    u8 nb[256];
    u16 val[256];
    int valid; /* a table is held */
} huf_ctab;

typedef struct {
    u32 count;
    u16 parent;
    u8 byte;
    u8 nbBits;
} hnode;

static u32 huf_set_max_height(hnode *huffNode, u32 lastNonNull, u32 maxNbBits) {
    const u32 largestBits = huffNode[lastNonNull].nbBits;
    if (largestBits <= maxNbBits) return largestBits;
    {
        int totalCost = 0;
        const u32 baseCost = 1u << (largestBits - maxNbBits);
        int n = (int)lastNonNull;
        while (huffNode[n].nbBits > maxNbBits) {
            totalCost += (int)(baseCost - (1u << (largestBits - huffNode[n].nbBits)));
            huffNode[n].nbBits = (u8)maxNbBits;
            n--;
        }
        while (huffNode[n].nbBits == maxNbBits) n--;
        totalCost >>= (largestBits - maxNbBits);
        {
            const u32 noSymbol = 0xF0F0F0F0;
            u32 rankLast[HUF_TLOG_MAX + 2];
            memset(rankLast, 0xF0, sizeof(rankLast));
            {
                u32 currentNbBits = maxNbBits;
                int pos;
                for (pos = n; pos >= 0; pos--) {
                    if (huffNode[pos].nbBits >= currentNbBits) continue;
                    currentNbBits = huffNode[pos].nbBits;
                    rankLast[maxNbBits - currentNbBits] = (u32)pos;
                }
            }
            while (totalCost > 0) {
                u32 nBitsToDecrease = hb32((u32)totalCost) + 1;
                for (; nBitsToDecrease > 1; nBitsToDecrease--) {
                    const u32 highPos = rankLast[nBitsToDecrease], lowPos = rankLast[nBitsToDecrease - 1];
                    if (highPos == noSymbol) continue;
                    if (lowPos == noSymbol) break;
                    {
                        const u32 highTotal = huffNode[highPos].count, lowTotal = 2 * huffNode[lowPos].count;
                        if (highTotal <= lowTotal) break;
                    }
                }
                while (nBitsToDecrease <= HUF_TLOG_MAX && rankLast[nBitsToDecrease] == noSymbol) nBitsToDecrease++;
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
            while (totalCost < 0) {
                if (rankLast[1] == noSymbol) {
                    while (huffNode[n].nbBits == maxNbBits) n--;
                    huffNode[n + 1].nbBits--;
                    rankLast[1] = (u32)(n + 1);
                    totalCost++;
                    continue;
                }
                huffNode[rankLast[1] + 1].nbBits--;
                rankLast[1]++;
                totalCost++;
            }
        }
    }
    return maxNbBits;
}

/* HUF_buildCTable_wksp: returns the maximum code length */
static unsigned huf_build(huf_ctab *t, const unsigned *count, unsigned maxsv, unsigned maxNbBits) {
    hnode node0[2 * 256 + 2];
    hnode *const huffNode = node0 + 1;
    const int STARTNODE = 256;
    int nonNullRank, lowS, lowN, nodeNb = STARTNODE, n, nodeRoot;
    unsigned i;
    memset(node0, 0, sizeof(node0));
    /* HUF_sort: decreasing count, ties in symbol order (stable) */
    {
        int m = 0;
        for (i = 0; i <= maxsv; i++) {
            const u32 c = count[i];
            int pos = m++;
            while (pos > 0 && c > huffNode[pos - 1].count) {
                huffNode[pos] = huffNode[pos - 1];
                pos--;
            }
            huffNode[pos].count = c;
            huffNode[pos].byte = (u8)i;
            huffNode[pos].parent = 0;
            huffNode[pos].nbBits = 0;
        }
    }
    nonNullRank = (int)maxsv;
    while (huffNode[nonNullRank].count == 0) nonNullRank--;
    lowS = nonNullRank;
    nodeRoot = nodeNb + lowS - 1;
    lowN = nodeNb;
    huffNode[nodeNb].count = huffNode[lowS].count + huffNode[lowS - 1].count;
    huffNode[lowS].parent = huffNode[lowS - 1].parent = (u16)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (n = nodeNb; n <= nodeRoot; n++) huffNode[n].count = 1u << 30;
    node0[0].count = 1u << 31;
    while (nodeNb <= nodeRoot) {
        const int n1 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        const int n2 = (huffNode[lowS].count < huffNode[lowN].count) ? lowS-- : lowN++;
        huffNode[nodeNb].count = huffNode[n1].count + huffNode[n2].count;
        huffNode[n1].parent = huffNode[n2].parent = (u16)nodeNb;
        nodeNb++;
    }
    huffNode[nodeRoot].nbBits = 0;
    for (n = nodeRoot - 1; n >= STARTNODE; n--) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    for (n = 0; n <= nonNullRank; n++) huffNode[n].nbBits = huffNode[huffNode[n].parent].nbBits + 1;
    maxNbBits = huf_set_max_height(huffNode, (u32)nonNullRank, maxNbBits);
    {
        u16 nbPerRank[HUF_TLOG_MAX + 1], valPerRank[HUF_TLOG_MAX + 1];
        memset(nbPerRank, 0, sizeof(nbPerRank));
        memset(valPerRank, 0, sizeof(valPerRank));
        for (n = 0; n <= nonNullRank; n++) nbPerRank[huffNode[n].nbBits]++;
        {
            u16 min = 0;
            for (n = (int)maxNbBits; n > 0; n--) {
                valPerRank[n] = min;
                min += nbPerRank[n];
                min >>= 1;
            }
        }
        memset(t->nb, 0, sizeof(t->nb));
        memset(t->val, 0, sizeof(t->val));
        for (n = 0; n <= (int)maxsv; n++) t->nb[huffNode[n].byte] = huffNode[n].nbBits;
        for (n = 0; n <= (int)maxsv; n++) t->val[n] = valPerRank[t->nb[n]]++;
    }
    t->valid = 1;
    return maxNbBits;
}

/* HUF_compressWeights */
static size_t huf_compress_weights(u8 *dst, size_t cap, const u8 *w, size_t wtSize) {
    unsigned maxsv = HUF_TLOG_MAX, tlog = 6, count[HUF_TLOG_MAX + 1];
    short norm[HUF_TLOG_MAX + 1];
    fse_ctab ct;
    size_t hs, cs;
    unsigned s, maxc = 0;
    if (wtSize <= 1) return 0;
    memset(count, 0, sizeof(count));
    for (s = 0; s < wtSize; s++) count[w[s]]++;
    while (!count[maxsv]) maxsv--;
    for (s = 0; s <= maxsv; s++) maxc = count[s] > maxc ? count[s] : maxc;
    if (maxc == wtSize) return 1;
    if (maxc == 1) return 0;
    tlog = fse_opt_tlog(tlog, wtSize, maxsv);
    if (fse_normalize(norm, tlog, count, wtSize, maxsv, 0) < 0) return 0;
    hs = fse_write_ncount(dst, norm, maxsv, tlog);
    fse_build(&ct, norm, maxsv, tlog);
    cs = fse_compress_ct(dst + hs, cap - hs, w, wtSize, &ct);
    if (cs == 0) return 0;
    return hs + cs;
}

/* HUF_writeCTable: 0 on error (raw weights impossible) */
static size_t huf_write_ctable(u8 *op, size_t cap, const huf_ctab *t, unsigned maxsv, unsigned huffLog) {
    u8 b2w[HUF_TLOG_MAX + 1], hw[256];
    unsigned n;
    b2w[0] = 0;
    for (n = 1; n < huffLog + 1; n++) b2w[n] = (u8)(huffLog + 1 - n);
    for (n = 0; n < maxsv; n++) hw[n] = b2w[t->nb[n]];
    {
        const size_t hs = huf_compress_weights(op + 1, cap - 1, hw, maxsv);
        if (hs > 1 && hs < maxsv / 2) {
            op[0] = (u8)hs;
            return hs + 1;
        }
    }
    if (maxsv > 128) return 0;
    op[0] = (u8)(128 + (maxsv - 1));
    hw[maxsv] = 0;
    for (n = 0; n < maxsv; n += 2) op[n / 2 + 1] = (u8)((hw[n] << 4) + hw[n + 1]);
    return (maxsv + 1) / 2 + 1;
}

static size_t huf_1x(u8 *dst, size_t cap, const u8 *src, size_t n, const huf_ctab *t) {
    bitw b;
    size_t i;
    if (cap < 8) return 0;
    bw_init(&b, dst, cap);
    for (i = n; i > 0; i--) { /* last symbol first */
        bw_add(&b, t->val[src[i - 1]], t->nb[src[i - 1]]);
        bw_flush(&b);
    }
    return bw_close(&b);
}
static size_t huf_4x(u8 *dst, size_t cap, const u8 *src, size_t n, const huf_ctab *t) {
    const size_t seg = (n + 3) / 4;
    u8 *op = dst + 6;
    const u8 *ip = src;
    int k;
    if (cap < 6 + 1 + 1 + 1 + 8) return 0;
    if (n < 12) return 0;
    for (k = 0; k < 3; k++) {
        const size_t c = huf_1x(op, (size_t)(dst + cap - op), ip, seg, t);
        if (c == 0) return 0;
        dst[2 * k] = (u8)c;
        dst[2 * k + 1] = (u8)(c >> 8);
        op += c;
        ip += seg;
    }
    {
        const size_t c = huf_1x(op, (size_t)(dst + cap - op), ip, (size_t)(src + n - ip), t);
        if (c == 0) return 0;
        op += c;
    }
    return (size_t)(op - dst);
}
/* HUF_compressCTable_internal */
static size_t huf_ct_internal(u8 *ostart, u8 *op, u8 *oend, const u8 *src, size_t n, int single, const huf_ctab *t) {
    const size_t c = single ? huf_1x(op, (size_t)(oend - op), src, n, t) : huf_4x(op, (size_t)(oend - op), src, n, t);
    if (c == 0) return 0;
    op += c;
    if ((size_t)(op - ostart) >= n - 1) return 0;
    return (size_t)(op - ostart);
}

typedef enum { HUF_none = 0, HUF_check = 1, HUF_valid = 2 } huf_repeat;

typedef struct {
    huf_ctab t;
    huf_repeat repeat;
} huf_state;

static size_t huf_estimate(const huf_ctab *t, const unsigned *count, unsigned maxsv) {
    size_t nb = 0;
    unsigned s;
    for (s = 0; s <= maxsv; s++) nb += (size_t)t->nb[s] * count[s];
    return nb >> 3;
}

/* HUF_compress_internal; table = the next block's state (starts as a copy of prev) */
static size_t huf_compress(u8 *dst, size_t cap, const u8 *src, size_t n, int single, huf_ctab *oldTable,
                           huf_repeat *repeat, int preferRepeat) {
    unsigned count[256], maxsv = 255, s;
    size_t largest = 0;
    u8 *const ostart = dst, *const oend = dst + cap;
    u8 *op = ostart;
    huf_ctab nt;
    unsigned huffLog;
    if (!n || !cap) return 0;
    if (preferRepeat && *repeat == HUF_valid) return huf_ct_internal(ostart, op, oend, src, n, single, oldTable);
    memset(count, 0, sizeof(count));
    for (s = 0; s < n; s++) count[src[s]]++;
    while (!count[maxsv]) maxsv--;
    for (s = 0; s <= maxsv; s++) largest = count[s] > largest ? count[s] : largest;
    if (largest == n) { *ostart = src[0]; return 1; }
    if (largest <= (n >> 7) + 4) return 0;
    if (*repeat == HUF_check) {
        int bad = 0;
        for (s = 0; s <= maxsv; s++) bad |= (count[s] != 0) & (oldTable->nb[s] == 0);
        if (bad) *repeat = HUF_none;
    }
    if (preferRepeat && *repeat != HUF_none) return huf_ct_internal(ostart, op, oend, src, n, single, oldTable);
    huffLog = fse_opt_tlog_internal(HUF_TLOG_DEFAULT, n, maxsv, 1);
    huffLog = huf_build(&nt, count, maxsv, huffLog);
    {
        const size_t hs = huf_write_ctable(op, cap, &nt, maxsv, huffLog);
        if (hs == 0) return 0; /* (raw weights impossible: libzstd errors out and the block stores raw literals) */
        if (*repeat != HUF_none) {
            const size_t oldSize = huf_estimate(oldTable, count, maxsv), newSize = huf_estimate(&nt, count, maxsv);
            if (oldSize <= hs + newSize || hs + 12 >= n) return huf_ct_internal(ostart, op, oend, src, n, single, oldTable);
        }
        if (hs + 12 >= n) return 0;
        op += hs;
        *repeat = HUF_none;
        *oldTable = nt;
    }
    return huf_ct_internal(ostart, op, oend, src, n, single, oldTable);
}

static size_t no_compress_literals(u8 *dst, const u8 *src, size_t n) {
    const unsigned fl = 1 + (n > 31) + (n > 4095);
    switch (fl) {
    case 1: dst[0] = (u8)(0 + (n << 3)); break;
    case 2: { const u32 v = 0 + (1u << 2) + ((u32)n << 4); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); break; }
    default: { const u32 v = 0 + (3u << 2) + ((u32)n << 4); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); }
    }
    memcpy(dst + fl, src, n);
    return n + fl;
}
static size_t rle_literals(u8 *dst, const u8 *src, size_t n) {
    const unsigned fl = 1 + (n > 31) + (n > 4095);
    switch (fl) {
    case 1: dst[0] = (u8)(1 + (n << 3)); break;
    case 2: { const u32 v = 1 + (1u << 2) + ((u32)n << 4); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); break; }
    default: { const u32 v = 1 + (3u << 2) + ((u32)n << 4); dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); }
    }
    dst[fl] = src[0];
    return fl + 1;
}

/* ZSTD_compressLiterals (strategy fast, literal compression enabled) */
static size_t compress_literals(const huf_state *prev, huf_state *next, u8 *dst, size_t cap, const u8 *src, size_t n) {
    const size_t minGain = (n >> 6) + 2;
    const size_t lhSize = 3 + (n >= 1024) + (n >= 16384);
    int single = n < 256;
    int compressed_type = 1; /* set_compressed (2) vs set_repeat (3) */
    size_t cLit;
    *next = *prev;
    {
        const size_t minLit = prev->repeat == HUF_valid ? 6 : 63;
        if (n <= minLit) return no_compress_literals(dst, src, n);
    }
    {
        huf_repeat repeat = prev->repeat;
        const int preferRepeat = n <= 1024;
        if (repeat == HUF_valid && lhSize == 3) single = 1;
        cLit = huf_compress(dst + lhSize, cap - lhSize, src, n, single, &next->t, &repeat, preferRepeat);
        if (repeat != HUF_none) compressed_type = 0;
    }
    if (cLit == 0 || cLit >= n - minGain) {
        *next = *prev;
        return no_compress_literals(dst, src, n);
    }
    if (cLit == 1) {
        *next = *prev;
        return rle_literals(dst, src, n);
    }
    if (compressed_type) next->repeat = HUF_check;
    {
        const u32 hType = compressed_type ? 2 : 3;
        switch (lhSize) {
        case 3: {
            const u32 v = hType + ((u32)(!single) << 2) + ((u32)n << 4) + ((u32)cLit << 14);
            dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16);
            break;
        }
        case 4: {
            const u32 v = hType + (2u << 2) + ((u32)n << 4) + ((u32)cLit << 18);
            dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); dst[3] = (u8)(v >> 24);
            break;
        }
        default: {
            const u32 v = hType + (3u << 2) + ((u32)n << 4) + ((u32)cLit << 22);
            dst[0] = (u8)v; dst[1] = (u8)(v >> 8); dst[2] = (u8)(v >> 16); dst[3] = (u8)(v >> 24);
            dst[4] = (u8)(cLit >> 10);
        }
        }
    }
    return lhSize + cLit;
}

/* ---------------------------------------------------------------- sequences section */
static const u8 LL_Code[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                               16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21,
                               22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                               24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
static const u8 LL_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                               1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const u8 ML_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                               0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                               2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const short LL_defaultNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                         2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const short ML_defaultNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const short OF_defaultNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                         1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

static unsigned ll_code(u32 ll) { return ll > 63 ? hb32(ll) + 19 : LL_Code[ll]; }
static unsigned ml_code(u32 mlb) {
    static u8 ML_Code[128];
    static int init = 0;
    if (!init) {
        /* RFC 8878 match-length codes 0..42 cover Match_Length - 3 = 0..127 */
        static const u32 base[43] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                     16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                     32, 34, 36, 38, 40, 44, 48, 56, 64, 80, 96};
        unsigned c = 0, v;
        for (v = 0; v < 128; v++) {
            while (c + 1 < 43 && base[c + 1] <= v) c++;
            ML_Code[v] = (u8)c;
        }
        init = 1;
    }
    return mlb > 127 ? hb32(mlb) + 36 : ML_Code[mlb];
}

enum { set_basic = 0, set_rle = 1, set_compressed = 2, set_repeat = 3 };

/* ZSTD_selectEncodingType for strategy fast (no repeat: tables never become valid without a dictionary) */
static int select_type(const unsigned *count, unsigned max, size_t mostFrequent, size_t nbSeq, unsigned defaultNormLog,
                       int defaultAllowed) {
    (void)count;
    (void)max;
    if (mostFrequent == nbSeq) {
        if (defaultAllowed && nbSeq <= 2) return set_basic;
        return set_rle;
    }
    if (defaultAllowed) {
        const size_t mult = 10 - 1; /* strategy fast = 1 */
        const size_t dynMin = (((size_t)1 << defaultNormLog) * mult) >> 3;
        if (nbSeq < dynMin || mostFrequent < (nbSeq >> (defaultNormLog - 1))) return set_basic;
    }
    return set_compressed;
}

/* ZSTD_buildCTable; returns the table-description bytes written */
static size_t build_ctable(u8 *op, fse_ctab *ct, unsigned FSELog, int type, unsigned *count, unsigned max,
                           const u8 *codes, size_t nbSeq, const short *defNorm, unsigned defLog, unsigned defMax) {
    switch (type) {
    case set_rle: fse_build_rle(ct, max); *op = codes[0]; return 1;
    case set_basic: fse_build(ct, defNorm, defMax, defLog); return 0;
    default: {
        short norm[64];
        size_t nbSeq_1 = nbSeq;
        const unsigned tlog = fse_opt_tlog(FSELog, nbSeq, max);
        if (count[codes[nbSeq - 1]] > 1) {
            count[codes[nbSeq - 1]]--;
            nbSeq_1--;
        }
        fse_normalize(norm, tlog, count, nbSeq_1, max, nbSeq_1 >= 2048);
        {
            const size_t hs = fse_write_ncount(op, norm, max, tlog);
            fse_build(ct, norm, max, tlog);
            return hs;
        }
    }
    }
}

/* ZSTD_entropyCompressSequences (+ _internal): 0 = store the block raw */
static size_t entropy_compress(const zseqstore *ss, const huf_state *prevHuf, huf_state *nextHuf, u8 *dst, size_t cap,
                               size_t srcSize) {
    u8 *const ostart = dst;
    u8 *op = dst;
    const size_t nbSeq = ss->ns;
    u8 *llc = NULL, *ofc = NULL, *mlc = NULL, *seqHead, *lastNCount = NULL;
    unsigned count[64];
    static fse_ctab ctLL, ctOF, ctML;
    int LLtype, OFtype, MLtype;
    size_t i;
    op += compress_literals(prevHuf, nextHuf, op, cap, ss->lit, ss->nl);
    if (nbSeq < 128) {
        *op++ = (u8)nbSeq;
    } else if (nbSeq < 0x7F00) {
        op[0] = (u8)((nbSeq >> 8) + 0x80);
        op[1] = (u8)nbSeq;
        op += 2;
    } else {
        op[0] = 0xFF;
        op[1] = (u8)(nbSeq - 0x7F00);
        op[2] = (u8)((nbSeq - 0x7F00) >> 8);
        op += 3;
    }
    if (nbSeq == 0) goto done;
    seqHead = op++;
    llc = (u8 *)malloc(nbSeq);
    ofc = (u8 *)malloc(nbSeq);
    mlc = (u8 *)malloc(nbSeq);
    for (i = 0; i < nbSeq; i++) {
        llc[i] = (u8)ll_code(ss->seq[i].ll);
        mlc[i] = (u8)ml_code(ss->seq[i].mlb);
        ofc[i] = (u8)hb32(ss->seq[i].ofv);
    }
    /* LL */
    {
        unsigned max = 35;
        size_t mf = 0;
        memset(count, 0, sizeof(count));
        for (i = 0; i < nbSeq; i++) count[llc[i]]++;
        while (!count[max]) max--;
        for (i = 0; i <= max; i++) mf = count[i] > mf ? count[i] : mf;
        LLtype = select_type(count, max, mf, nbSeq, 6, 1);
        {
            const size_t hs = build_ctable(op, &ctLL, 9, LLtype, count, max, llc, nbSeq, LL_defaultNorm, 6, 35);
            if (LLtype == set_compressed) lastNCount = op;
            op += hs;
        }
    }
    /* OF */
    {
        unsigned max = 31;
        size_t mf = 0;
        memset(count, 0, sizeof(count));
        for (i = 0; i < nbSeq; i++) count[ofc[i]]++;
        while (!count[max]) max--;
        for (i = 0; i <= max; i++) mf = count[i] > mf ? count[i] : mf;
        OFtype = select_type(count, max, mf, nbSeq, 5, max <= 28);
        {
            const size_t hs = build_ctable(op, &ctOF, 8, OFtype, count, max, ofc, nbSeq, OF_defaultNorm, 5, 28);
            if (OFtype == set_compressed) lastNCount = op;
            op += hs;
        }
    }
    /* ML */
    {
        unsigned max = 52;
        size_t mf = 0;
        memset(count, 0, sizeof(count));
        for (i = 0; i < nbSeq; i++) count[mlc[i]]++;
        while (!count[max]) max--;
        for (i = 0; i <= max; i++) mf = count[i] > mf ? count[i] : mf;
        MLtype = select_type(count, max, mf, nbSeq, 6, 1);
        {
            const size_t hs = build_ctable(op, &ctML, 9, MLtype, count, max, mlc, nbSeq, ML_defaultNorm, 6, 52);
            if (MLtype == set_compressed) lastNCount = op;
            op += hs;
        }
    }
    *seqHead = (u8)((LLtype << 6) + (OFtype << 4) + (MLtype << 2));
    /* ZSTD_encodeSequences */
    {
        bitw b;
        fse_state sML, sOF, sLL;
        size_t n, bsz;
        bw_init(&b, op, (size_t)(ostart + cap - op));
        fse_init2(&sML, &ctML, mlc[nbSeq - 1]);
        fse_init2(&sOF, &ctOF, ofc[nbSeq - 1]);
        fse_init2(&sLL, &ctLL, llc[nbSeq - 1]);
        bw_add(&b, ss->seq[nbSeq - 1].ll, LL_bits[llc[nbSeq - 1]]);
        bw_add(&b, ss->seq[nbSeq - 1].mlb, ML_bits[mlc[nbSeq - 1]]);
        bw_add(&b, ss->seq[nbSeq - 1].ofv, ofc[nbSeq - 1]);
        bw_flush(&b);
        for (n = nbSeq - 1; n-- > 0;) {
            const unsigned llC = llc[n], ofC = ofc[n], mlC = mlc[n];
            fse_enc(&b, &sOF, ofC);
            fse_enc(&b, &sML, mlC);
            fse_enc(&b, &sLL, llC);
            bw_flush(&b);
            bw_add(&b, ss->seq[n].ll, LL_bits[llC]);
            bw_add(&b, ss->seq[n].mlb, ML_bits[mlC]);
            bw_flush(&b);
            bw_add(&b, ss->seq[n].ofv, ofC);
            bw_flush(&b);
        }
        fse_flush_state(&b, &sML);
        fse_flush_state(&b, &sOF);
        fse_flush_state(&b, &sLL);
        bsz = bw_close(&b);
        op += bsz;
        if (lastNCount && (op - lastNCount) < 4) {
            free(llc); free(ofc); free(mlc);
            return 0;
        }
    }
    free(llc);
    free(ofc);
    free(mlc);
done:
    {
        const size_t cSize = (size_t)(op - ostart);
        const size_t maxCSize = srcSize - ((srcSize >> 6) + 2); /* ZSTD_minGain, strategy fast */
        if (cSize >= maxCSize) return 0;
        return cSize;
    }
}

/* ---------------------------------------------------------------- frame */
static size_t write_frame_header(u8 *op, u64 n, unsigned wlog) {
    const u32 windowSize = 1u << wlog;
    const int single = windowSize >= n;
    const unsigned fcsCode = (n >= 256) + (n >= 65536 + 256) + (n >= 0xFFFFFFFFu);
    size_t pos = 4;
    op[0] = 0x28; op[1] = 0xB5; op[2] = 0x2F; op[3] = 0xFD;
    op[pos++] = (u8)((single << 5) + (fcsCode << 6));
    if (!single) op[pos++] = (u8)((wlog - 10) << 3);
    switch (fcsCode) {
    case 0: if (single) op[pos++] = (u8)n; break;
    case 1: { const u32 v = (u32)(n - 256); op[pos] = (u8)v; op[pos + 1] = (u8)(v >> 8); pos += 2; break; }
    case 2: { const u32 v = (u32)n; memcpy(op + pos, &v, 4); pos += 4; break; }
    default: memcpy(op + pos, &n, 8); pos += 8;
    }
    return pos;
}

static int is_rle(const u8 *p, size_t n) {
    size_t i;
    for (i = 1; i < n; i++)
        if (p[i] != p[0]) return 0;
    return 1;
}

/* ZSTD_compress(dst, cap, src, n, 1); cap must be >= ZSTD_compressBound(n).
 * Optional per-block report (blk_out: 4 int32 per 128 KiB block: kind 0 raw /
 * 1 rle / 2 compressed, size, sequences, literals). */
int64_t oracle_zstd_compress_l1_ex(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int32_t *blk_out) {
    const zl1_params P = zl1_get_params((u64)n);
    const size_t blockSize = (size_t)1 << (P.wlog < 17 ? P.wlog : 17);
    u32 *T = (u32 *)calloc((size_t)1 << P.hlog, sizeof(u32));
    zseqstore ss;
    huf_state prevHuf, nextHuf;
    u32 rep[2] = {1, 4}; /* repStartValue {1, 4, 8} */
    u8 *op = dst;
    size_t bs = 0, k = 0;
    int first = 1;
    (void)cap;
    if (!T) return -1;
    memset(&prevHuf, 0, sizeof(prevHuf));
    prevHuf.repeat = HUF_none;
    ss.seq = (zseq *)malloc(sizeof(zseq) * (blockSize / 3 + 16));
    ss.lit = (u8 *)malloc(blockSize + 64);
    op += write_frame_header(op, (u64)n, P.wlog);
    if (n == 0) {
        op[0] = 1; op[1] = 0; op[2] = 0; /* last empty raw block */
        op += 3;
    }
    while (bs < (size_t)n) {
        const size_t bsz = (size_t)n - bs < blockSize ? (size_t)n - bs : blockSize;
        const int last = bs + bsz == (size_t)n;
        size_t cSize = 0;
        u32 nrep[2] = {rep[0], rep[1]};
        ss.ns = 0;
        ss.nl = 0;
        if (bsz >= 7) { /* MIN_CBLOCK_SIZE + ZSTD_blockHeaderSize + 1 */
            const size_t lastLL = fast_block(T, &P, src, bs, bs + bsz, nrep, &ss);
            memcpy(ss.lit + ss.nl, src + bs + bsz - lastLL, lastLL);
            ss.nl += lastLL;
            cSize = entropy_compress(&ss, &prevHuf, &nextHuf, op + 3, (size_t)(dst + cap - op - 3), bsz);
            if (!first && cSize < 25 && is_rle(src + bs, bsz)) cSize = 1;
        }
        if (cSize > 1) { /* ZSTD_confirmRepcodesAndEntropyTables */
            rep[0] = nrep[0];
            rep[1] = nrep[1];
            prevHuf = nextHuf;
        }
        if (blk_out) {
            blk_out[4 * k + 0] = cSize == 0 ? 0 : cSize == 1 ? 1 : 2;
            blk_out[4 * k + 1] = (int32_t)(cSize == 0 ? bsz : cSize == 1 ? 1 : cSize);
            blk_out[4 * k + 2] = (int32_t)ss.ns;
            blk_out[4 * k + 3] = (int32_t)ss.nl;
        }
        if (cSize == 0) {
            const u32 h = (u32)last + (0u << 1) + (u32)(bsz << 3);
            op[0] = (u8)h; op[1] = (u8)(h >> 8); op[2] = (u8)(h >> 16);
            memcpy(op + 3, src + bs, bsz);
            op += 3 + bsz;
        } else if (cSize == 1) {
            const u32 h = (u32)last + (1u << 1) + (u32)(bsz << 3);
            op[0] = (u8)h; op[1] = (u8)(h >> 8); op[2] = (u8)(h >> 16);
            op[3] = src[bs];
            op += 4;
        } else {
            const u32 h = (u32)last + (2u << 1) + (u32)(cSize << 3);
            op[0] = (u8)h; op[1] = (u8)(h >> 8); op[2] = (u8)(h >> 16);
            op += 3 + cSize;
        }
        first = 0;
        bs += bsz;
        k++;
    }
    free(T);
    free(ss.seq);
    free(ss.lit);
    return (int64_t)(op - dst);
}

int64_t oracle_zstd_compress_l1(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
    return oracle_zstd_compress_l1_ex(src, n, dst, cap, NULL);
}
