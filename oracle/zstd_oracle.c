/*
 * oracle/zstd_oracle.c -- CPU restatement of Zstandard frame decoding
 * (TEST INFRASTRUCTURE ONLY; loaded by tests/, smoke() and bench.py's
 * cpu_baseline leg, never by the product library).
 *
 * Restates ZSTD_decompress as reached from pkg/compress/compress.go:94-103
 * (ZStandard.Decompress -> github.com/DataDog/zstd v1.5.6 zstd.Decompress ->
 * ZSTD_decompress).  The library is third-party and not in /root/reference;
 * this follows the published format (RFC 8878) and libzstd's decoding choices
 * (FSE_readNCount, HUF X1 table layout, 2-state FSE weight decoding,
 * sequence bit order, repeat-offset rules incl. "0 -> 1"), pinned against
 * libzstd 1.4.9 fixtures in tests/golden/zstd_golden.json.
 *
 * Return: decoded size (>= 0), or
 *   ZO_ERR_CORRUPT  (-1)  malformed input (any ZSTD_decompress error other than below)
 *   ZO_ERR_DSTSMALL (-2)  output does not fit in dstCapacity
 *   ZO_ERR_SRCSIZE  (-3)  source size wrong (truncated / trailing bytes)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define ZO_ERR_CORRUPT (-1)
#define ZO_ERR_DSTSMALL (-2)
#define ZO_ERR_SRCSIZE (-3)

/* Symbol_Compression_Modes reserved bits (RFC 8878 3.1.1.3.2.1 "must be
 * all-zeroes"): zstd >= 1.5 (the reference pins 1.5.6) rejects them, 1.4.9
 * (the library the golden corpus was generated with) ignores them.  Default:
 * reject, like the pinned version; tests flip it to pin against 1.4.9. */
static int zo_strict_reserved = 1;
void oracle_zstd_set_strict_reserved(int on) { zo_strict_reserved = on; }

/* ---------------------------------------------------------------- XXH64 */
static const uint64_t P1 = 11400714785074694791ULL, P2 = 14029467366897019727ULL, P3 = 1609587929392839161ULL,
                      P4 = 9650029242287828579ULL, P5 = 2870177450012600261ULL;
static inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t rd64le(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32le(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t xround(uint64_t acc, uint64_t in) { acc += in * P2; acc = rotl(acc, 31); return acc * P1; }
static inline uint64_t xmerge(uint64_t acc, uint64_t v) { v = xround(0, v); acc ^= v; return acc * P1 + P4; }

uint64_t oracle_xxh64(const uint8_t *p, size_t len, uint64_t seed) {
    const uint8_t *end = p + len;
    uint64_t h;
    if (len >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        const uint8_t *lim = end - 32;
        do {
            v1 = xround(v1, rd64le(p)); v2 = xround(v2, rd64le(p + 8));
            v3 = xround(v3, rd64le(p + 16)); v4 = xround(v4, rd64le(p + 24));
            p += 32;
        } while (p <= lim);
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
        h = xmerge(h, v1); h = xmerge(h, v2); h = xmerge(h, v3); h = xmerge(h, v4);
    } else {
        h = seed + P5;
    }
    h += (uint64_t)len;
    while (p + 8 <= end) { h ^= xround(0, rd64le(p)); h = rotl(h, 27) * P1 + P4; p += 8; }
    if (p + 4 <= end) { h ^= (uint64_t)rd32le(p) * P1; h = rotl(h, 23) * P2 + P3; p += 4; }
    while (p < end) { h ^= (*p) * P5; h = rotl(h, 11) * P1; p++; }
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}

/* ------------------------------------------------------- bit readers */
/* forward, LSB-first (FSE table descriptions) */
typedef struct { const uint8_t *p; int64_t nbits, pos; } fbr;
static inline uint32_t fbr_peek(const fbr *b, int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; i++) {
        int64_t q = b->pos + i;
        uint32_t bit = q < b->nbits ? (b->p[q >> 3] >> (q & 7)) & 1u : 0u;
        v |= bit << i;
    }
    return v;
}

/* backward (Huffman / FSE streams): bits are consumed from the highest
 * position downwards, starting below the final padding 1-bit.  Reading past
 * the start yields zeros and counts as overflow (libzstd's BIT_DStream). */
typedef struct { const uint8_t *p; int64_t total, left; } bbr;
static int bbr_init(bbr *b, const uint8_t *p, int64_t n) {
    if (n <= 0) return -1;
    uint8_t last = p[n - 1];
    if (last == 0) return -1;
    int hb = 31 - __builtin_clz(last);
    b->p = p;
    b->total = (n - 1) * 8 + hb;  /* bits below the padding bit */
    b->left = b->total;
    return 0;
}
static inline uint32_t bbr_read(bbr *b, int n) {  /* MSB-first value of the next n bits */
    uint32_t v = 0;
    for (int i = 0; i < n; i++) {
        b->left--;
        uint32_t bit = 0;
        if (b->left >= 0) bit = (b->p[b->left >> 3] >> (b->left & 7)) & 1u;
        v = (v << 1) | bit;
    }
    return v;
}
static inline uint32_t bbr_peek(const bbr *b, int n) { bbr t = *b; return bbr_read(&t, n); }
static inline int bbr_overflow(const bbr *b) { return b->left < 0; }
static inline int bbr_done(const bbr *b) { return b->left == 0; }

/* -------------------------------------------------------------- FSE */
typedef struct { uint16_t sym; uint8_t nb; uint16_t base; } fse_cell;
typedef struct { int al; fse_cell t[1 << 9]; } fse_table;

/* FSE_readNCount: returns bytes consumed or -1 */
static int64_t read_ncount(const uint8_t *src, int64_t n, int16_t *norm, int *maxsym, int *al, int maxal) {
    fbr b = {src, n * 8, 0};
    if (n < 1) return -1;
    int nbBits = (int)fbr_peek(&b, 4) + 5;
    b.pos = 4;
    if (nbBits > maxal) return -1;
    *al = nbBits;
    int remaining = (1 << nbBits) + 1, threshold = 1 << nbBits;
    nbBits++;
    int sym = 0, prev0 = 0;
    for (int i = 0; i <= *maxsym; i++) norm[i] = 0;
    while (remaining > 1 && sym <= *maxsym) {
        if (prev0) {
            int n0 = sym;
            for (;;) {
                uint32_t r = fbr_peek(&b, 2);
                b.pos += 2;
                n0 += (int)r;
                if (r != 3) break;
            }
            if (n0 > *maxsym) return -1;
            while (sym < n0) norm[sym++] = 0;
            if (b.pos > b.nbits) return -1;
        }
        int max = (2 * threshold - 1) - remaining;
        uint32_t v = fbr_peek(&b, nbBits);
        int count;
        if ((int)(v & (uint32_t)(threshold - 1)) < max) {
            count = (int)(v & (uint32_t)(threshold - 1));
            b.pos += nbBits - 1;
        } else {
            count = (int)(v & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= max;
            b.pos += nbBits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        norm[sym++] = (int16_t)count;
        prev0 = !count;
        while (remaining < threshold) { nbBits--; threshold >>= 1; }
        if (b.pos > b.nbits) return -1;
    }
    if (remaining != 1) return -1;
    *maxsym = sym - 1;
    return (b.pos + 7) >> 3;
}

static int build_fse(fse_table *t, const int16_t *norm, int maxsym, int al) {
    int size = 1 << al, high = size - 1;
    uint16_t next[256];
    uint16_t sym_at[1 << 9];
    for (int s = 0; s <= maxsym; s++) {
        if (norm[s] == -1) { sym_at[high--] = (uint16_t)s; next[s] = 1; }
        else next[s] = (uint16_t)norm[s];
    }
    int step = (size >> 1) + (size >> 3) + 3, mask = size - 1, pos = 0;
    for (int s = 0; s <= maxsym; s++) {
        for (int i = 0; i < norm[s]; i++) {
            sym_at[pos] = (uint16_t)s;
            do { pos = (pos + step) & mask; } while (pos > high);
        }
    }
    if (pos != 0) return -1;
    t->al = al;
    for (int u = 0; u < size; u++) {
        int s = sym_at[u];
        uint32_t ns = next[s]++;
        int nb = al - (31 - __builtin_clz(ns));
        t->t[u].sym = (uint16_t)s;
        t->t[u].nb = (uint8_t)nb;
        t->t[u].base = (uint16_t)((ns << nb) - (uint32_t)size);
    }
    return 0;
}

static void build_rle(fse_table *t, int sym) {
    t->al = 0;
    t->t[0].sym = (uint16_t)sym;
    t->t[0].nb = 0;
    t->t[0].base = 0;
}

/* ---------------------------------------------------------- Huffman */
typedef struct { int maxbits; uint8_t sym[1 << 12]; uint8_t nb[1 << 12]; int valid; } huf_table;

/* returns bytes consumed or -1 */
static int64_t read_huf(huf_table *h, const uint8_t *src, int64_t n) {
    uint8_t w[256];
    int nw = 0;
    if (n < 1) return -1;
    int hb = src[0];
    int64_t used;
    if (hb < 128) {  /* FSE-compressed weights */
        if (hb + 1 > n) return -1;
        int16_t norm[256];
        int maxsym = 255, al;
        int64_t c = read_ncount(src + 1, hb, norm, &maxsym, &al, 6);
        if (c < 0 || c > hb) return -1;
        fse_table t;
        if (build_fse(&t, norm, maxsym, al)) return -1;
        bbr b;
        if (bbr_init(&b, src + 1 + c, hb - c)) return -1;
        uint32_t s1 = bbr_read(&b, al), s2 = bbr_read(&b, al);
        for (;;) {
            if (nw > 253) return -1;
            w[nw++] = (uint8_t)t.t[s1].sym;
            s1 = t.t[s1].base + bbr_read(&b, t.t[s1].nb);
            if (bbr_overflow(&b)) { w[nw++] = (uint8_t)t.t[s2].sym; break; }
            if (nw > 253) return -1;
            w[nw++] = (uint8_t)t.t[s2].sym;
            s2 = t.t[s2].base + bbr_read(&b, t.t[s2].nb);
            if (bbr_overflow(&b)) { w[nw++] = (uint8_t)t.t[s1].sym; break; }
        }
        used = 1 + hb;
    } else {  /* direct 4-bit weights */
        nw = hb - 127;
        int64_t bytes = (nw + 1) / 2;
        if (1 + bytes > n) return -1;
        for (int i = 0; i < nw; i++) {
            uint8_t b = src[1 + i / 2];
            w[i] = (i & 1) ? (b & 15) : (b >> 4);
        }
        used = 1 + bytes;
    }
    /* implied last weight */
    uint32_t sum = 0;
    for (int i = 0; i < nw; i++) {
        if (w[i] >= 12) return -1;  /* HUF_TABLELOG_MAX */
        if (w[i]) sum += 1u << (w[i] - 1);
    }
    if (sum == 0) return -1;
    int maxbits = 32 - __builtin_clz(sum);  /* highbit(sum) + 1 */
    if (maxbits > 12) return -1;
    uint32_t rest = (1u << maxbits) - sum;
    if (rest & (rest - 1)) return -1;       /* must be a power of two */
    w[nw++] = (uint8_t)((31 - __builtin_clz(rest)) + 1);
    {   /* a valid prefix code has an even number (>= 2) of longest codes */
        int r1 = 0;
        for (int i = 0; i < nw; i++) r1 += w[i] == 1;
        if (r1 < 2 || (r1 & 1)) return -1;
    }
    /* table: by weight ascending, then symbol order; weight w -> 2^(w-1) cells */
    uint32_t start[14] = {0}, cnt[14] = {0};
    for (int i = 0; i < nw; i++) cnt[w[i]]++;
    uint32_t acc = 0;
    for (int k = 1; k <= maxbits; k++) { start[k] = acc; acc += cnt[k] << (k - 1); }
    for (int i = 0; i < nw; i++) {
        int k = w[i];
        if (!k) continue;
        uint32_t len = 1u << (k - 1);
        for (uint32_t u = start[k]; u < start[k] + len; u++) {
            h->sym[u] = (uint8_t)i;
            h->nb[u] = (uint8_t)(maxbits + 1 - k);
        }
        start[k] += len;
    }
    h->maxbits = maxbits;
    h->valid = 1;
    return used;
}

static int huf_stream(const huf_table *h, const uint8_t *src, int64_t n, uint8_t *out, int64_t cnt) {
    bbr b;
    if (bbr_init(&b, src, n)) return -1;
    for (int64_t i = 0; i < cnt; i++) {
        uint32_t v = bbr_peek(&b, h->maxbits);
        out[i] = h->sym[v];
        b.left -= h->nb[v];
        if (b.left < 0) return -1;
    }
    return bbr_done(&b) ? 0 : -1;
}

/* --------------------------------------------------------- sequences */
static const int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t LL_BASE[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,   10,  11,  12,   13,   14,   15,    16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t ML_BASE[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,  16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,  32,  33,  34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,  0,  0,  0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

typedef struct {
    fse_table ll, of, ml;
    int have_ll, have_of, have_ml;
    huf_table huf;
    uint32_t rep[3];
} zo_state;

/* one table per mode; returns bytes consumed or -1 */
static int64_t seq_table(fse_table *t, int *have, int mode, const uint8_t *src, int64_t n, const int16_t *def,
                         int defmax, int defal, int maxsym, int maxal) {
    if (mode == 0) {
        /* the predefined distribution covers symbols 0..defmax (RFC 8878
         * 3.1.1.3.2.2; OF: 0..28 while codes go to 31) */
        int16_t norm[64];
        memcpy(norm, def, sizeof(int16_t) * (defmax + 1));
        if (build_fse(t, norm, defmax, defal)) return -1;
        *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (n < 1 || src[0] > maxsym) return -1;
        build_rle(t, src[0]);
        *have = 1;
        return 1;
    }
    if (mode == 2) {
        int16_t norm[64];
        int ms = maxsym, al;
        int64_t c = read_ncount(src, n, norm, &ms, &al, maxal);
        if (c < 0 || c > n) return -1;
        if (build_fse(t, norm, ms, al)) return -1;
        *have = 1;
        return c;
    }
    return *have ? 0 : -1;  /* repeat */
}

/* decode one compressed block */
static int64_t zo_block(zo_state *st, const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap, int64_t op,
                        int64_t base, uint8_t *litbuf) {
    if (n < 3) return ZO_ERR_CORRUPT;  /* MIN_CBLOCK_SIZE */
    /* literals */
    int ltype = src[0] & 3, sf = (src[0] >> 2) & 3;
    int64_t regen, csize = 0, hsz;
    int streams = 1;
    int64_t ip;
    if (ltype <= 1) {
        if (sf == 0 || sf == 2) { regen = src[0] >> 3; hsz = 1; }
        else if (sf == 1) { if (n < 2) return ZO_ERR_CORRUPT; regen = (src[0] >> 4) | (src[1] << 4); hsz = 2; }
        else { if (n < 3) return ZO_ERR_CORRUPT; regen = (src[0] >> 4) | (src[1] << 4) | ((int64_t)src[2] << 12); hsz = 3; }
        if (ltype == 0) {
            if (hsz + regen > n) return ZO_ERR_CORRUPT;
            memcpy(litbuf, src + hsz, regen);
            ip = hsz + regen;
        } else {
            if (hsz + 1 > n) return ZO_ERR_CORRUPT;
            memset(litbuf, src[hsz], regen);
            ip = hsz + 1;
        }
    } else {
        uint32_t h = 0;
        if (ltype == 3 && !st->huf.valid) return ZO_ERR_CORRUPT;
        if (n < 5) return ZO_ERR_CORRUPT;
        if (sf <= 1) {
            if (n < 3) return ZO_ERR_CORRUPT;
            h = src[0] | (src[1] << 8) | ((uint32_t)src[2] << 16);
            regen = (h >> 4) & 0x3FF; csize = (h >> 14) & 0x3FF; hsz = 3; streams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
            if (n < 4) return ZO_ERR_CORRUPT;
            h = rd32le(src);
            regen = (h >> 4) & 0x3FFF; csize = (h >> 18) & 0x3FFF; hsz = 4; streams = 4;
        } else {
            if (n < 5) return ZO_ERR_CORRUPT;
            uint64_t hh = rd32le(src) | ((uint64_t)src[4] << 32);
            regen = (hh >> 4) & 0x3FFFF; csize = (hh >> 22) & 0x3FFFF; hsz = 5; streams = 4;
        }
        if (regen > (128 << 10)) return ZO_ERR_CORRUPT;
        if (hsz + csize > n) return ZO_ERR_CORRUPT;
        const uint8_t *lp = src + hsz;
        int64_t ln = csize;
        if (ltype == 2) {
            int64_t u = read_huf(&st->huf, lp, ln);
            if (u < 0) return ZO_ERR_CORRUPT;
            lp += u; ln -= u;
        }
        if (streams == 1) {
            if (huf_stream(&st->huf, lp, ln, litbuf, regen)) return ZO_ERR_CORRUPT;
        } else {
            if (ln < 10) return ZO_ERR_CORRUPT;
            int64_t s1 = lp[0] | (lp[1] << 8), s2 = lp[2] | (lp[3] << 8), s3 = lp[4] | (lp[5] << 8);
            int64_t s4 = ln - 6 - s1 - s2 - s3;
            if (s4 < 1) return ZO_ERR_CORRUPT;
            int64_t seg = (regen + 3) / 4;
            const uint8_t *q = lp + 6;
            if (huf_stream(&st->huf, q, s1, litbuf, seg)) return ZO_ERR_CORRUPT;
            if (huf_stream(&st->huf, q + s1, s2, litbuf + seg, seg)) return ZO_ERR_CORRUPT;
            if (huf_stream(&st->huf, q + s1 + s2, s3, litbuf + 2 * seg, seg)) return ZO_ERR_CORRUPT;
            int64_t c4 = regen - 3 * seg > 0 ? regen - 3 * seg : 0;
            if (huf_stream(&st->huf, q + s1 + s2 + s3, s4, litbuf + 3 * seg, c4)) return ZO_ERR_CORRUPT;
        }
        ip = hsz + csize;
    }
    /* sequences */
    if (ip >= n) return ZO_ERR_SRCSIZE;
    int64_t nseq = src[ip++];
    if (nseq >= 128) {
        if (nseq == 255) {
            if (ip + 2 > n) return ZO_ERR_SRCSIZE;
            nseq = src[ip] + (src[ip + 1] << 8) + 0x7F00;
            ip += 2;
        } else {
            if (ip + 1 > n) return ZO_ERR_SRCSIZE;
            nseq = ((nseq - 128) << 8) + src[ip];
            ip += 1;
        }
    }
    int64_t lit_used = 0;
    if (nseq > 0) {
        if (ip >= n) return ZO_ERR_SRCSIZE;
        int modes = src[ip++];
        if ((modes & 3) && zo_strict_reserved) return ZO_ERR_CORRUPT;
        int64_t c;
        c = seq_table(&st->ll, &st->have_ll, modes >> 6, src + ip, n - ip, LL_DEF, 35, 6, 35, 9);
        if (c < 0) return ZO_ERR_CORRUPT;
        ip += c;
        c = seq_table(&st->of, &st->have_of, (modes >> 4) & 3, src + ip, n - ip, OF_DEF, 28, 5, 31, 8);
        if (c < 0) return ZO_ERR_CORRUPT;
        ip += c;
        c = seq_table(&st->ml, &st->have_ml, (modes >> 2) & 3, src + ip, n - ip, ML_DEF, 52, 6, 52, 9);
        if (c < 0) return ZO_ERR_CORRUPT;
        ip += c;
        bbr b;
        if (bbr_init(&b, src + ip, n - ip)) return ZO_ERR_CORRUPT;
        uint32_t sll = bbr_read(&b, st->ll.al), sof = bbr_read(&b, st->of.al), sml = bbr_read(&b, st->ml.al);
        for (int64_t i = 0; i < nseq; i++) {
            /* libzstd checks the bit budget before decoding each sequence, so
             * the sequence whose reads over-ran is still executed first. */
            if (bbr_overflow(&b)) return ZO_ERR_CORRUPT;
            uint32_t llc = st->ll.t[sll].sym, ofc = st->of.t[sof].sym, mlc = st->ml.t[sml].sym;
            if (llc > 35 || mlc > 52 || ofc > 31) return ZO_ERR_CORRUPT;
            uint64_t ofv = (1ull << ofc) + bbr_read(&b, ofc);  /* offset bits first */
            uint64_t ml = ML_BASE[mlc] + bbr_read(&b, ML_BITS[mlc]);
            uint64_t ll = LL_BASE[llc] + bbr_read(&b, LL_BITS[llc]);
            uint64_t off;
            if (ofv > 3) {
                off = ofv - 3;
                st->rep[2] = st->rep[1]; st->rep[1] = st->rep[0]; st->rep[0] = (uint32_t)off;
            } else {
                uint32_t k = (uint32_t)ofv - 1 + (ll == 0);  /* 0..3 */
                if (k == 0) {
                    off = st->rep[0];
                } else {
                    uint64_t t = k == 3 ? (uint64_t)st->rep[0] - 1 : st->rep[k];
                    if (t == 0) t = 1;  /* libzstd: 0 is invalid, forced to 1 */
                    if (k != 1) st->rep[2] = st->rep[1];
                    st->rep[1] = st->rep[0];
                    st->rep[0] = (uint32_t)t;
                    off = t;
                }
            }
            if (i + 1 < nseq) {  /* state updates: LL, ML, OF */
                sll = st->ll.t[sll].base + bbr_read(&b, st->ll.t[sll].nb);
                sml = st->ml.t[sml].base + bbr_read(&b, st->ml.t[sml].nb);
                sof = st->of.t[sof].base + bbr_read(&b, st->of.t[sof].nb);
            }
            /* execute */
            if (op + (int64_t)ll + (int64_t)ml > cap) return ZO_ERR_DSTSMALL;
            if (lit_used + (int64_t)ll > regen) return ZO_ERR_CORRUPT;
            memcpy(dst + op, litbuf + lit_used, ll);
            op += ll;
            lit_used += ll;
            if (off > (uint64_t)(op - base)) return ZO_ERR_CORRUPT;
            for (uint64_t k2 = 0; k2 < ml; k2++) dst[op + k2] = dst[op - off + k2];
            op += ml;
        }
        if (!bbr_done(&b)) return ZO_ERR_CORRUPT;
    } else if (ip != n) {
        return ZO_ERR_SRCSIZE;
    }
    int64_t rest = regen - lit_used;
    if (op + rest > cap) return ZO_ERR_DSTSMALL;
    memcpy(dst + op, litbuf + lit_used, rest);
    return op + rest;
}

/* ZSTD_getFrameContentSize-like probe of the first frame: FCS or -1 (unknown / error / skippable) */
int64_t oracle_zstd_frame_content_size(const uint8_t *src, int64_t n) {
    if (n < 5) return -1;
    uint32_t magic = rd32le(src);
    if (magic != 0xFD2FB528u) return -1;
    int fhd = src[4];
    int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
    int64_t p = 5 + (single ? 0 : 1) + (did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4);
    int fcs_size = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (fcs_size == 0) return -1;
    if (p + fcs_size > n) return -1;
    uint64_t v = 0;
    for (int i = 0; i < fcs_size; i++) v |= (uint64_t)src[p + i] << (8 * i);
    if (fcs_size == 2) v += 256;
    return (int64_t)v;
}

/* ZSTD_decompress(dst, cap, src, n) */
int64_t oracle_zstd_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap) {
    int64_t ip = 0, op = 0;
    static __thread uint8_t *litbuf = 0;
    if (!litbuf) litbuf = (uint8_t *)malloc((128 << 10) + 64);
    zo_state *st = (zo_state *)malloc(sizeof(zo_state));
    int64_t ret = 0;
    int frames_done = 0;
    /* ZSTD_decompressMultiFrame: frames while >= 5 input bytes remain */
    while (n - ip >= 5) {
        uint32_t magic = rd32le(src + ip);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  /* skippable frame */
            if (n - ip < 8) { ret = ZO_ERR_SRCSIZE; goto done; }
            uint64_t sz = rd32le(src + ip + 4);
            if ((uint64_t)(n - ip - 8) < sz) { ret = ZO_ERR_SRCSIZE; goto done; }
            ip += 8 + (int64_t)sz;
            continue;
        }
        /* ZSTD_decompressFrame: size checks come before the header is validated */
        if (n - ip < 6 + 3) { ret = ZO_ERR_SRCSIZE; goto done; }
        int64_t p = ip + 4;
        int fhd = src[p++];
        int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, check = (fhd >> 2) & 1, did = fhd & 3;
        int did_size = did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
        int fcs_size = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        int64_t fhs = 5 + (single ? 0 : 1) + did_size + fcs_size;
        if (n - ip < fhs + 3) { ret = ZO_ERR_SRCSIZE; goto done; }
        if (magic != 0xFD2FB528u) {  /* prefix_unknown; garbage after a frame reads as srcSize_wrong */
            ret = frames_done ? ZO_ERR_SRCSIZE : ZO_ERR_CORRUPT;
            goto done;
        }
        if (fhd & 8) { ret = ZO_ERR_CORRUPT; goto done; }  /* reserved bit */
        if (!single) {
            int wd = src[p++];
            if ((wd >> 3) + 10 > 31) { ret = ZO_ERR_CORRUPT; goto done; }  /* windowLog > ZSTD_WINDOWLOG_MAX */
        }
        if (did) {
            uint32_t id = 0;
            for (int i = 0; i < did_size; i++) id |= (uint32_t)src[p + i] << (8 * i);
            p += did_size;
            if (id != 0) { ret = ZO_ERR_CORRUPT; goto done; }  /* dictionary_wrong: none loaded */
        }
        int64_t fcs = -1;
        if (fcs_size) {
            uint64_t v = 0;
            for (int i = 0; i < fcs_size; i++) v |= (uint64_t)src[p + i] << (8 * i);
            if (fcs_size == 2) v += 256;
            fcs = (int64_t)v;
            p += fcs_size;
        }
        memset(st, 0, sizeof(*st));
        st->rep[0] = 1; st->rep[1] = 4; st->rep[2] = 8;
        int64_t fstart = op;
        for (;;) {
            if (n - p < 3) { ret = ZO_ERR_SRCSIZE; goto done; }
            uint32_t bh = src[p] | (src[p + 1] << 8) | ((uint32_t)src[p + 2] << 16);
            p += 3;
            int last = bh & 1, btype = (bh >> 1) & 3;
            int64_t bsize = bh >> 3;
            if (btype == 3) { ret = ZO_ERR_CORRUPT; goto done; }
            int64_t csize = btype == 1 ? 1 : bsize;
            if (csize > n - p) { ret = ZO_ERR_SRCSIZE; goto done; }
            if (btype == 1) {
                if (op + bsize > cap) { ret = ZO_ERR_DSTSMALL; goto done; }
                memset(dst + op, src[p], bsize);
                op += bsize;
            } else if (btype == 0) {
                if (op + bsize > cap) { ret = ZO_ERR_DSTSMALL; goto done; }
                memcpy(dst + op, src + p, bsize);
                op += bsize;
            } else {
                if (bsize >= (128 << 10)) { ret = ZO_ERR_SRCSIZE; goto done; }
                int64_t r = zo_block(st, src + p, bsize, dst, cap, op, fstart, litbuf);
                if (r < 0) { ret = r; goto done; }
                op = r;
            }
            p += csize;
            if (last) break;
        }
        if (fcs >= 0 && op - fstart != fcs) { ret = ZO_ERR_CORRUPT; goto done; }
        if (check) {  /* checksum_wrong when missing or different */
            if (n - p < 4) { ret = ZO_ERR_CORRUPT; goto done; }
            uint32_t want = rd32le(src + p);
            uint32_t got = (uint32_t)oracle_xxh64(dst + fstart, (size_t)(op - fstart), 0);
            if (want != got) { ret = ZO_ERR_CORRUPT; goto done; }
            p += 4;
        }
        ip = p;
        frames_done = 1;
    }
    if (n - ip > 0) { ret = ZO_ERR_SRCSIZE; goto done; }  /* input not entirely consumed */
    ret = op;
done:
    free(st);
    return ret;
}
