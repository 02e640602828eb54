/*
 * oracle/lz4_oracle.c -- CPU restatement of the LZ4 *block* codec that JuiceFS
 * reaches through pkg/compress (TEST INFRASTRUCTURE ONLY).
 *
 * This file is the parity checker for the HIP kernels.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product library (libjfsgpu.so) never links or calls it.
 *
 * What it restates
 *   pkg/compress/compress.go:112  LZ4.CompressBound  -> lz4.CompressBound  -> LZ4_compressBound
 *   pkg/compress/compress.go:115  LZ4.Compress       -> lz4.CompressDefault -> LZ4_compress_default
 *   pkg/compress/compress.go:120  LZ4.Decompress     -> lz4.DecompressSafe  -> LZ4_decompress_safe
 * The arithmetic lives in the third-party dependency
 *   github.com/hungys/go-lz4 v0.0.0-20170805124057-19ff7f07f099 (go.mod:48),
 * which vendors LZ4 C sources that are not present in /root/reference.  This
 * restatement follows the published LZ4 block format and the control flow of
 * liblz4 1.9.3 (LZ4_compress_generic / LZ4_decompress_generic with the x86-64
 * LZ4_FAST_DEC_LOOP), the version available in this image.  It is *pinned* by
 * tests/golden (fixtures produced by liblz4 1.9.3 via ctypes) -- byte-exact
 * compressed output, exact return values (including the negative error
 * positions) on a mutation corpus.  Parity against the 2017 vendored copy is
 * unverified (no Go toolchain / module cache offline); see DESIGN.md.
 */
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

#define MINMATCH 4
#define MFLIMIT 12
#define LASTLITERALS 5
#define RUN_MASK 15
#define ML_MASK 15
#define LZ4_MAX_INPUT_SIZE 0x7E000000
#define LZ4_64KLIMIT (65536 + MFLIMIT - 1)
#define DISTANCE_MAX 65535
#define FASTLOOP_SAFE_DISTANCE 64

int64_t oracle_lz4_bound(int64_t n) {
    if (n < 0 || n > LZ4_MAX_INPUT_SIZE) return 0;
    return n + n / 255 + 16;
}

static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }

/* hash of the 4 (byU16) or 5 (byU32, 64-bit reg) bytes at p */
static inline uint32_t hpos(const uint8_t *p, int u16) {
    if (u16) return (rd32(p) * 2654435761u) >> 19;               /* 13-bit, 8192 x u16 */
    return (uint32_t)(((rd64(p) << 24) * 889523592379ull) >> 52); /* 12-bit, 4096 x u32 */
}

/* Emit one length field continuation (255-runs) */
static inline uint8_t *put_len(uint8_t *op, uint32_t len) {
    for (; len >= 255; len -= 255) *op++ = 255;
    *op++ = (uint8_t)len;
    return op;
}

/* LZ4_compress_default(src, dst, n, cap): greedy single-pass parse with the
 * acceleration-1 skip schedule.  Returns compressed size, or 0 when it does not
 * fit in cap (liblz4's limitedOutput checks are exact-or-weaker, so "fits"
 * decides it). */
int oracle_lz4_compress_default(const uint8_t *src, uint8_t *dst, int n, int cap) {
    if ((uint32_t)n > (uint32_t)LZ4_MAX_INPUT_SIZE) return 0;
    if (n == 0) {
        if (cap <= 0) return 0;
        dst[0] = 0;
        return 1;
    }
    /* unbounded scratch: worst case is the bound */
    int64_t bound = oracle_lz4_bound(n);
    uint8_t *out = dst;
    uint8_t *tmp = 0;
    static __thread uint8_t *scratch = 0; static __thread int64_t scap = 0;
    if (cap < bound) {
        if (scap < bound) { free(scratch); scratch = (uint8_t *)malloc((size_t)bound); scap = bound; }
        tmp = scratch; out = tmp;
    }
    const int u16 = n < LZ4_64KLIMIT;
    uint32_t table32[4096]; uint16_t table16[8192];
    if (u16) memset(table16, 0, sizeof table16); else memset(table32, 0, sizeof table32);
#define TGET(h) (u16 ? (uint32_t)table16[h] : table32[h])
#define TPUT(h, v) do { if (u16) table16[h] = (uint16_t)(v); else table32[h] = (uint32_t)(v); } while (0)

    const int64_t iend = n, mflimitP1 = n - MFLIMIT + 1, matchlimit = n - LASTLITERALS;
    int64_t ip = 0, anchor = 0;
    uint8_t *op = out;
    if (n < MFLIMIT + 1) goto last_literals;
    TPUT(hpos(src, u16), 0);
    ip = 1;
    uint32_t fh = hpos(src + ip, u16);
    for (;;) {
        int64_t match;
        /* search */
        {
            int64_t fip = ip;
            int step = 1, snb = 1 << 6;
            for (;;) {
                uint32_t h = fh;
                int64_t cur = fip;
                uint32_t mi = TGET(h);
                ip = fip;
                fip += step;
                step = snb++ >> 6;
                if (fip > mflimitP1) goto last_literals;
                match = mi;
                fh = hpos(src + fip, u16);
                TPUT(h, cur);
                if (!u16 && mi + DISTANCE_MAX < cur) continue;
                if (rd32(src + match) == rd32(src + ip)) break;
            }
        }
        /* catch up */
        while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) { ip--; match--; }
        uint8_t *token;
        {
            uint32_t lit = (uint32_t)(ip - anchor);
            token = op++;
            if (lit >= RUN_MASK) { *token = RUN_MASK << 4; op = put_len(op, lit - RUN_MASK); }
            else *token = (uint8_t)(lit << 4);
            memcpy(op, src + anchor, lit);
            op += lit;
        }
    next_match:
        op[0] = (uint8_t)(ip - match); op[1] = (uint8_t)((ip - match) >> 8); op += 2;
        {
            int64_t a = ip + MINMATCH, b = match + MINMATCH;
            while (a < matchlimit && src[a] == src[b]) { a++; b++; }
            uint32_t mc = (uint32_t)(a - (ip + MINMATCH));
            ip = a;
            if (mc >= ML_MASK) { *token += ML_MASK; op = put_len(op, mc - ML_MASK); }
            else *token += (uint8_t)mc;
        }
        anchor = ip;
        if (ip >= mflimitP1) break;
        TPUT(hpos(src + ip - 2, u16), ip - 2);
        {
            uint32_t h = hpos(src + ip, u16);
            uint32_t mi = TGET(h);
            TPUT(h, ip);
            if ((u16 || mi + DISTANCE_MAX >= (uint64_t)ip) && rd32(src + mi) == rd32(src + ip)) {
                match = mi;
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fh = hpos(src + (++ip), u16);
    }
last_literals:
    {
        uint32_t last = (uint32_t)(iend - anchor);
        if (last >= RUN_MASK) { *op++ = RUN_MASK << 4; op = put_len(op, last - RUN_MASK); }
        else *op++ = (uint8_t)(last << 4);
        memcpy(op, src + anchor, last);
        op += last;
    }
    int64_t csize = op - out;
    if (tmp) {
        if (csize > cap) return 0;
        memcpy(dst, tmp, (size_t)csize);
    }
    return (int)csize;
#undef TGET
#undef TPUT
}

/* read_variable_length(): returns 0 ok, -1 initial error, -2 loop error */
static inline int rvl(const uint8_t *src, int64_t *ip, int64_t lencheck, int loop_check,
                      int initial_check, uint64_t *len) {
    if (initial_check && *ip >= lencheck) return -1;
    uint32_t s;
    do {
        s = src[(*ip)++];
        *len += s;
        if (loop_check && *ip >= lencheck) return -2;
    } while (s == 255);
    return 0;
}

/* forward copy of a match with liblz4's output semantics (offset 0 -> zeros) */
static inline void match_copy(uint8_t *dst, int64_t op, int64_t off, int64_t len) {
    if (off == 0) { memset(dst + op, 0, (size_t)len); return; }
    for (int64_t i = 0; i < len; i++) dst[op + i] = dst[op - off + i];
}

/* LZ4_decompress_safe(src, dst, srcSize, cap): decode sequence by sequence with
 * the acceptance checks of liblz4 1.9.3 in the order it makes them (fast loop
 * while >= 64 bytes of output room remain, then the safe loop), so the return
 * value -- decoded size, or -(input position of the failing check)-1 -- is the
 * same.  Bytes [0, ret) of dst are the decoded block on success. */
int oracle_lz4_decompress_safe(const uint8_t *src, uint8_t *dst, int srcSize, int cap) {
    if (!src) return -1;
    const int64_t iend = srcSize, oend = cap;
    int64_t ip = 0, op = 0;
    if (cap == 0) return (srcSize == 1 && src[0] == 0) ? 0 : -1;
    if (srcSize == 0) return -1;
    const int64_t shortiend = iend - 14 - 2, shortoend = oend - 14 - 18;
    uint32_t token;
    uint64_t length;
    int64_t offset, match, cpy;

    if (oend - op < FASTLOOP_SAFE_DISTANCE) goto safe_decode;
    for (;;) { /* fast loop */
        token = src[ip++];
        length = token >> 4;
        if (length == RUN_MASK) {
            int e = rvl(src, &ip, iend - RUN_MASK, 1, 1, &length);
            if (e == -1) goto output_error;
            cpy = op + (int64_t)length;
            if (cpy > oend - 32 || ip + (int64_t)length > iend - 32) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += length; op = cpy;
        } else {
            cpy = op + (int64_t)length;
            if (ip > iend - 17) goto safe_literal_copy;
            memcpy(dst + op, src + ip, length);
            ip += length; op = cpy;
        }
        offset = src[ip] | (src[ip + 1] << 8); ip += 2;
        match = op - offset;
        length = token & ML_MASK;
        if (length == ML_MASK) {
            if (match < 0) goto output_error;
            int e = rvl(src, &ip, iend - LASTLITERALS + 1, 1, 0, &length);
            if (e != 0) goto output_error;
            length += MINMATCH;
            if (op + (int64_t)length >= oend - FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
        } else {
            length += MINMATCH;
            if (op + (int64_t)length >= oend - FASTLOOP_SAFE_DISTANCE) goto safe_match_copy;
        }
        if (match < 0) goto output_error;
        match_copy(dst, op, offset, length);
        op += length;
    }
safe_decode:
    for (;;) {
        token = src[ip++];
        length = token >> 4;
        if (length != RUN_MASK && ip < shortiend && op <= shortoend) {
            memcpy(dst + op, src + ip, length);
            op += length; ip += length;
            length = token & ML_MASK;
            offset = src[ip] | (src[ip + 1] << 8); ip += 2;
            match = op - offset;
            if (length != ML_MASK && offset >= 8 && match >= 0) {
                match_copy(dst, op, offset, length + MINMATCH);
                op += length + MINMATCH;
                continue;
            }
            goto copy_match;
        }
        if (length == RUN_MASK) {
            int e = rvl(src, &ip, iend - RUN_MASK, 1, 1, &length);
            if (e == -1) goto output_error;
        }
        cpy = op + (int64_t)length;
    safe_literal_copy:
        if (cpy > oend - MFLIMIT || ip + (int64_t)length > iend - (2 + 1 + LASTLITERALS)) {
            if (ip + (int64_t)length != iend || cpy > oend) goto output_error;
            memmove(dst + op, src + ip, length);
            ip += length; op += length;
            break;
        }
        memcpy(dst + op, src + ip, length);
        ip += length; op = cpy;
        offset = src[ip] | (src[ip + 1] << 8); ip += 2;
        match = op - offset;
        length = token & ML_MASK;
    copy_match:
        if (length == ML_MASK) {
            int e = rvl(src, &ip, iend - LASTLITERALS + 1, 1, 0, &length);
            if (e != 0) goto output_error;
        }
        length += MINMATCH;
    safe_match_copy:
        if (match < 0) goto output_error;
        cpy = op + (int64_t)length;
        if (cpy > oend - 12) {
            if (cpy > oend - LASTLITERALS) goto output_error;
        }
        match_copy(dst, op, offset, length);
        op = cpy;
    }
    return (int)op;
output_error:
    return (int)(-ip) - 1;
}
