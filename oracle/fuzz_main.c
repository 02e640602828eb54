/* Sanitizer driver for the CPU oracle (test infrastructure only): builds
 * valid LZ4 blocks and Zstd frames with the oracle's own encoder / from
 * caller-provided frames, then decodes them and thousands of truncated and
 * bit-flipped variants into exact-size and short destinations.  Built with
 * -fsanitize=address,undefined by `make -C oracle asan`; any out-of-bounds
 * access or UB aborts the run (tests/test_oracle_sanitize.py). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

int64_t oracle_lz4_bound(int64_t n);
int oracle_lz4_compress_default(const uint8_t *src, uint8_t *dst, int n, int cap);
int oracle_lz4_decompress_safe(const uint8_t *src, uint8_t *dst, int srcSize, int cap);
int64_t oracle_zstd_decompress(const uint8_t *src, int64_t n, uint8_t *dst, int64_t cap);

static uint64_t rs = 0x1234567u;
static uint64_t rnd(void) {
    uint64_t z = (rs += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* text-ish bytes: words from a small vocabulary with random runs */
static void gen(uint8_t *p, int n) {
    static const char *w[] = {"the ", "data ", "block ", "chunk ", "slice ", "juice ", "object ", "cache "};
    int i = 0;
    while (i < n) {
        if (rnd() % 40 == 0) {
            int r = 1 + (int)(rnd() % 200);
            for (int k = 0; k < r && i < n; k++) p[i++] = (uint8_t)rnd();
        } else {
            const char *s = w[rnd() % 8];
            for (int k = 0; s[k] && i < n; k++) p[i++] = (uint8_t)s[k];
        }
    }
}

/* decode one input into heap buffers of exactly `cap` bytes (ASan sees overruns) */
static void lz4_one(const uint8_t *c, int n, int cap) {
    uint8_t *src = (uint8_t *)malloc(n > 0 ? (size_t)n : 1);
    uint8_t *dst = (uint8_t *)malloc(cap > 0 ? (size_t)cap : 1);
    if (n > 0) memcpy(src, c, (size_t)n);
    (void)oracle_lz4_decompress_safe(src, dst, n, cap);
    free(src);
    free(dst);
}
static void zstd_one(const uint8_t *c, int64_t n, int64_t cap) {
    uint8_t *src = (uint8_t *)malloc(n > 0 ? (size_t)n : 1);
    uint8_t *dst = (uint8_t *)malloc(cap > 0 ? (size_t)cap : 1);
    if (n > 0) memcpy(src, c, (size_t)n);
    (void)oracle_zstd_decompress(src, n, dst, cap);
    free(src);
    free(dst);
}

static long read_file(const char *path, uint8_t **out) {
    FILE *f = fopen(path, "rb");
    if (!f) return -1;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    *out = (uint8_t *)malloc((size_t)n);
    if (fread(*out, 1, (size_t)n, f) != (size_t)n) n = -1;
    fclose(f);
    return n;
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 2000;
    long cases = 0;
    /* LZ4: oracle-encoded blocks, then variants */
    for (int it = 0; it < iters; it++) {
        const int n = 1 + (int)(rnd() % (it % 10 == 0 ? 300000 : 5000));
        uint8_t *raw = (uint8_t *)malloc((size_t)n);
        gen(raw, n);
        const int bound = (int)oracle_lz4_bound(n);
        uint8_t *c = (uint8_t *)malloc((size_t)bound);
        const int m = oracle_lz4_compress_default(raw, c, n, bound);
        if (m <= 0) { fprintf(stderr, "encode failed\n"); return 2; }
        lz4_one(c, m, n);
        lz4_one(c, m, n > 1 ? n - 1 - (int)(rnd() % (n > 16 ? 16 : n - 1)) : 0);
        lz4_one(c, (int)(rnd() % (unsigned)m), n);
        for (int k = 0; k < 4; k++) {
            uint8_t *d = (uint8_t *)malloc((size_t)m);
            memcpy(d, c, (size_t)m);
            for (int f = 0; f < 1 + (int)(rnd() % 4); f++) d[rnd() % (unsigned)m] ^= (uint8_t)(1u << (rnd() % 8));
            if (rnd() % 3 == 0) d[rnd() % (unsigned)m] = 0xFF;
            lz4_one(d, m, n);
            lz4_one(d, m, (int)(rnd() % (unsigned)(n + 1)));
            free(d);
        }
        cases += 7;
        free(raw);
        free(c);
    }
    /* Zstd: frames from a file of (u32 size, bytes) records, then variants */
    for (int a = 2; a < argc; a++) {
        uint8_t *buf = NULL;
        const long len = read_file(argv[a], &buf);
        if (len < 0) { fprintf(stderr, "cannot read %s\n", argv[a]); return 2; }
        long o = 0;
        while (o + 8 <= len) {
            uint32_t fs, us;
            memcpy(&fs, buf + o, 4);
            memcpy(&us, buf + o + 4, 4);
            o += 8;
            if (o + fs > (uint32_t)len) break;
            const uint8_t *fr = buf + o;
            o += fs;
            zstd_one(fr, fs, us);
            zstd_one(fr, fs, us ? us - 1 : 0);
            for (int k = 0; k < 24; k++) {
                uint8_t *d = (uint8_t *)malloc(fs ? fs : 1);
                memcpy(d, fr, fs);
                const int64_t cut = rnd() % 4 == 0 ? (int64_t)(rnd() % (fs + 1)) : (int64_t)fs;
                for (int f = 0; f < 1 + (int)(rnd() % 3) && fs; f++) d[rnd() % fs] ^= (uint8_t)(1u << (rnd() % 8));
                zstd_one(d, cut, us + (int64_t)(rnd() % 64));
                free(d);
            }
            cases += 26;
        }
        free(buf);
    }
    printf("sanitized oracle run: %ld cases\n", cases);
    return 0;
}
