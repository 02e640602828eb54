// Deterministic synthetic block generator, shared by the
// HIP generator kernel and the host-side generator.  Byte-identical to
// juicefs_amd/blockgen.py.  This is benchmark/test *input* generation, not part
// of the codec path.
//
// Classes
//   'T' text-like: a fixed 4096-word vocabulary (word length 2..11, letters
//       'a'+r%26), word index drawn from 12 log-uniform buckets (~Zipf(1)),
//       space-separated, '\n' every 512 words, and with p=1/50 per line a
//       random-byte run of 64+(r%960) bytes at the start of the line.
//   'Z' zeros, 'R' uniform random bytes (splitmix64 output, little endian).
// Block i of a batch uses seed base+i.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define JFS_HD __host__ __device__ __forceinline__
#else
#define JFS_HD static inline
#endif

#define JFS_VOCAB_SEED 0x4A7566734C5A3421ull
#define JFS_VOCAB_WORDS 4096
#define JFS_WORDS_PER_LINE 512

JFS_HD uint64_t jfs_sm64(uint64_t *s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Vocabulary: 4096 entries of 16 bytes: byte 0 = length, bytes 1..11 = letters.
JFS_HD void jfs_build_vocab(uint8_t *vocab /* 4096*16 */) {
    uint64_t s = JFS_VOCAB_SEED;
    for (int w = 0; w < JFS_VOCAB_WORDS; w++) {
        uint8_t *e = vocab + 16 * w;
        int len = 2 + (int)(jfs_sm64(&s) % 10);
        e[0] = (uint8_t)len;
        for (int i = 0; i < len; i++) e[1 + i] = (uint8_t)(97 + jfs_sm64(&s) % 26);
        for (int i = 1 + len; i < 16; i++) e[i] = 0;
    }
}

// Produce exactly n bytes of class cls; emit(byte) is called n times in order.
template <class Emit>
JFS_HD void jfs_gen_stream(const uint8_t *vocab, char cls, uint64_t seed, int64_t n, Emit &emit) {
    uint64_t s = seed;
    int64_t pos = 0;
    if (cls == 'Z') {
        for (; pos < n; pos++) emit(0);
        return;
    }
    if (cls == 'R') {
        while (pos < n) {
            uint64_t r = jfs_sm64(&s);
            for (int k = 0; k < 8 && pos < n; k++, pos++) emit((uint8_t)(r >> (8 * k)));
        }
        return;
    }
    int wl = 0;
    int newline = 1;
    while (pos < n) {
        if (newline) {
            newline = 0;
            if (jfs_sm64(&s) % 50 == 0) {
                int64_t L = 64 + (int64_t)(jfs_sm64(&s) % 960);
                int64_t k = 0;
                while (k < L) {
                    uint64_t r = jfs_sm64(&s);
                    for (int b = 0; b < 8 && k < L; b++, k++) {
                        if (pos < n) emit((uint8_t)(r >> (8 * b)));
                        pos++;
                    }
                }
                continue;
            }
        }
        uint64_t x = jfs_sm64(&s);
        uint32_t kb = (uint32_t)(x % 12);
        uint32_t idx = (1u << kb) - 1 + (uint32_t)((x >> 8) % (1u << kb));
        const uint8_t *e = vocab + 16 * idx;
        int len = e[0];
        for (int i = 0; i < len; i++) {
            if (pos < n) emit(e[1 + i]);
            pos++;
        }
        wl++;
        uint8_t sep = ' ';
        if (wl == JFS_WORDS_PER_LINE) {
            sep = '\n';
            wl = 0;
            newline = 1;
        }
        if (pos < n) emit(sep);
        pos++;
    }
}
