/* Native concurrent callers of the one-call C ABI -- a bench harness, not
 * part of the product library.  JuiceFS calls Compress / Decompress from
 * goroutines (pkg/chunk/cached_store.go, up to max-downloads 200 /
 * max-uploads 20 at once, cmd/flags.go:133-139); Python threads serialize
 * on the interpreter lock between calls, so bench.py also drives the same
 * entry point from n pthreads to measure the library alone.
 *
 * jfs_native_callers: n threads x k calls of fn(algo, dst, cap, src, len)
 * (fn = jfs_compress or jfs_decompress), all released by one barrier; call
 * (t, r) uses source (t + r) % nsrc and destination dsts[t * k + r]; its
 * latency (s) and result go to lat / ret[t * k + r].  Returns the wall time
 * (s) from the release to the last call's return. */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

typedef int64_t (*call_fn)(int, uint8_t *, int64_t, const uint8_t *, int64_t);

struct job {
    call_fn fn;
    int algo, t, k, nsrc;
    const uint8_t *const *srcs;
    const int64_t *lens;
    uint8_t *const *dsts;
    int64_t cap;
    double *lat;
    int64_t *ret;
    pthread_barrier_t *bar;
};

static double now(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + (double)ts.tv_nsec * 1e-9;
}

static void *run(void *p) {
    struct job *j = (struct job *)p;
    pthread_barrier_wait(j->bar);
    for (int r = 0; r < j->k; r++) {
        const int i = (j->t + r) % j->nsrc, o = j->t * j->k + r;
        const double t0 = now();
        j->ret[o] = j->fn(j->algo, j->dsts[o], j->cap, j->srcs[i], j->lens[i]);
        j->lat[o] = now() - t0;
    }
    return NULL;
}

double jfs_native_callers(void *fn, int algo, int n, int k, const uint8_t *const *srcs, const int64_t *lens, int nsrc,
                          uint8_t *const *dsts, int64_t cap, double *lat, int64_t *ret) {
    if (n <= 0 || k <= 0 || nsrc <= 0) return -1.0;
    pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof *th);
    struct job *jb = (struct job *)calloc((size_t)n, sizeof *jb);
    pthread_barrier_t bar;
    if (!th || !jb || pthread_barrier_init(&bar, NULL, (unsigned)n + 1)) {
        free(th);
        free(jb);
        return -1.0;
    }
    int started = 0;
    for (int t = 0; t < n; t++) {
        jb[t] = (struct job){(call_fn)fn, algo, t, k, nsrc, srcs, lens, dsts, cap, lat, ret, &bar};
        if (pthread_create(&th[t], NULL, run, &jb[t])) break;
        started++;
    }
    double wall = -1.0;
    if (started == n) {
        pthread_barrier_wait(&bar);
        const double t0 = now();
        for (int t = 0; t < n; t++) pthread_join(th[t], NULL);
        wall = now() - t0;
    } else {
        /* cannot release a partial barrier safely: abort the process (harness only) */
        abort();
    }
    pthread_barrier_destroy(&bar);
    free(th);
    free(jb);
    return wall;
}
