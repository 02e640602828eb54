// libjfsgpu.so host side: the C ABI declared in include/jfs_gpucodec.h.
//
// Mirrors pkg/compress (compress.go:31-125) for the Go/cgo caller and adds the
// batch and device-resident entry points.  Every LZ4 byte is produced by the
// HIP kernels; if no gfx950 device is usable the codec calls fail with
// JFS_ERR_NO_DEVICE -- there is no CPU fallback.  Only the "none" codec is a
// host memcpy, because that is what noOp is (compress.go:55-68).
//
// Concurrency model (pkg/chunk runs up to 20 Compress + 200 Decompress calls
// at once, cmd/flags.go:133-139): single-block calls enqueue on a per-process
// coalescer; NLANE worker threads per device drain the queue, each gathering a
// burst of calls (a short gather window, Gather below) into one batch, and a
// device runs the next batch while the previous one is in flight (one lane of
// staging and streams per worker).  Batches go host -> pinned staging -> HBM
// -> kernel -> HBM -> pinned -> host, pipelined in chunks (run_batch).
#include <hip/hip_runtime.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/jfs_gpucodec_test.h"
#include "blockgen.h"
#include "jfs_internal.h"

#define JFS_VERSION "jfs-gpucodec 0.1.0 (gfx950)"

namespace {

constexpr int64_t LZ4_MAX_INPUT = 0x7E000000;

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

// JFS_HOST_TRACE=1: per-chunk host timings on stderr (diagnostics)
bool host_trace() {
    static bool v = getenv("JFS_HOST_TRACE") != nullptr;
    return v;
}
double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
// (trace) a staging or scratch allocation: hipFree waits for the whole device
void trace_alloc(const char *what, int64_t bytes, double t0) {
    if (host_trace())
        fprintf(stderr, "[jfs host] t=%.2f alloc %s %.1f MiB %.2f ms\n", now_ms(), what, bytes / 1048576.0,
                now_ms() - t0);
}

// One pinned host + device staging area: chunk k of a batch uses slot
// k % NSLOT, so chunk k+1's H2D and chunk k-1's D2H run while chunk k's
// kernel runs.  (Four slots measured 42.8 vs 42.0 GiB/s on a lone 4,096-block
// host-to-host decode, but 28 vs 41 right after a configs[0] round trip had
// grown the staging: kept at three.)
#ifndef JFS_NSLOT
#define JFS_NSLOT 3
#endif
constexpr int NSLOT = JFS_NSLOT;
static_assert(NSLOT >= 2, "the staging pipeline overlaps a chunk's copies with the next chunk's");
// disk-cache checksum piece (pkg/chunk/disk_cache_file.go:139-152: csBlock)
constexpr int64_t CSUM_SEG = 32 << 10;

// Upper bound on one slot's staging (JFS_STAGING_MAX_MB; default none): a
// request that needs more fails alone with JFS_ERR_NO_MEMORY.
// Footprint without a cap: a slot holds one chunk's input + output, at most
// the chunk limit (2 GiB decode, 4 GiB LZ4 / Zstd compress) plus one block;
// a lane has NSLOT = 3 slots and a device NLANE = 2 lanes, each slot pinned
// on the host and mirrored in HBM.  Peak per device: 2 x 3 x 4 GiB = 24 GiB
// pinned + 24 GiB HBM when both lanes run compress batches (e.g. LZ4 and Zstd
// at once), 12 + 12 GiB for two decode lanes; freed after JFS_STAGING_IDLE_MS
// of inactivity or by jfs_release_staging().  Hosts with less memory to pin
// set JFS_STAGING_MAX_MB (and JFS_HOST_CHUNK_MB[_LZ4C] to keep chunks under it).
int64_t staging_max_bytes() {
    static int64_t v = [] {
        const char *e = getenv("JFS_STAGING_MAX_MB");
        return e ? (int64_t)atoll(e) << 20 : INT64_MAX;
    }();
    return v;
}

// The output D2H of a (non-encrypted) chunk goes in up to NPIECE pieces, each
// with its own event, so the host copy-out of a piece overlaps the D2H of the
// next -- at the end of a batch only the last piece's copy-out is left.
#ifndef JFS_NPIECE
#define JFS_NPIECE 4
#endif
constexpr int NPIECE = JFS_NPIECE;

// Output pieces of a one-block chunk (a lone cache miss): its output D2H goes
// in NPIECE byte ranges and the caller copies each out as soon as it lands,
// spinning on the piece's event (a blocking wait per piece cost more than the
// overlap saved).  Lone 4 MiB one-call decode in the full bench: LZ4 0.81 ->
// 0.70 ms, Zstd 2.34 -> 2.23 ms (scripts/r6_bpiece3.sh).
// JFS_BYTE_PIECES=n overrides (0 or 1 = whole output).
int byte_npiece() {
    static int v = [] {
        const char *e = getenv("JFS_BYTE_PIECES");
        return e ? std::min(NPIECE, std::max(0, atoi(e))) : NPIECE;
    }();
    return v;
}

static_assert(NPIECE >= 1, "at least one output piece per chunk (finish() waits on ev_p[npiece - 1])");
struct Slot {
    hipEvent_t ev_in = nullptr, ev_k = nullptr, ev = nullptr;  // H2D done, kernel done, D2H done
    hipEvent_t ev_p[NPIECE] = {};                              // output piece p landed
    uint8_t *h = nullptr;
    int64_t h_cap = 0;
    uint8_t *d = nullptr;
    int64_t d_cap = 0;
    // Zstd decode scratch of this slot (planned on the host per chunk)
    uint8_t *z_lit = nullptr, *z_items = nullptr;
    uint16_t *z_tabs = nullptr;
    uint64_t z_lit_cap = 0, z_items_cap = 0, z_tabs_cap = 0;
    // small-batch decode scratch (LZ4: lz4_split.hip, Zstd: zstd_split.inc)
    uint8_t *sp = nullptr;
    int64_t sp_cap = 0;

    bool ensure_split(int64_t bytes) {
        if (bytes <= sp_cap) return true;
        const double t0 = host_trace() ? now_ms() : 0.0;
        if (sp) (void)hipFree(sp);
        sp = nullptr;
        sp_cap = 0;
        int64_t want = 64ll << 20;
        while (want < bytes) want <<= 1;
        if (hipMalloc((void **)&sp, (size_t)want) != hipSuccess) return false;
        sp_cap = want;
        trace_alloc("split", want, t0);
        return true;
    }

    bool ensure_zstd(const uint64_t *t) {  // t: items, literal bytes, table cells
        auto grow = [](auto **p, uint64_t *cap, uint64_t want, size_t elem) {
            if (*cap >= want) return true;
            const double t0 = host_trace() ? now_ms() : 0.0;
            if (*p) (void)hipFree(*p);
            *p = nullptr;
            *cap = 0;
            const uint64_t n = want + want / 4;
            if (hipMalloc((void **)p, (size_t)(n * elem)) != hipSuccess) return false;
            *cap = n;
            trace_alloc("zstd", (int64_t)(n * elem), t0);
            return true;
        };
        return grow(&z_items, &z_items_cap, t[0], 16) && grow(&z_lit, &z_lit_cap, t[1], 1) &&
               grow(&z_tabs, &z_tabs_cap, t[2], 2);
    }

    bool ensure(int64_t bytes) {
        // grow to the next power of two (at least 64 MiB): pinning costs about
        // 0.1 s per GiB, so a growing workload should re-pin rarely
        int64_t want = 64ll << 20;
        while (want < bytes) want <<= 1;
        if (bytes > staging_max_bytes()) return false;
        const double t0 = host_trace() ? now_ms() : 0.0;
        if (bytes > h_cap) {
            if (h) (void)hipHostFree(h);
            if (hipHostMalloc((void **)&h, (size_t)want, hipHostMallocDefault) != hipSuccess) {
                h = nullptr;
                h_cap = 0;
                return false;
            }
            h_cap = want;
            trace_alloc("pinned", want, t0);
        }
        if (bytes > d_cap) {
            if (d) (void)hipFree(d);
            if (hipMalloc((void **)&d, (size_t)want) != hipSuccess) {
                d = nullptr;
                d_cap = 0;
                return false;
            }
            d_cap = want;
            trace_alloc("device", want, t0);
        }
        return true;
    }
};

// Streams: a process gets GPU_MAX_HW_QUEUES (4 by default) hardware queues
// per device, and work on two streams that share one runs in submission
// order -- kernels "on different streams" then serialise (measured: five
// streams of one 0.5 s kernel each take 1.0 s; scripts/stream_probe.py).  So
// the library uses exactly four streams per device: one for every H2D copy,
// one for every D2H copy (a D2H waiting for its kernel must not hold up the
// next chunk's H2D), and one kernel stream per lane.
// A lane is one staging pipeline (NSLOT slots + its kernel stream); a device
// has NLANE of them, so a second batch (the coalescer's next one, or another
// caller's jfs_*_batch) runs while the first is still in flight.
struct Lane {
    std::mutex mu;  // serialises use of this lane's slots
    Slot slot[NSLOT];
    hipStream_t s_k = nullptr;  // this lane's kernels, in chunk order
    std::atomic<int> kind{-1};  // algo * 2 + dir of the batch it last ran (acquire_lane)
    // free the pinned host and HBM staging (caller holds mu)
    void release_staging() {
        for (Slot &sl : slot) {
            if (sl.h) (void)hipHostFree(sl.h);
            if (sl.d) (void)hipFree(sl.d);
            if (sl.z_lit) (void)hipFree(sl.z_lit);
            if (sl.z_items) (void)hipFree(sl.z_items);
            if (sl.z_tabs) (void)hipFree(sl.z_tabs);
            if (sl.sp) (void)hipFree(sl.sp);
            sl.sp = nullptr;
            sl.sp_cap = 0;
            sl.h = sl.d = sl.z_lit = sl.z_items = nullptr;
            sl.z_tabs = nullptr;
            sl.h_cap = sl.d_cap = 0;
            sl.z_lit_cap = sl.z_items_cap = sl.z_tabs_cap = 0;
        }
    }
    bool holds_staging() const {
        for (const Slot &sl : slot)
            if (sl.h || sl.d || sl.z_items || sl.sp) return true;
        return false;
    }
};
constexpr int NLANE = 2;

struct DevCtx {
    int id = -1;
    Lane lane[NLANE];
    hipStream_t s_in = nullptr, s_out = nullptr;  // all H2D / all D2H copies of the device
    std::atomic<unsigned> next_lane{0};
    std::mutex vocab_mu;
    uint8_t *d_vocab = nullptr;
    std::atomic<int64_t> last_use_ms{0};  // staging janitor: release after an idle period
    std::atomic<uint64_t> batches{0}, blocks{0};  // per-device counters (jfs_device_stats)

    // a lane for a batch call: a free one if any, else wait for one
    // (kind = algo * 2 + dir, or -1: a free lane that last ran the same kind
    // first, since its staging and scratch already fit such batches -- a lane
    // that must grow them waits on hipFree, i.e. on the whole device)
    Lane &acquire_lane(std::unique_lock<std::mutex> &lk, int kind = -1) {
        for (int pass = kind < 0 ? 1 : 0; pass < 2; pass++)
            for (int k = 0; k < NLANE; k++) {
                if (pass == 0 && lane[k].kind.load(std::memory_order_relaxed) != kind) continue;
                std::unique_lock<std::mutex> t(lane[k].mu, std::try_to_lock);
                if (t.owns_lock()) {
                    lk = std::move(t);
                    return lane[k];
                }
            }
        Lane &l = lane[next_lane.fetch_add(1) % NLANE];
        lk = std::unique_lock<std::mutex>(l.mu);
        return l;
    }
};

// The library never leaves the caller on another device: every entry point
// that selects a device restores the caller's current device on return (the
// caller's runtime -- e.g. PyTorch's current stream and events -- reads it).
struct DevGuard {
    int prev = -1;
    DevGuard() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// JFS_GPU_CODEC (include/jfs_gpucodec.h): off | auto (default) | force
int gpu_mode() {
    static int m = [] {
        const char *e = getenv("JFS_GPU_CODEC");
        if (!e) return JFS_MODE_AUTO;
        std::string v(e);
        for (auto &ch : v) ch = (char)tolower((unsigned char)ch);
        if (v == "off" || v == "0" || v == "false") return JFS_MODE_OFF;
        if (v == "force") return JFS_MODE_FORCE;
        return JFS_MODE_AUTO;
    }();
    return m;
}

// JFS_GPU_DEVICES: "all" (default), a comma list of ordinals, or a 0x mask
uint64_t device_select_mask() {
    const char *e = getenv("JFS_GPU_DEVICES");
    if (!e || !*e || !strcmp(e, "all")) return ~0ull;
    if (e[0] == '0' && (e[1] == 'x' || e[1] == 'X')) return strtoull(e + 2, nullptr, 16);
    uint64_t m = 0;
    for (const char *p = e; *p;) {
        char *end = nullptr;
        const long v = strtol(p, &end, 10);
        if (end == p) break;
        if (v >= 0 && v < 64) m |= 1ull << v;
        p = *end == ',' ? end + 1 : end;
    }
    return m;
}

// per-(algo, dir) counters behind jfs_stats()
struct OpStats {
    std::atomic<uint64_t> calls{0}, blocks{0}, bytes_in{0}, bytes_out{0}, errors{0}, nanos{0}, batches{0};
};
OpStats g_stats[JFS_STATS_N];

inline OpStats *op_stats(int algo, int dir) {
    return (algo >= 0 && algo <= 2 && (dir == 0 || dir == 1)) ? &g_stats[algo * 2 + dir] : nullptr;
}

int64_t steady_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// one host-path block's outcome
inline void stat_block(OpStats *st, int64_t in, int64_t out) {
    if (!st) return;
    st->blocks.fetch_add(1, std::memory_order_relaxed);
    if (out >= 0) {
        st->bytes_in.fetch_add((uint64_t)(in > 0 ? in : 0), std::memory_order_relaxed);
        st->bytes_out.fetch_add((uint64_t)out, std::memory_order_relaxed);
    } else {
        st->errors.fetch_add(1, std::memory_order_relaxed);
    }
}

inline void stat_launch(int algo, int dir, int nblk) {
    if (OpStats *st = op_stats(algo, dir)) {
        st->calls.fetch_add(1, std::memory_order_relaxed);
        if (nblk > 0) st->blocks.fetch_add((uint64_t)nblk, std::memory_order_relaxed);
    }
}

std::once_flag g_once;
// never destroyed: the coalescer workers and the staging janitor are detached
// threads that may still look at it while static destructors run at exit
std::vector<DevCtx *> &g_devs = *new std::vector<DevCtx *>();
std::atomic<bool> g_exiting{false};

void init_devices() {
    if (gpu_mode() == JFS_MODE_OFF) return;
    DevGuard guard;
    const uint64_t sel = device_select_mask();
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    for (int i = 0; i < n; i++) {
        if (i >= 64 || !((sel >> i) & 1ull)) continue;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) continue;
        DevCtx *d = new DevCtx();
        d->id = i;
        (void)hipSetDevice(i);
        bool ok = true;
        ok = ok && hipStreamCreateWithFlags(&d->s_in, hipStreamNonBlocking) == hipSuccess;
        ok = ok && hipStreamCreateWithFlags(&d->s_out, hipStreamNonBlocking) == hipSuccess;
        for (Lane &ln : d->lane) {
            ok = ok && hipStreamCreateWithFlags(&ln.s_k, hipStreamNonBlocking) == hipSuccess;
            for (Slot &sl : ln.slot) {
                ok = ok && hipEventCreateWithFlags(&sl.ev_in, hipEventDisableTiming) == hipSuccess;
                ok = ok && hipEventCreateWithFlags(&sl.ev_k, hipEventDisableTiming) == hipSuccess;
                ok = ok && hipEventCreateWithFlags(&sl.ev, hipEventDisableTiming) == hipSuccess;
                for (hipEvent_t &e : sl.ev_p)
                    ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            }
        }
        if (!ok) {
            delete d;
            continue;
        }
        g_devs.push_back(d);
    }
}

std::vector<DevCtx *> &devices() {
    std::call_once(g_once, init_devices);
    return g_devs;
}

int64_t steady_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// Pinned staging (up to NSLOT x 2 GiB host + HBM per device) is released after
// JFS_STAGING_IDLE_MS (default 15 s; 0 = keep forever) without a batch, so an
// idle FUSE daemon does not hold it.  jfs_release_staging() frees it at once.
int64_t staging_idle_ms() {
    static int64_t v = [] {
        const char *e = getenv("JFS_STAGING_IDLE_MS");
        return e ? (int64_t)atoll(e) : (int64_t)15000;
    }();
    return v;
}

void release_lane_staging(DevCtx *d, Lane &ln) {
    (void)hipSetDevice(d->id);  // janitor thread / explicit release: no caller device to keep
    ln.release_staging();
}

// At exit the janitor must not call into a HIP runtime that is being torn
// down: the handler raises g_exiting and then takes every lane lock once,
// which waits out a release already in progress.
void on_exit_handler() {
    g_exiting = true;
    for (DevCtx *d : g_devs)
        for (Lane &ln : d->lane) {
            std::lock_guard<std::mutex> lk(ln.mu);
        }
}

void start_janitor() {
    static std::once_flag once;
    if (staging_idle_ms() <= 0) return;
    std::call_once(once, [] {
        atexit(on_exit_handler);
        std::thread([] {
            while (!g_exiting) {
                std::this_thread::sleep_for(std::chrono::milliseconds(std::min<int64_t>(1000, staging_idle_ms())));
                for (DevCtx *d : g_devs) {
                    if (steady_ms() - d->last_use_ms.load() < staging_idle_ms()) continue;
                    for (Lane &ln : d->lane) {
                        std::unique_lock<std::mutex> lk(ln.mu, std::try_to_lock);
                        if (!lk.owns_lock() || g_exiting) continue;
                        if (ln.holds_staging()) release_lane_staging(d, ln);
                    }
                }
            }
        }).detach();
    });
}

// crc32.Update(crc, crc32c, p[0:n]) on the host (pkg/object/checksum.go:30-45):
// table-driven, for the few hundred header bytes of an envelope and the
// "none" codec; block payloads are summed by crc32c.hip
uint32_t host_crc32c(uint32_t crc, const uint8_t *p, int64_t n) {
    static uint32_t tab[256];
    static std::once_flag once;
    std::call_once(once, [] {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ ((c & 1u) ? 0x82F63B78u : 0u);
            tab[i] = c;
        }
    });
    crc = ~crc;
    for (int64_t i = 0; i < n; i++) crc = tab[(crc ^ p[i]) & 255u] ^ (crc >> 8);
    return ~crc;
}

enum Dir { COMPRESS = 0, DECOMPRESS = 1 };
constexpr int COMPRESS_DIR = COMPRESS, DECOMPRESS_DIR = DECOMPRESS;

// Per-block result conversion from the kernel's raw value to the C-ABI value.
// DataDog/zstd v1.5.6 decompressSizeHint: the first frame's content size if
// known and non-zero, else max(50*len(src), 1e6); capped at that bound.
int64_t zstd_size_hint(const uint8_t *src, int64_t n) {
    int64_t upper = std::max<int64_t>(50 * n, 1000000);
    int64_t hint = upper;
    if (n >= 5 && src[0] == 0x28 && src[1] == 0xB5 && src[2] == 0x2F && src[3] == 0xFD) {
        int fhd = src[4];
        int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, did = fhd & 3;
        int64_t p = 5 + (single ? 0 : 1) + (did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4);
        int fs = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (fs && p + fs <= n && !(fhd & 8)) {
            uint64_t v = 0;
            for (int i = 0; i < fs; i++) v |= (uint64_t)src[p + i] << (8 * i);
            if (fs == 2) v += 256;
            if (v > 0 && v < (uint64_t)INT64_MAX) hint = (int64_t)v;
        }
    }
    return std::min(hint, upper);
}

int64_t finish_result(int algo, int dir, int32_t raw) {
    if (algo == JFS_ALGO_LZ4) {
        if (dir == COMPRESS) return raw > 0 ? raw : JFS_ERR_COMPRESS_FAIL;
        return raw;  // LZ4_decompress_safe value, passed through like lz4.DecompressSafe
    }
    if (algo == JFS_ALGO_ZSTD) {
        if (raw >= 0) return raw;
        if (dir == COMPRESS) return raw == -2 ? JFS_ERR_SHORT_BUFFER : JFS_ERR_COMPRESS_FAIL;
        if (raw == -2) return JFS_ERR_SHORT_BUFFER;
        return JFS_ERR_CORRUPT;
    }
    return JFS_ERR_INVALID;
}

// Staged output capacity of one block (what the kernel may write).
int64_t staged_cap(int algo, int dir, const jfs_iov &v) {
    int64_t cap = v.dst_cap;
    // LZ4 compress: the kernel never writes at/after cap; stage at most the bound
    if (algo == JFS_ALGO_LZ4 && dir == COMPRESS) cap = std::min<int64_t>(cap, v.src_len + v.src_len / 255 + 16);
    // Zstd decompress with cap(dst) < DataDog's size hint: DataDog decodes into
    // a buffer of its own, so compress.go:99-101 answers "buffer too short"
    // unless the frames decode to nothing ((0, nil)) or are corrupt (their own
    // error).  Decoding into zero bytes of staging tells those three apart
    // without staging a size the caller cannot hold.
    if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS && cap < zstd_size_hint(v.src, v.src_len)) cap = 0;
    if (algo == JFS_ALGO_ZSTD && dir == COMPRESS) cap = std::min<int64_t>(cap, jfs_compress_bound(JFS_ALGO_ZSTD, v.src_len));
    // the kernels take int32 capacities (jfs_dev_block)
    return std::min<int64_t>(std::max<int64_t>(cap, 0), INT32_MAX);
}

// HBM/pinned bytes one block occupies in a chunk
int64_t staged_bytes(int algo, int dir, const jfs_iov &v) { return align16(v.src_len) + align16(staged_cap(algo, dir, v)); }

// Host staging chunk (input + output bytes per pipeline stage); default 2 GiB,
// JFS_HOST_CHUNK_MB overrides.  The decode kernel needs many blocks in flight
// (one workgroup per block), so chunks stay large.
int64_t chunk_limit() {
    static int64_t v = [] {
        const char *e = getenv("JFS_HOST_CHUNK_MB");
        long long mb = e ? atoll(e) : 2048;
        return (int64_t)std::max(mb, 16ll) << 20;
    }();
    return v;
}

// Decode chunk ramp (run_batch): the number of small first chunks (32, 64,
// 128, then 128 blocks); JFS_HOST_RAMP overrides (0 = off).
int host_ramp_len() {
    static int v = [] {
        const char *e = getenv("JFS_HOST_RAMP");
        return e ? std::min(8, std::max(0, atoi(e))) : 3;  // 32 << k stays well inside int
    }();
    return v;
}
bool host_ramp() { return host_ramp_len() > 0; }

// LZ4 compress chunks: the serial-parse encoder holds 8 blocks per CU and a
// launch lasts one block's parse (~0.5 s) whatever its size, so a 2 GiB chunk
// (256 blocks at ~8 MiB staged each) fills an eighth of the GPU; 4 GiB chunks
// (512 blocks) with two chunk kernels side by side fill half of it.  The
// same holds for Zstd compress (one frame's serial parse, ~0.7 s at 4 MiB):
// a mixed 64 KiB-4 MiB batch in 1 GiB chunks paid its longest chain per chunk.
// JFS_HOST_CHUNK_MB_LZ4C overrides.
int64_t chunk_limit_lz4c() {
    static int64_t v = [] {
        const char *e = getenv("JFS_HOST_CHUNK_MB_LZ4C");
        long long mb = e ? atoll(e) : 4096;
        return (int64_t)std::max(mb, 16ll) << 20;
    }();
    return v;
}

// Batches of at most this many LZ4 decode blocks take the small-batch path
// (lz4_split.hip: every block spread over the whole GPU) instead of one
// workgroup per block; JFS_LZ4_SPLIT_MAX overrides (0 = never).
int split_max() {
    static int v = [] {
        const char *e = getenv("JFS_LZ4_SPLIT_MAX");
        return e ? std::max(0, atoi(e)) : 128;
    }();
    return v;
}

// memcpy jobs spread over host threads (pageable <-> pinned is CPU-bound)
struct CopyJob {
    uint8_t *dst;
    const uint8_t *src;
    int64_t n;
};
// One process-wide pool of copy threads shared by every lane of every device:
// concurrent batches (two lanes per GPU, up to eight GPUs) interleave their
// pieces instead of each spawning its own 16 threads, which oversubscribed the
// CPU quota (a 38 MiB stage-in took 65 ms next to another lane's copy-out).
// Size: JFS_COPY_THREADS, default min(16, CPUs this process may run on).
class CopyPool {
   public:
    static CopyPool &get() {
        static CopyPool *p = new CopyPool();  // never destroyed: workers outlive static dtors
        return *p;
    }
    int threads() const { return nthr_; }
    void run(std::vector<CopyJob> &pc) {
        Task t;
        t.pc = pc.data();
        t.n = pc.size();
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back(&t);
        }
        cv_.notify_all();
        work(t);  // the caller copies too
        std::unique_lock<std::mutex> lk(mu_);
        q_.erase(std::find(q_.begin(), q_.end(), &t));  // no worker picks it up any more
        done_cv_.wait(lk, [&] { return t.done.load() == t.n && t.active == 0; });
    }

   private:
    struct Task {
        CopyJob *pc = nullptr;
        size_t n = 0;
        std::atomic<size_t> next{0}, done{0};
        int active = 0;  // workers inside work(*this) (guarded by mu_)
    };
    std::mutex mu_;
    std::condition_variable cv_, done_cv_;
    std::deque<Task *> q_;
    int nthr_ = 1;

    static int cpu_share() {
        cpu_set_t set;
        CPU_ZERO(&set);
        if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, CPU_COUNT(&set));
        return (int)std::max(1u, std::thread::hardware_concurrency());
    }
    CopyPool() {
        const char *e = getenv("JFS_COPY_THREADS");
        nthr_ = e ? std::max(1, atoi(e)) : std::min(16, cpu_share());
        for (int i = 1; i < nthr_; i++) std::thread([this] { loop(); }).detach();
    }
    static void work(Task &t) {
        for (size_t i; (i = t.next.fetch_add(1)) < t.n;) {
            memcpy(t.pc[i].dst, t.pc[i].src, (size_t)t.pc[i].n);
            t.done.fetch_add(1);
        }
    }
    void loop() {
        for (;;) {
            Task *t = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] {
                    for (Task *x : q_)
                        if (x->next.load() < x->n) return true;
                    return false;
                });
                for (Task *x : q_)  // the oldest task with pieces left
                    if (x->next.load() < x->n) { t = x; break; }
                if (t) t->active++;
            }
            if (!t) continue;
            work(*t);
            {
                std::lock_guard<std::mutex> lk(mu_);
                if (--t->active == 0) done_cv_.notify_all();
            }
        }
    }
};

void par_copy(std::vector<CopyJob> &jobs) {
    int64_t total = 0;
    for (const CopyJob &j : jobs) total += j.n;
    CopyPool &pool = CopyPool::get();
    if (total < (16ll << 20) || pool.threads() == 1) {
        for (const CopyJob &j : jobs) memcpy(j.dst, j.src, (size_t)j.n);
        return;
    }
    // cut into <= 4 MiB pieces, handed out one at a time
    constexpr int64_t PIECE = 4ll << 20;
    std::vector<CopyJob> pc;
    for (const CopyJob &j : jobs)
        for (int64_t o = 0; o < j.n; o += PIECE) pc.push_back({j.dst + o, j.src + o, std::min(PIECE, j.n - o)});
    pool.run(pc);
}

// LZ4 encode batches of at most this many blocks take the segment-parallel
// parse (lz4_encode.hip, lz4_eseg): latency of a few segment parses instead of
// one whole-block parse per wave
int eseg_max() {
    static int v = [] {
        const char *e = getenv("JFS_LZ4E_SEG_MAX");
        return e ? atoi(e) : 256;
    }();
    return v;
}

int launch_kernel(int algo, int dir, const jfs_dev_block *d_desc, int nblk, int32_t *d_ret, hipStream_t st) {
    if (algo == JFS_ALGO_LZ4 && dir == DECOMPRESS) return jfs_launch_lz4_decode(d_desc, nblk, d_ret, st);
    if (algo == JFS_ALGO_LZ4 && dir == COMPRESS) return jfs_launch_lz4_encode(d_desc, nblk, d_ret, st);
    if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS) return jfs_launch_zstd_decode(d_desc, nblk, d_ret, nullptr, st);
    if (algo == JFS_ALGO_ZSTD && dir == COMPRESS) return jfs_launch_zstd_encode(d_desc, nblk, d_ret, st);
    return -1;
}

// Object encryption around the codec (pkg/object/encrypt.go
// dataEncryptor, installed after compression on PUT and before decompression
// on GET, cmd/format.go:289-302).  Arrays are parallel to the iov run_batch
// gets (whose src/src_len/dst_cap are the staged payload and capacity); orig
// holds the caller's buffers, which receive the envelope (seal) or the
// plaintext block (open).
struct Aead {
    int cipher;
    bool seal;
    const jfs_iov *orig;
    const uint8_t *const *key;    // data key per block
    const uint8_t *const *nonce;  // 12-byte nonce per block
    const jfs_seal_param *sp;     // seal: wrapped key per block
    const int64_t *hdr;           // seal: header bytes per block
    Aead at(int64_t h) const {
        Aead a = *this;
        a.orig += h;
        a.key += h;
        a.nonce += h;
        if (a.sp) a.sp += h;
        if (a.hdr) a.hdr += h;
        return a;
    }
};

// Run blocks [0,nblk) of iov on one device through one lane (the caller holds
// ln.mu); returns when every result is in out[].  Blocks that the C-ABI
// answers without a kernel (empty input, noOp) are handled by the caller.  The
// batch is cut into chunks pipelined over the lane's NSLOT (stream, pinned,
// HBM) slots: host copy-in of chunk k (threads) | H2D k+1, kernel k, D2H k-1
// (streams) | host copy-out of chunk k-NSLOT.  A chunk holds at most
// chunk_limit() staging bytes; the lane's kernels run in chunk order, so a
// batch is not cut finer than that (a decode kernel over fewer blocks than
// CUs lasts about one block's latency whatever its size).
// max_chunk_blocks (> 0) also caps a chunk's block count; on_chunk (optional)
// is called with [s, e) as soon as those blocks' results and outputs are final
// (the coalescer releases their callers there, before later chunks finish).
int64_t run_batch(DevCtx *dev, Lane &ln, int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out,
                  const Aead *ae = nullptr, uint32_t *crc_out = nullptr, int max_chunk_blocks = 0,
                  const std::function<void(int, int)> *on_chunk = nullptr, uint8_t *const *csum_out = nullptr) {
    if (nblk <= 0) return JFS_OK;
    DevGuard guard;
    (void)hipSetDevice(dev->id);
    dev->last_use_ms = steady_ms();
    ln.kind.store(algo * 2 + dir, std::memory_order_relaxed);
    dev->batches.fetch_add(1, std::memory_order_relaxed);
    dev->blocks.fetch_add((uint64_t)nblk, std::memory_order_relaxed);
    if (OpStats *st = op_stats(algo, dir)) st->batches.fetch_add(1, std::memory_order_relaxed);
    start_janitor();
    struct Touch {  // the idle clock starts when the batch ends
        DevCtx *d;
        ~Touch() { d->last_use_ms = steady_ms(); }
    } touch{dev};
    // Chunk kernels alternate between this lane's kernel stream and the other
    // lane's: an encode launch lasts one block's latency (~0.5 s) whatever its
    // size, so two chunks' kernels must run side by side (a device has only
    // two kernel streams: see Lane).
    Lane &other = dev->lane[(&ln - dev->lane + 1) % NLANE];
    auto kstream = [&](int chunk) { return (chunk & 1) ? other.s_k : ln.s_k; };
    std::vector<int64_t> cap(nblk), in_off(nblk), out_off(nblk);
    struct Chunk {
        int s, e, slot;
        int64_t tin, tout;
        hipStream_t ks;  // its kernel stream
    };
    std::vector<Chunk> ch;
    {
        const int64_t limit =
            (algo == JFS_ALGO_LZ4 || algo == JFS_ALGO_ZSTD) && dir == COMPRESS && !ae ? chunk_limit_lz4c() : chunk_limit();
        // Decode ramp: the first output cannot leave before chunk 0's H2D and
        // kernel are done, and the one-workgroup-per-block kernels take a
        // block's whole latency (~20 ms) whatever the chunk size; so a long
        // decode starts with chunks of 32, 64 and 128 blocks (the small-batch
        // kernels) that put the D2H stream to work while the first full chunk
        // is staged and decoded, and ends with a chunk of at most 128 blocks
        // so that little copy-out is left after the last D2H.  Measured on
        // 2,048 x 4 MiB LZ4 (scripts/hostpath.py): no ramp 34.9-36.5 GiB/s,
        // 3 ramp chunks 39.7-40.0, 5: 37.5, 7: 36.5.
        int64_t total = 0;
        for (int i = 0; i < nblk; i++) total += staged_bytes(algo, dir, iov[i]);
        const bool ramp = dir == DECOMPRESS && !ae && max_chunk_blocks <= 0 && total > 2 * limit && host_ramp();
        int s = 0;
        while (s < nblk) {
            Chunk c{s, s, (int)(ch.size() % NSLOT), 0, 0, kstream((int)ch.size())};
            const int k = (int)ch.size();
#ifndef JFS_HOST_FIRST_BIG
#define JFS_HOST_FIRST_BIG 192  // blocks in the first full chunk after the ramp (0: no cap)
#endif
            // (the first full chunk's H2D and one-block kernel latency are on
            // the critical path: a smaller one reaches the D2H stream sooner)
            int cap_blocks = ramp && k < host_ramp_len() ? std::min(32 << k, 128) : max_chunk_blocks;
            if (JFS_HOST_FIRST_BIG > 0 && ramp && k == host_ramp_len()) cap_blocks = JFS_HOST_FIRST_BIG;
            while (c.e < nblk) {
                const int64_t ci = ae ? iov[c.e].dst_cap : staged_cap(algo, dir, iov[c.e]);
                const int64_t ib = align16(iov[c.e].src_len), ob = align16(ci);  // = staged_bytes()
                if (c.e > s && (c.tin + c.tout + ib + ob > limit || (cap_blocks > 0 && c.e - s >= cap_blocks)))
                    break;
                cap[c.e] = ci;
                in_off[c.e] = c.tin;
                out_off[c.e] = c.tout;
                c.tin += ib;
                c.tout += ob;
                c.e++;
            }
            ch.push_back(c);
            s = c.e;
        }
        if (ramp && ch.size() > 4 && ch.back().e - ch.back().s > 128) {  // ramp down: split the last chunk
            Chunk &l = ch.back();
            const int mid = l.e - 128;
            Chunk t{mid, l.e, (int)(ch.size() % NSLOT), 0, 0, kstream((int)ch.size())};
            l.e = mid;
            l.tin = l.tout = 0;
            for (int i = l.s; i < l.e; i++) {
                in_off[i] = l.tin;
                out_off[i] = l.tout;
                l.tin += align16(iov[i].src_len);
                l.tout += align16(cap[i]);
            }
            for (int i = t.s; i < t.e; i++) {
                in_off[i] = t.tin;
                out_off[i] = t.tout;
                t.tin += align16(iov[i].src_len);
                t.tout += align16(cap[i]);
            }
            ch.push_back(t);
        }
    }
    // Zstd decode: the per-input scratch plan (ZInfo) rides in the chunk
    const bool zplan = algo == JFS_ALGO_ZSTD && dir == DECOMPRESS && !ae;
    const int64_t zib = zplan ? (int64_t)jfs_zstd_info_bytes() : 0;
    // aead extras per block: descriptor, second result, 64 bytes of key (32) + nonce (12)
    const int64_t aeb = ae ? (int64_t)sizeof(jfs_aead_block) + 4 + 64 : 0;
    // output pieces of a chunk (see NPIECE): large chunks in block ranges
    // [piece_b(c, p), piece_b(c, p + 1)); a one-block chunk (a lone cache
    // miss) in byte ranges of the output area (byte_npiece), so that the
    // copy-out of one piece overlaps the D2H of the next; other small chunks
    // (the coalescer's 16-block ones) stay whole: a piece's host copy is a
    // thread-pool round of its own.  piece_o(c, p) = the piece's first byte.
    auto byte_pieces = [&](const Chunk &c) { return byte_npiece() > 1 && c.e - c.s == 1; };
    // input staging pieces: block ranges of large chunks only
    auto in_npiece = [&](const Chunk &c) { return c.e - c.s >= 64 ? std::min(NPIECE, c.e - c.s) : 1; };
    auto in_piece_b = [&](const Chunk &c, int p) {
        return c.s + (int)((int64_t)(c.e - c.s) * p / in_npiece(c));
    };
    auto npiece = [&](const Chunk &c) {
        return c.e - c.s >= 64 ? std::min(NPIECE, c.e - c.s) : byte_pieces(c) ? byte_npiece() : 1;
    };
    auto piece_b = [&](const Chunk &c, int p) {
        return byte_pieces(c) ? c.s : c.s + (int)((int64_t)(c.e - c.s) * p / npiece(c));
    };
    auto piece_o = [&](const Chunk &c, int p) -> int64_t {
        const int np = npiece(c);
        if (p >= np) return c.tout;
        if (byte_pieces(c)) return (c.tout * p / np) & ~(int64_t)15;
        const int b = piece_b(c, p);
        return b < c.e ? out_off[b] : c.tout;
    };
    auto layout = [&](const Chunk &c, uint8_t *base, uint8_t **in, uint8_t **outp, jfs_dev_block **desc, int32_t **ret,
                      uint8_t **zinfo) {
        const int64_t desc_bytes = align16((int64_t)(c.e - c.s) * (int64_t)sizeof(jfs_dev_block));
        const int64_t ret_bytes = align16((int64_t)(c.e - c.s) * 4);
        *in = base;
        *outp = base + c.tin;
        *desc = (jfs_dev_block *)(base + c.tin + c.tout);
        *ret = (int32_t *)(base + c.tin + c.tout + desc_bytes);
        *zinfo = base + c.tin + c.tout + desc_bytes + ret_bytes;
    };
    // the aead area follows the Zstd plan area: descriptors, results, key+nonce slots
    auto aead_layout = [&](const Chunk &c, uint8_t *base, jfs_aead_block **ad, int32_t **ret2, uint8_t **kn) {
        const int64_t nb = c.e - c.s;
        uint8_t *p = base + c.tin + c.tout + align16(nb * (int64_t)sizeof(jfs_dev_block)) + align16(nb * 4) +
                     align16(nb * zib);
        *ad = (jfs_aead_block *)p;
        p += align16(nb * (int64_t)sizeof(jfs_aead_block));
        *ret2 = (int32_t *)p;
        p += align16(nb * 4);
        *kn = p;
    };
    auto aead_bytes = [&](int64_t nb) {
        return ae ? align16(nb * (int64_t)sizeof(jfs_aead_block)) + align16(nb * 4) + align16(nb * 64) : 0;
    };
    // PUT-payload checksums: descriptors, seeds, results (after the aead area)
    auto crc_layout = [&](const Chunk &c, uint8_t *base, jfs_dev_block **cd, uint32_t **seed, uint32_t **crc) {
        const int64_t nb = c.e - c.s;
        uint8_t *p = base + c.tin + c.tout + align16(nb * (int64_t)sizeof(jfs_dev_block)) + align16(nb * 4) +
                     align16(nb * zib) + aead_bytes(nb);
        *cd = (jfs_dev_block *)p;
        p += align16(nb * (int64_t)sizeof(jfs_dev_block));
        *seed = (uint32_t *)p;
        p += align16(nb * 4);
        *crc = (uint32_t *)p;
    };
    // decode-side disk-cache checksums (csum_out): descriptors, then every
    // block's ((cap-1)/32 KiB+1)*4 checksum bytes (after the crc area)
    const bool want_csum = csum_out && dir == DECOMPRESS && !ae;
    auto csum_words = [&](int i) { return cap[i] > 0 ? (cap[i] - 1) / CSUM_SEG + 1 : 1; };
    auto crc_bytes = [&](int64_t nb) {
        return crc_out ? align16(nb * (int64_t)sizeof(jfs_dev_block)) + 2 * align16(nb * 4) : 0;
    };
    auto csum_layout = [&](const Chunk &c, uint8_t *base, jfs_dev_block **cd, uint8_t **area) {
        const int64_t nb = c.e - c.s;
        uint8_t *p = base + c.tin + c.tout + align16(nb * (int64_t)sizeof(jfs_dev_block)) + align16(nb * 4) +
                     align16(nb * zib) + aead_bytes(nb) + crc_bytes(nb);
        *cd = (jfs_dev_block *)p;
        *area = p + align16(nb * (int64_t)sizeof(jfs_dev_block));
    };
    auto csum_area_bytes = [&](const Chunk &c) {
        int64_t t = 0;
        for (int i = c.s; i < c.e; i++) t += align16(4 * csum_words(i));
        return t;
    };
    auto chunk_bytes = [&](const Chunk &c) {
        const int64_t nb = c.e - c.s;
        return c.tin + c.tout + align16(nb * (int64_t)sizeof(jfs_dev_block)) + align16(nb * 4) + align16(nb * zib) +
               aead_bytes(nb) + crc_bytes(nb) +
               (want_csum ? align16(nb * (int64_t)sizeof(jfs_dev_block)) + csum_area_bytes(c) : 0);
    };
    // stage the checksum descriptors: the decoded output is the data, the
    // checksum bytes go to the chunk's checksum area
    auto stage_csum = [&](const Chunk &c, Slot &sl, uint8_t *d_out) -> int64_t {
        if (!want_csum) return JFS_OK;
        const int n = c.e - c.s;
        jfs_dev_block *h_cd, *d_cd;
        uint8_t *h_area, *d_area;
        csum_layout(c, sl.h, &h_cd, &h_area);
        csum_layout(c, sl.d, &d_cd, &d_area);
        int64_t o = 0;
        for (int k = 0; k < n; k++) {
            const int i = c.s + k;
            h_cd[k] = jfs_dev_block{d_out + out_off[i], d_area + o, 0, (int32_t)(4 * csum_words(i))};
            o += align16(4 * csum_words(i));
        }
        return hipMemcpyAsync(d_cd, h_cd, (size_t)n * sizeof(jfs_dev_block), hipMemcpyHostToDevice, dev->s_in) ==
                       hipSuccess
                   ? JFS_OK
                   : JFS_ERR_HIP;
    };
    auto run_csum = [&](const Chunk &c, Slot &sl, const int32_t *d_lens) -> int64_t {
        if (!want_csum) return JFS_OK;
        jfs_dev_block *d_cd;
        uint8_t *d_area;
        csum_layout(c, sl.d, &d_cd, &d_area);
        return jfs_launch_crc32c_segs_lens(d_cd, c.e - c.s, CSUM_SEG, d_lens, c.ks) == 0 ? JFS_OK : JFS_ERR_HIP;
    };
    auto fetch_csum = [&](const Chunk &c, Slot &sl) -> int64_t {
        if (!want_csum) return JFS_OK;
        jfs_dev_block *h_cd, *d_cd;
        uint8_t *h_area, *d_area;
        csum_layout(c, sl.h, &h_cd, &h_area);
        csum_layout(c, sl.d, &d_cd, &d_area);
        return hipMemcpyAsync(h_area, d_area, (size_t)csum_area_bytes(c), hipMemcpyDeviceToHost, dev->s_out) ==
                       hipSuccess
                   ? JFS_OK
                   : JFS_ERR_HIP;
    };
    // stage the checksum descriptors (payload = the codec's output area) and
    // queue their H2D on s_in; seeds: the envelope header's CRC for a seal
    auto stage_crc = [&](const Chunk &c, Slot &sl, uint8_t *d_out) -> int64_t {
        if (!crc_out) return JFS_OK;
        const int n = c.e - c.s;
        jfs_dev_block *h_cd, *d_cd;
        uint32_t *h_seed, *d_seed, *h_crc, *d_crc;
        crc_layout(c, sl.h, &h_cd, &h_seed, &h_crc);
        crc_layout(c, sl.d, &d_cd, &d_seed, &d_crc);
        for (int k = 0; k < n; k++) {
            const int i = c.s + k;
            h_cd[k] = jfs_dev_block{d_out + out_off[i], nullptr, 0, 0};
            h_seed[k] = 0;
            if (ae && ae->seal) {
                const jfs_seal_param &p = ae->sp[i];
                const uint8_t h3[3] = {(uint8_t)(p.wrapped_len >> 8), (uint8_t)(p.wrapped_len & 0xFF), 12};
                uint32_t v = host_crc32c(0, h3, 3);
                v = host_crc32c(v, p.wrapped, p.wrapped_len);
                h_seed[k] = host_crc32c(v, ae->nonce[i], 12);
            }
        }
        const size_t bytes = (size_t)(align16((int64_t)n * (int64_t)sizeof(jfs_dev_block)) + align16((int64_t)n * 4));
        return hipMemcpyAsync(d_cd, h_cd, bytes, hipMemcpyHostToDevice, dev->s_in) == hipSuccess ? JFS_OK : JFS_ERR_HIP;
    };
    // after the kernels: the checksum launch (lengths from the device) and its D2H
    auto run_crc = [&](const Chunk &c, Slot &sl, const int32_t *d_lens) -> int64_t {
        if (!crc_out) return JFS_OK;
        const int n = c.e - c.s;
        jfs_dev_block *d_cd;
        uint32_t *d_seed, *d_crc;
        crc_layout(c, sl.d, &d_cd, &d_seed, &d_crc);
        return jfs_launch_crc32c_lens(d_cd, n, d_lens, d_seed, d_crc, c.ks) == 0 ? JFS_OK : JFS_ERR_HIP;
    };
    auto fetch_crc = [&](const Chunk &c, Slot &sl) -> int64_t {
        if (!crc_out) return JFS_OK;
        jfs_dev_block *h_cd, *d_cd;
        uint32_t *h_seed, *d_seed, *h_crc, *d_crc;
        crc_layout(c, sl.h, &h_cd, &h_seed, &h_crc);
        crc_layout(c, sl.d, &d_cd, &d_seed, &d_crc);
        return hipMemcpyAsync(h_crc, d_crc, (size_t)(c.e - c.s) * 4, hipMemcpyDeviceToHost, dev->s_out) == hipSuccess
                   ? JFS_OK
                   : JFS_ERR_HIP;
    };
    (void)aeb;
    // compress -> seal, or open -> decompress (the staged inputs and the
    // LZ4 encode of a staged chunk: segment-parallel for small batches
    auto lz4_encode = [&](Slot &sl, const jfs_dev_block *h_desc, const jfs_dev_block *d_desc, int n, int32_t *d_ret,
                          hipStream_t ks) -> int64_t {
        if (n > eseg_max()) return jfs_launch_lz4_encode(d_desc, n, d_ret, ks) == 0 ? JFS_OK : JFS_ERR_HIP;
        std::vector<int32_t> lens(n);
        for (int k = 0; k < n; k++) lens[k] = h_desc[k].src_len;
        if (!sl.ensure_split(jfs_lz4_eseg_scratch_bytes(n, lens.data()))) return JFS_ERR_NO_MEMORY;
        return jfs_launch_lz4_encode_seg(d_desc, n, lens.data(), d_ret, sl.sp, sl.sp_cap, ks) == 0 ? JFS_OK
                                                                                                   : JFS_ERR_HIP;
    };
    // codec descriptors are already in place; run on the lane's kernel stream)
    auto launch_aead = [&](const Chunk &c, Slot &sl, uint8_t *h_in, uint8_t *h_out, jfs_dev_block *h_desc,
                           int32_t *h_ret, uint8_t *d_in, uint8_t *d_out, jfs_dev_block *d_desc,
                           int32_t *d_ret) -> int64_t {
        const int n = c.e - c.s;
        jfs_aead_block *h_ad, *d_ad;
        int32_t *h_r2, *d_r2;
        uint8_t *h_kn, *d_kn;
        aead_layout(c, sl.h, &h_ad, &h_r2, &h_kn);
        aead_layout(c, sl.d, &d_ad, &d_r2, &d_kn);
        const int klen = jfs_cipher_key_size(ae->cipher);
        for (int k = 0; k < n; k++) {
            const int i = c.s + k;
            memcpy(h_kn + 64 * k, ae->key[i], (size_t)klen);
            memcpy(h_kn + 64 * k + 32, ae->nonce[i], 12);
            jfs_aead_block &a = h_ad[k];
            a.key = d_kn + 64 * k;
            a.nonce = d_kn + 64 * k + 32;
            if (ae->seal) {
                // the codec writes the payload area; the seal runs in place over it
                h_desc[k].dst_cap = (int32_t)(cap[i] - 16);
                a.src = algo == JFS_ALGO_NONE ? d_in + in_off[i] : d_out + out_off[i];
                a.dst = d_out + out_off[i];
                a.src_len = (int32_t)iov[i].src_len;
                a.dst_cap = (int32_t)cap[i];
            } else {
                // open in place over the staged payload (into the output for "none"),
                // then the codec reads the plaintext: the payload minus its tag
                h_desc[k].src_len = (int32_t)std::max<int64_t>(iov[i].src_len - 16, 0);
                a.src = d_in + in_off[i];
                a.dst = algo == JFS_ALGO_NONE ? d_out + out_off[i] : d_in + in_off[i];
                a.src_len = (int32_t)iov[i].src_len;
                a.dst_cap = algo == JFS_ALGO_NONE ? (int32_t)cap[i] : (int32_t)iov[i].src_len;
            }
        }
        const int64_t ab = aead_bytes(n);
        if (hipMemcpyAsync(d_in, h_in, (size_t)c.tin, hipMemcpyHostToDevice, dev->s_in) != hipSuccess) return JFS_ERR_HIP;
        if (hipMemcpyAsync(d_desc, h_desc, (size_t)n * sizeof(jfs_dev_block), hipMemcpyHostToDevice, dev->s_in) !=
            hipSuccess)
            return JFS_ERR_HIP;
        if (hipMemcpyAsync(d_ad, h_ad, (size_t)ab, hipMemcpyHostToDevice, dev->s_in) != hipSuccess) return JFS_ERR_HIP;
        if (stage_crc(c, sl, d_out) != JFS_OK) return JFS_ERR_HIP;
        if (hipEventRecord(sl.ev_in, dev->s_in) != hipSuccess) return JFS_ERR_HIP;
        if (hipStreamWaitEvent(c.ks, sl.ev_in, 0) != hipSuccess) return JFS_ERR_HIP;
        int lk = 0;
        if (ae->seal) {
            if (algo == JFS_ALGO_LZ4) {
                const int64_t r = lz4_encode(sl, h_desc, d_desc, n, d_ret, c.ks);
                if (r == JFS_ERR_NO_MEMORY) return r;
                lk = r == JFS_OK ? 0 : -1;
            } else if (algo != JFS_ALGO_NONE) {
                lk = launch_kernel(algo, COMPRESS, d_desc, n, d_ret, c.ks);
            }
            if (lk == 0)
                lk = jfs_launch_aead(ae->cipher, d_ad, n, 0, d_r2, algo != JFS_ALGO_NONE ? d_ret : nullptr, c.ks);
        } else {
            lk = jfs_launch_aead(ae->cipher, d_ad, n, 1, d_r2, nullptr, c.ks);
            if (lk == 0 && algo == JFS_ALGO_LZ4) {
                if (n <= split_max()) {
                    std::vector<int32_t> lens(n), caps(n);
                    int64_t nseg = 0, max_cap = 0, norg = 0;
                    for (int k = 0; k < n; k++) {
                        lens[k] = h_desc[k].src_len;
                        caps[k] = h_desc[k].dst_cap;
                        nseg += (std::max(lens[k], 0) + JFS_LZ4_SPLIT_SEG - 1) / JFS_LZ4_SPLIT_SEG;
                        max_cap = std::max<int64_t>(max_cap, caps[k]);
                        norg += (std::max<int64_t>(caps[k], 0) + 3) & ~3ll;
                    }
                    if (!sl.ensure_split(jfs_lz4_split_scratch_bytes(n, lens.data(), caps.data())))
                        return JFS_ERR_NO_MEMORY;
                    lk = jfs_launch_lz4_split(d_desc, n, d_ret, sl.sp, nseg, max_cap, norg, c.ks);
                } else {
                    lk = jfs_launch_lz4_decode(d_desc, n, d_ret, c.ks);
                }
            } else if (lk == 0 && algo == JFS_ALGO_ZSTD) {
                // the host holds ciphertext only: the device API plans the scratch itself
                lk = jfs_launch_zstd_decode(d_desc, n, d_ret, nullptr, c.ks);
            }
        }
        if (lk != 0) return JFS_ERR_HIP;
        if (ae->seal && run_crc(c, sl, d_r2) != JFS_OK) return JFS_ERR_HIP;
        if (hipEventRecord(sl.ev_k, c.ks) != hipSuccess) return JFS_ERR_HIP;
        if (hipStreamWaitEvent(dev->s_out, sl.ev_k, 0) != hipSuccess) return JFS_ERR_HIP;
        if (hipMemcpyAsync(h_ret, d_ret, (size_t)n * 4, hipMemcpyDeviceToHost, dev->s_out) != hipSuccess)
            return JFS_ERR_HIP;
        if (hipMemcpyAsync(h_r2, d_r2, (size_t)n * 4, hipMemcpyDeviceToHost, dev->s_out) != hipSuccess)
            return JFS_ERR_HIP;
        if (ae->seal && fetch_crc(c, sl) != JFS_OK) return JFS_ERR_HIP;
        if (hipMemcpyAsync(h_out, d_out, (size_t)c.tout, hipMemcpyDeviceToHost, dev->s_out) != hipSuccess)
            return JFS_ERR_HIP;
        if (hipEventRecord(sl.ev, dev->s_out) != hipSuccess) return JFS_ERR_HIP;
        return JFS_OK;
    };
    auto launch = [&](const Chunk &c) -> int64_t {
        Slot &sl = ln.slot[c.slot];
        if (!sl.ensure(chunk_bytes(c))) return JFS_ERR_NO_MEMORY;
        uint8_t *h_in, *h_out, *d_in, *d_out, *h_zi, *d_zi;
        jfs_dev_block *h_desc, *d_desc;
        int32_t *h_ret, *d_ret;
        layout(c, sl.h, &h_in, &h_out, &h_desc, &h_ret, &h_zi);
        layout(c, sl.d, &d_in, &d_out, &d_desc, &d_ret, &d_zi);
        for (int i = c.s; i < c.e; i++) {
            const int k = i - c.s;
            h_desc[k].src = d_in + in_off[i];
            h_desc[k].dst = d_out + out_off[i];
            h_desc[k].src_len = (int32_t)iov[i].src_len;
            h_desc[k].dst_cap = (int32_t)std::min<int64_t>(cap[i], INT32_MAX);
        }
        const double t0 = host_trace() ? now_ms() : 0.0;
        // Stage the inputs in pieces (NPIECE), each piece's H2D issued as soon as
        // it is staged so that it overlaps the staging of the next (the
        // encrypted path stages everything first: launch_aead issues its H2D).
        for (int p = 0; p < in_npiece(c); p++) {
            const int b0 = in_piece_b(c, p), b1 = in_piece_b(c, p + 1);
            std::vector<CopyJob> jobs;
            for (int i = b0; i < b1; i++)
                if (iov[i].src_len > 0) jobs.push_back({h_in + in_off[i], iov[i].src, iov[i].src_len});
            par_copy(jobs);
            if (ae) continue;
            const int64_t o0 = in_off[b0], o1 = b1 < c.e ? in_off[b1] : c.tin;
            if (o1 > o0 && hipMemcpyAsync(d_in + o0, h_in + o0, (size_t)(o1 - o0), hipMemcpyHostToDevice, dev->s_in) !=
                               hipSuccess)
                return JFS_ERR_HIP;
        }
        if (host_trace())
            fprintf(stderr, "[jfs host] t=%.2f lane %d algo %d dir %d chunk %d-%d stage-in %.1f MiB %.2f ms\n",
                    now_ms(), (int)(&ln - dev->lane), algo, dir, c.s, c.e, c.tin / 1048576.0, now_ms() - t0);
        const int n = c.e - c.s;
        uint64_t ztot[6] = {0, 0, 0, 0, 0, 0};
        if (ae) return launch_aead(c, sl, h_in, h_out, h_desc, h_ret, d_in, d_out, d_desc, d_ret);
        if (algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_UNSUPPORTED;
        if (zplan) {  // plan the Zstd scratch from the staged inputs: no device round trip
            std::vector<const uint8_t *> srcs(n);
            std::vector<int32_t> lens(n), caps(n);
            for (int k = 0; k < n; k++) {
                srcs[k] = h_in + in_off[c.s + k];
                lens[k] = h_desc[k].src_len;
                caps[k] = h_desc[k].dst_cap;
            }
            jfs_zstd_plan_host(srcs.data(), lens.data(), caps.data(), n, h_zi, ztot);
            if (!sl.ensure_zstd(ztot)) return JFS_ERR_NO_MEMORY;
            if (jfs_zstd_split_ok(n, ztot) && !sl.ensure_split(jfs_zstd_split_bytes(n, ztot))) return JFS_ERR_NO_MEMORY;
        }
        if (hipMemcpyAsync(d_desc, h_desc, (size_t)n * sizeof(jfs_dev_block), hipMemcpyHostToDevice, dev->s_in) !=
            hipSuccess)
            return JFS_ERR_HIP;
        if (zplan && hipMemcpyAsync(d_zi, h_zi, (size_t)(n * zib), hipMemcpyHostToDevice, dev->s_in) != hipSuccess)
            return JFS_ERR_HIP;
        if (dir == COMPRESS && stage_crc(c, sl, d_out) != JFS_OK) return JFS_ERR_HIP;
        if (stage_csum(c, sl, d_out) != JFS_OK) return JFS_ERR_HIP;
        if (hipEventRecord(sl.ev_in, dev->s_in) != hipSuccess) return JFS_ERR_HIP;
        if (hipStreamWaitEvent(c.ks, sl.ev_in, 0) != hipSuccess) return JFS_ERR_HIP;
        int lk;
        if (zplan) {
            lk = jfs_launch_zstd_decode_planned(d_desc, n, d_ret, d_zi, sl.z_lit, sl.z_tabs, sl.z_items,
                                                jfs_zstd_split_ok(n, ztot) ? sl.sp : nullptr, ztot, c.ks);
        } else if (algo == JFS_ALGO_LZ4 && dir == DECOMPRESS && n <= split_max()) {
            std::vector<int32_t> lens(n), caps(n);
            int64_t nseg = 0, max_cap = 0, norg = 0;
            for (int k = 0; k < n; k++) {
                lens[k] = h_desc[k].src_len;
                caps[k] = h_desc[k].dst_cap;
                nseg += (std::max(lens[k], 0) + JFS_LZ4_SPLIT_SEG - 1) / JFS_LZ4_SPLIT_SEG;
                max_cap = std::max<int64_t>(max_cap, caps[k]);
                norg += (std::max<int64_t>(caps[k], 0) + 3) & ~3ll;
            }
            if (!sl.ensure_split(jfs_lz4_split_scratch_bytes(n, lens.data(), caps.data()))) return JFS_ERR_NO_MEMORY;
            lk = jfs_launch_lz4_split(d_desc, n, d_ret, sl.sp, nseg, max_cap, norg, c.ks);
        } else if (algo == JFS_ALGO_LZ4 && dir == COMPRESS) {
            const int64_t r = lz4_encode(sl, h_desc, d_desc, n, d_ret, c.ks);
            if (r == JFS_ERR_NO_MEMORY) return r;
            lk = r == JFS_OK ? 0 : -1;
        } else {
            lk = launch_kernel(algo, dir, d_desc, n, d_ret, c.ks);
        }
        if (lk != 0) return JFS_ERR_HIP;
        if (dir == COMPRESS && run_crc(c, sl, d_ret) != JFS_OK) return JFS_ERR_HIP;
        if (run_csum(c, sl, d_ret) != JFS_OK) return JFS_ERR_HIP;
        if (hipEventRecord(sl.ev_k, c.ks) != hipSuccess) return JFS_ERR_HIP;
        if (hipStreamWaitEvent(dev->s_out, sl.ev_k, 0) != hipSuccess) return JFS_ERR_HIP;
        if (hipMemcpyAsync(h_ret, d_ret, (size_t)n * 4, hipMemcpyDeviceToHost, dev->s_out) != hipSuccess)
            return JFS_ERR_HIP;
        if (dir == COMPRESS && fetch_crc(c, sl) != JFS_OK) return JFS_ERR_HIP;
        if (fetch_csum(c, sl) != JFS_OK) return JFS_ERR_HIP;
        for (int p = 0; p < npiece(c); p++) {  // output bytes [piece_o(c, p), piece_o(c, p + 1))
            const int64_t o0 = piece_o(c, p), o1 = piece_o(c, p + 1);
            if (o1 > o0 && hipMemcpyAsync(h_out + o0, d_out + o0, (size_t)(o1 - o0), hipMemcpyDeviceToHost,
                                          dev->s_out) != hipSuccess)
                return JFS_ERR_HIP;
            if (hipEventRecord(sl.ev_p[p], dev->s_out) != hipSuccess) return JFS_ERR_HIP;
        }
        if (hipEventRecord(sl.ev, dev->s_out) != hipSuccess) return JFS_ERR_HIP;
        return JFS_OK;
    };
    auto finish = [&](const Chunk &c) -> int64_t {
        Slot &sl = ln.slot[c.slot];
        const double t0 = host_trace() ? now_ms() : 0.0;
        // (results, CRCs and checksums land before the first output piece)
        if (hipEventSynchronize(ae ? sl.ev : sl.ev_p[0]) != hipSuccess) return JFS_ERR_HIP;
        const double t1 = host_trace() ? now_ms() : 0.0;
        uint8_t *h_in, *h_out, *h_zi;
        jfs_dev_block *h_desc;
        int32_t *h_ret;
        layout(c, sl.h, &h_in, &h_out, &h_desc, &h_ret, &h_zi);
        std::vector<CopyJob> jobs;
        if (ae) {
            jfs_aead_block *h_ad;
            int32_t *h_r2;
            uint8_t *h_kn;
            aead_layout(c, sl.h, &h_ad, &h_r2, &h_kn);
            for (int i = c.s; i < c.e; i++) {
                const int k = i - c.s;
                const jfs_iov &o = ae->orig[i];
                if (ae->seal) {
                    // encrypt.go:244-254: be16(len(wrapped)) | len(nonce) | wrapped | nonce | sealed
                    const int64_t rc = algo == JFS_ALGO_NONE ? iov[i].src_len : finish_result(algo, COMPRESS, h_ret[k]);
                    const int64_t hdr = ae->hdr[i];
                    if (rc < 0) {
                        out[i] = rc;
                    } else if (h_r2[k] != rc + 16) {
                        out[i] = JFS_ERR_HIP;
                    } else if (hdr + rc + 16 > o.dst_cap) {
                        out[i] = JFS_ERR_SHORT_BUFFER;
                    } else {
                        const jfs_seal_param &p = ae->sp[i];
                        o.dst[0] = (uint8_t)(p.wrapped_len >> 8);
                        o.dst[1] = (uint8_t)(p.wrapped_len & 0xFF);
                        o.dst[2] = 12;
                        if (p.wrapped_len > 0) memcpy(o.dst + 3, p.wrapped, (size_t)p.wrapped_len);
                        memcpy(o.dst + 3 + p.wrapped_len, ae->nonce[i], 12);
                        jobs.push_back({o.dst + hdr, h_out + out_off[i], rc + 16});
                        out[i] = hdr + rc + 16;
                    }
                } else {
                    // aead.Open first (encrypt.go:283), then the codec
                    const int64_t r = h_r2[k] < 0 ? JFS_ERR_AUTH
                                      : algo == JFS_ALGO_NONE ? (int64_t)h_r2[k]
                                                              : finish_result(algo, DECOMPRESS, h_ret[k]);
                    if (r > 0) jobs.push_back({o.dst, h_out + out_off[i], r});
                    out[i] = r;
                }
            }
        } else {
            for (int i = c.s; i < c.e; i++) out[i] = finish_result(algo, dir, h_ret[i - c.s]);
            for (int p = 0; p < npiece(c); p++) {  // each piece's copy-out as soon as it landed
                if (p > 0 && byte_pieces(c)) {  // (a piece of a lone block: spin, it lands within microseconds)
                    hipError_t q;
                    while ((q = hipEventQuery(sl.ev_p[p])) == hipErrorNotReady) {
                    }
                    if (q != hipSuccess) return JFS_ERR_HIP;
                } else if (p > 0 && hipEventSynchronize(sl.ev_p[p]) != hipSuccess) {
                    return JFS_ERR_HIP;
                }
                std::vector<CopyJob> pj;
                const int64_t p0 = piece_o(c, p), p1 = piece_o(c, p + 1);
                const int i0 = byte_pieces(c) ? c.s : piece_b(c, p), i1 = byte_pieces(c) ? c.e : piece_b(c, p + 1);
                for (int i = i0; i < i1; i++) {  // the part of block i's output inside the piece
                    if (out[i] <= 0) continue;
                    const int64_t lo = std::max(out_off[i], p0), hi = std::min(out_off[i] + out[i], p1);
                    if (hi > lo) pj.push_back({iov[i].dst + (lo - out_off[i]), h_out + lo, hi - lo});
                }
                par_copy(pj);
            }
        }
        if (crc_out) {
            jfs_dev_block *h_cd;
            uint32_t *h_seed, *h_crc;
            crc_layout(c, sl.h, &h_cd, &h_seed, &h_crc);
            for (int i = c.s; i < c.e; i++) crc_out[i] = out[i] >= 0 ? h_crc[i - c.s] : 0u;
        }
        if (want_csum) {
            jfs_dev_block *h_cd;
            uint8_t *h_area;
            csum_layout(c, sl.h, &h_cd, &h_area);
            int64_t o = 0;
            for (int i = c.s; i < c.e; i++) {
                if (csum_out[i] && out[i] >= 0) {
                    const int64_t nw = out[i] > 0 ? (out[i] - 1) / CSUM_SEG + 1 : 1;
                    jobs.push_back({csum_out[i], h_area + o, 4 * nw});
                }
                o += align16(4 * csum_words(i));
            }
        }
        par_copy(jobs);
        if (host_trace())
            fprintf(stderr, "[jfs host] t=%.2f chunk %d-%d wait %.2f ms copy-out %.1f MiB %.2f ms\n", now_ms(), c.s, c.e, t1 - t0,
                    c.tout / 1048576.0, now_ms() - t1);
        return JFS_OK;
    };
    const int nch = (int)ch.size();
    // Size every slot for all of its chunks (staging, LZ4 small-batch scratch)
    // before the first launch: growing a slot mid-batch frees the old buffer,
    // and hipFree waits for the whole device -- the batch's own chunks in
    // flight (64 ms of a 273 ms 1,024-block decode).  A size that cannot be
    // had is left to the chunk's own ensure(), which reports it.
    {
        int64_t need[NSLOT] = {}, need_sp[NSLOT] = {};
        for (const Chunk &c : ch) {
            need[c.slot] = std::max(need[c.slot], chunk_bytes(c));
            const int n = c.e - c.s;
            if (algo == JFS_ALGO_LZ4 && dir == DECOMPRESS && !ae && n <= split_max()) {
                std::vector<int32_t> lens(n), caps(n);
                for (int k = 0; k < n; k++) {
                    lens[k] = (int32_t)iov[c.s + k].src_len;
                    caps[k] = (int32_t)std::min<int64_t>(cap[c.s + k], INT32_MAX);
                }
                need_sp[c.slot] = std::max(need_sp[c.slot], jfs_lz4_split_scratch_bytes(n, lens.data(), caps.data()));
            }
        }
        for (int s = 0; s < NSLOT; s++) {
            if (need[s] > 0) (void)ln.slot[s].ensure(need[s]);
            if (need_sp[s] > 0) (void)ln.slot[s].ensure_split(need_sp[s]);
        }
    }
    int64_t rc = JFS_OK;
    int done = 0;  // chunks [0, done) finished
    auto finish_next = [&]() -> int64_t {
        const Chunk &c = ch[done++];
        const int64_t r = finish(c);
        if (r == JFS_OK && on_chunk) (*on_chunk)(c.s, c.e);
        return r;
    };
    for (int k = 0; k < nch && rc == JFS_OK; k++) {
        if (k >= NSLOT) rc = finish_next();
        if (rc == JFS_OK) rc = launch(ch[k]);
    }
    while (done < nch && rc == JFS_OK) rc = finish_next();
    if (rc != JFS_OK) {  // leave no copy in flight into the staging slots
        (void)hipStreamSynchronize(dev->s_in);
        (void)hipStreamSynchronize(ln.s_k);
        (void)hipStreamSynchronize(other.s_k);
        (void)hipStreamSynchronize(dev->s_out);
    }
    return rc;
}

// run_batch with per-block error isolation (a GPU codec
// reports per-block errors): when a batch fails as a whole (staging
// allocation, a copy or launch error), it is split in halves and each half
// re-run, down to single blocks, so a failure is charged only to the blocks
// that fail alone and a few bad blocks cost O(log n) re-runs, not n.  After a
// sticky HIP error (the lane's streams no longer synchronise) nothing is
// re-run: the remaining blocks report JFS_ERR_HIP at once.
bool lane_healthy(DevCtx *dev, Lane &ln) {
    DevGuard guard;
    (void)hipSetDevice(dev->id);
    return hipStreamSynchronize(dev->s_in) == hipSuccess && hipStreamSynchronize(ln.s_k) == hipSuccess &&
           hipStreamSynchronize(dev->s_out) == hipSuccess;
}

void run_isolated(DevCtx *dev, Lane &ln, int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out,
                  const Aead *ae = nullptr, uint32_t *crc = nullptr, uint8_t *const *csum = nullptr) {
    if (nblk <= 0) return;
    const int64_t rc = run_batch(dev, ln, algo, dir, nblk, iov, out, ae, crc, 0, nullptr, csum);
    if (rc == JFS_OK) return;
    if (nblk == 1 || (rc == JFS_ERR_HIP && !lane_healthy(dev, ln))) {
        for (int i = 0; i < nblk; i++) out[i] = rc;
        return;
    }
    const int h = nblk / 2;
    run_isolated(dev, ln, algo, dir, h, iov, out, ae, crc, csum);
    if (ae) {
        const Aead a2 = ae->at(h);
        run_isolated(dev, ln, algo, dir, nblk - h, iov + h, out + h, &a2, crc ? crc + h : nullptr,
                     csum ? csum + h : nullptr);
    } else {
        run_isolated(dev, ln, algo, dir, nblk - h, iov + h, out + h, nullptr, crc ? crc + h : nullptr,
                     csum ? csum + h : nullptr);
    }
}

// ---------------------------------------------------------------------------
// coalescer for the one-call-per-block API
// ---------------------------------------------------------------------------
struct Pending {
    int algo, dir;
    jfs_iov iov;
    int64_t res;
    bool done;
    // the caller's own wake-up: a release wakes only the callers it answers
    // (one shared condition woke all ~200 waiting callers per released chunk,
    // each re-taking the queue mutex that the gathering worker needs)
    std::condition_variable cv;
};

// Gather window (microseconds): a worker that finds work waits until no new
// call has arrived for `gap` (or `max` has passed since it started), so a
// burst of concurrent calls (pkg/chunk runs up to 20 uploads and 200
// downloads at once, cmd/flags.go:133-139) becomes one batch.  A lone call
// pays `gap`.  JFS_GATHER_US=<decompress gap>,<compress gap> overrides the
// gaps (max = 16 x gap).
struct Gather {
    int64_t gap_us, max_us;
};
// Decode batches of the coalescer run in chunks of at most this many blocks
// (JFS_COALESCE_CHUNK, 0 = by staging bytes only): the first chunk's callers
// return while later chunks run, and chunk copies / kernels pipeline.
int coalesce_chunk_blocks() {
    static int v = [] {
        const char *e = getenv("JFS_COALESCE_CHUNK");
        return e ? std::max(0, atoi(e)) : 16;
    }();
    return v;
}

Gather gather_window(int dir) {
    static int64_t g[2] = {-1, -1};
    static std::once_flag once;
    std::call_once(once, [] {
        g[DECOMPRESS_DIR] = 300;  // a lone 4 MiB decode takes milliseconds
        g[COMPRESS_DIR] = 2000;   // an encode takes ~0.1-0.5 s: gather generously
        if (const char *e = getenv("JFS_GATHER_US")) {
            char *end = nullptr;
            g[DECOMPRESS_DIR] = std::max(0ll, strtoll(e, &end, 10));
            if (end && *end == ',') g[COMPRESS_DIR] = std::max(0ll, strtoll(end + 1, nullptr, 10));
        }
    });
    static const int64_t mx = [] {  // JFS_GATHER_MAX_X: max = gap x this (default 16)
        const char *e = getenv("JFS_GATHER_MAX_X");
        return e ? std::max(1ll, atoll(e)) : 16ll;
    }();
    const int64_t gap = g[dir == DECOMPRESS_DIR ? DECOMPRESS_DIR : COMPRESS_DIR];
    return {gap, gap * mx};
}

int64_t gather_probe_us() {
    static const int64_t v = [] {
        const char *e = getenv("JFS_GATHER_PROBE_US");
        return e ? std::max(0ll, atoll(e)) : 0ll;
    }();
    return v;
}

int64_t gather_probe_enc_us() {
    static const int64_t v = [] {
        const char *e = getenv("JFS_GATHER_PROBE_ENC_US");
        return e ? std::max(0ll, atoll(e)) : 300ll;
    }();
    return v;
}

// Work of one block for the dealer: the bytes it stages in and out.
int64_t block_cost(const jfs_iov &v) { return std::max<int64_t>(v.src_len, 0) + std::max<int64_t>(v.dst_cap, 0) + 4096; }

// Size-balanced deal (SURVEY.md 8e, config 4's mixed 64 KiB - 4 MiB blocks):
// longest-processing-time greedy -- blocks by decreasing cost (ties in block
// order), each to the device with the least cost so far (ties to the lowest
// device).  No device ends more than one block's cost above another.
void plan_deal(const int64_t *cost, int n, int ndev, int32_t *out_dev) {
    if (n <= 0) return;
    if (ndev <= 1) {
        for (int i = 0; i < n; i++) out_dev[i] = 0;
        return;
    }
    std::vector<int> ord(n);
    for (int i = 0; i < n; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int a, int b) { return cost[a] > cost[b]; });
    std::vector<int64_t> load(ndev, 0);
    for (int i : ord) {
        int best = 0;
        for (int d = 1; d < ndev; d++)
            if (load[d] < load[best]) best = d;
        out_dev[i] = best;
        load[best] += std::max<int64_t>(cost[i], 0);
    }
}

// A gathered burst is spread over other devices' idle lanes when it holds at
// least this many staged bytes (JFS_SPREAD_MIN_MB; default 8 MiB: two 4 MiB blocks).
int64_t spread_min_bytes() {
    static const int64_t v = [] {
        const char *e = getenv("JFS_SPREAD_MIN_MB");
        return e ? std::max(0ll, atoll(e)) << 20 : (int64_t)8 << 20;
    }();
    return v;
}

// The lanes a coalescer worker runs a gathered burst on: its own lane, and
// (spreading) one idle lane of each other device, at most
// `parts - 1` of them.  Lock order, so that no two workers can deadlock: the
// own lane is taken first and blocking, while the worker holds nothing else;
// other devices' lanes are only ever try-locked, so no thread ever waits while
// holding a lane that another thread waits for.  (Round 4 try-locked the
// foreign lanes first and then blocked on its own: two workers could each
// hold the other's lane.)  Host-only logic: jfs_test_spread_locking runs it on
// fake devices.
struct SpreadLanes {
    std::unique_lock<std::mutex> own;
    std::vector<DevCtx *> hdev;
    std::vector<Lane *> hlane;
    std::vector<std::unique_lock<std::mutex>> hlock;
    void release() {
        hlock.clear();
        hlane.clear();
        hdev.clear();
        if (own.owns_lock()) own.unlock();
    }
};

void spread_acquire(DevCtx *dev, Lane &ln, const std::vector<DevCtx *> &all, int parts, SpreadLanes &sl) {
    sl.own = std::unique_lock<std::mutex>(ln.mu);
    for (DevCtx *d : all) {
        if (d == dev || (int)sl.hdev.size() + 1 >= parts) continue;
        for (int k = 0; k < NLANE; k++) {
            std::unique_lock<std::mutex> t(d->lane[k].mu, std::try_to_lock);
            if (t.owns_lock()) {
                sl.hdev.push_back(d);
                sl.hlane.push_back(&d->lane[k]);
                sl.hlock.push_back(std::move(t));
                break;
            }
        }
    }
}

class Coalescer {
   public:
    static Coalescer &get() {
        static Coalescer *c = new Coalescer();  // never destroyed: worker threads outlive static dtors
        return *c;
    }
    int64_t submit(int algo, int dir, const jfs_iov &iov) {
        std::vector<DevCtx *> &ds = devices();
        if (ds.empty()) return JFS_ERR_NO_DEVICE;
        start(ds);
        int64_t res = 0;
        if (dir == DECOMPRESS && inline_lone() && run_inline(ds, algo, dir, iov, &res)) return res;
        Pending p{algo, dir, iov, 0, false, {}};
        std::unique_lock<std::mutex> lk(mu_);
        q_.push_back(&p);
        arrivals_++;
        cv_work_.notify_all();
        p.cv.wait(lk, [&] { return p.done; });
        return p.res;
    }

   private:
    // A batch holds every queued call of one codec and direction, up to a
    // decode launch's worth of resident blocks; run_batch cuts it into
    // pipelined chunks of at most chunk_limit() staging bytes.
    static constexpr int kMaxBlocks = 4096;
    std::mutex mu_;
    std::condition_variable cv_work_;
    std::deque<Pending *> q_;
    uint64_t arrivals_ = 0;
    bool gathering_ = false;  // one worker gathers at a time; the others run batches
    int waiting_batches_ = 0;  // batches running with callers not yet released (guarded by mu_)
    std::once_flag started_;

    void start(std::vector<DevCtx *> &ds) {
        std::call_once(started_, [&] {
            // NLANE workers per device: a device runs the next batch while the
            // previous one is still in flight (each worker owns one lane)
            for (DevCtx *d : ds)
                for (int k = 0; k < NLANE; k++) std::thread([this, d, k] { worker(d, d->lane[k]); }).detach();
        });
    }
    // A decode that finds nothing queued and no batch waiting on the devices
    // (a lone cache miss) runs on the calling thread when a lane is free: no
    // hand-off to a worker and back (JFS_INLINE_LONE=0: always hand off).  It
    // counts as a waiting batch, so calls arriving meanwhile gather.
    static bool inline_lone() {
        static const bool v = [] {
            const char *e = getenv("JFS_INLINE_LONE");
            return !e || atoi(e) != 0;
        }();
        return v;
    }
    bool run_inline(std::vector<DevCtx *> &ds, int algo, int dir, const jfs_iov &iov, int64_t *res) {
        DevCtx *dev = nullptr;
        Lane *ln = nullptr;
        std::unique_lock<std::mutex> lane_lk;
        {
            std::lock_guard<std::mutex> lk(mu_);
            if (!q_.empty() || gathering_ || waiting_batches_ != 0) return false;
            for (DevCtx *d : ds) {  // (lanes are only ever try-locked here)
                for (int k = 0; k < NLANE && !ln; k++) {
                    std::unique_lock<std::mutex> t(d->lane[k].mu, std::try_to_lock);
                    if (t.owns_lock()) {
                        lane_lk = std::move(t);
                        dev = d;
                        ln = &d->lane[k];
                    }
                }
                if (ln) break;
            }
            if (!ln) return false;
            waiting_batches_++;
        }
        const double t0 = host_trace() ? now_ms() : 0.0;
        jfs_iov v = iov;
        int64_t out = 0;
        if (run_batch(dev, *ln, algo, dir, 1, &v, &out, nullptr, nullptr, 0, nullptr) != JFS_OK)
            run_isolated(dev, *ln, algo, dir, 1, &v, &out);
        lane_lk.unlock();
        if (host_trace())
            fprintf(stderr, "[jfs coalescer] t=%.2f dev %d lane %d algo %d dir %d: 1 call inline, ran %.2f ms\n",
                    now_ms(), dev->id, (int)(ln - dev->lane), algo, dir, now_ms() - t0);
        {
            std::lock_guard<std::mutex> lk(mu_);
            waiting_batches_--;
        }
        cv_work_.notify_all();  // calls that queued meanwhile
        *res = out;
        return true;
    }
    int queued_like(int algo, int dir) const {
        int n = 0;
        for (const Pending *p : q_) n += p->algo == algo && p->dir == dir;
        return n;
    }
    void worker(DevCtx *dev, Lane &ln) {
        std::vector<Pending *> batch;
        std::vector<jfs_iov> iov;
        std::vector<int64_t> out;
        std::vector<char> released;
        double t_gather = 0.0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_work_.wait(lk, [&] { return !q_.empty() && !gathering_; });
                gathering_ = true;
                t_gather = host_trace() ? now_ms() : 0.0;
                const int algo = q_.front()->algo, dir = q_.front()->dir;
                // Decode on an idle device: a lone call (a cache miss) goes at
                // once -- or, with JFS_GATHER_PROBE_US set, once no second call
                // has followed it within that probe; under load the calls that
                // arrive while a batch runs form the next one.  (A burst's first
                // call alone costs the burst little: the 200-way legs measured
                // the same with a 40 us probe and without.)  Encode probes
                // longer (JFS_GATHER_PROBE_ENC_US, default 300): an encode
                // batch lasts about one block's parse whatever its size, so a
                // burst's first call sent alone would put the rest behind a
                // whole extra batch -- a burst's second call comes within the
                // probe, and a lone upload skips the 2 ms gather.
                Gather gw = gather_window(dir);
                if (waiting_batches_ == 0 && queued_like(algo, dir) == 1) {
                    const uint64_t s0 = arrivals_;
                    const int64_t probe = dir == DECOMPRESS ? gather_probe_us() : gather_probe_enc_us();
                    if (probe > 0)
                        cv_work_.wait_until(lk, std::chrono::steady_clock::now() + std::chrono::microseconds(probe),
                                            [&] { return arrivals_ != s0; });
                    if (arrivals_ == s0) gw.gap_us = 0;
                }
                const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(gw.max_us);
                uint64_t seen = arrivals_;
                while (gw.gap_us > 0 && queued_like(algo, dir) < kMaxBlocks) {
                    const auto until = std::min(t_end, std::chrono::steady_clock::now() +
                                                           std::chrono::microseconds(gw.gap_us));
                    cv_work_.wait_until(lk, until, [&] { return arrivals_ != seen; });
                    if (arrivals_ == seen || std::chrono::steady_clock::now() >= t_end) break;
                    seen = arrivals_;
                }
                batch.clear();
                for (auto it = q_.begin(); it != q_.end() && (int)batch.size() < kMaxBlocks;) {
                    if ((*it)->algo == algo && (*it)->dir == dir) {
                        batch.push_back(*it);
                        it = q_.erase(it);
                    } else {
                        ++it;
                    }
                }
                gathering_ = false;
                waiting_batches_++;
            }
            cv_work_.notify_all();  // the next worker may start gathering
            size_t nrel = 0;  // callers released so far (under mu_)
            bool counted = true;  // this batch is in waiting_batches_
            auto released_one = [&]() {
                if (++nrel == batch.size() && counted) {
                    counted = false;
                    waiting_batches_--;
                }
            };
            iov.resize(batch.size());
            out.assign(batch.size(), 0);
            released.assign(batch.size(), 0);
            for (size_t i = 0; i < batch.size(); i++) iov[i] = batch[i]->iov;
            {
                const double t0 = host_trace() ? now_ms() : 0.0;
                const int algo = batch[0]->algo, dir = batch[0]->dir, n = (int)batch.size();
                // Other devices with an idle lane take a size-balanced share of
                // the gathered burst: their lanes are locked here
                // and released after their parts finish.
                std::vector<int64_t> cost(n);
                int64_t tot = 0;
                for (int i = 0; i < n; i++) tot += (cost[i] = block_cost(iov[i]));
                SpreadLanes sl;
                spread_acquire(dev, ln, devices(), n >= 2 && tot >= spread_min_bytes() ? n : 1, sl);
                std::vector<DevCtx *> &hdev = sl.hdev;
                std::vector<Lane *> &hlane = sl.hlane;
                const int G = 1 + (int)hdev.size();
                std::vector<int32_t> where(n, 0);
                plan_deal(cost.data(), n, G, where.data());
                std::vector<std::vector<int>> pidx(G);
                for (int i = 0; i < n; i++) pidx[where[i]].push_back(i);
                // chunks of a decode batch release their callers as they finish:
                // those callers' next calls gather while the rest of the batch runs
                const int cb = dir == DECOMPRESS ? coalesce_chunk_blocks() : 0;
                auto run_part = [&](DevCtx *d, Lane &L, const std::vector<int> &idx) {
                    const int np = (int)idx.size();
                    if (np == 0) return;
                    std::vector<jfs_iov> piov(np);
                    std::vector<int64_t> pout(np, 0);
                    std::vector<char> prel(np, 0);
                    for (int k = 0; k < np; k++) piov[k] = iov[idx[k]];
                    const std::function<void(int, int)> release = [&](int s, int e) {
                        std::lock_guard<std::mutex> lk(mu_);
                        for (int k = s; k < e; k++) {
                            batch[idx[k]]->res = pout[k];
                            batch[idx[k]]->done = true;
                            batch[idx[k]]->cv.notify_one();
                            released[idx[k]] = 1;
                            prel[k] = 1;
                            released_one();
                        }
                    };
                    if (run_batch(d, L, algo, dir, np, piov.data(), pout.data(), nullptr, nullptr, cb, &release) !=
                        JFS_OK) {
                        // what was not released yet goes through the error-isolating path
                        std::vector<int> rest;
                        for (int k = 0; k < np; k++)
                            if (!prel[k]) rest.push_back(k);
                        std::vector<jfs_iov> iv2(rest.size());
                        std::vector<int64_t> o2(rest.size(), 0);
                        for (size_t q = 0; q < rest.size(); q++) iv2[q] = piov[rest[q]];
                        run_isolated(d, L, algo, dir, (int)rest.size(), iv2.data(), o2.data());
                        for (size_t q = 0; q < rest.size(); q++) pout[rest[q]] = o2[q];
                    }
                    for (int k = 0; k < np; k++) out[idx[k]] = pout[k];
                };
                std::vector<std::thread> th;
                for (int g = 1; g < G; g++) th.emplace_back([&, g] { run_part(hdev[g - 1], *hlane[g - 1], pidx[g]); });
                run_part(dev, ln, pidx[0]);
                for (auto &t : th) t.join();
                sl.release();
                if (host_trace())
                    fprintf(stderr, "[jfs coalescer] t=%.2f dev %d lane %d algo %d dir %d: %zu calls on %d device(s), gathered %.2f ms, ran %.2f ms\n",
                            now_ms(), dev->id, (int)(&ln - dev->lane), algo, dir, batch.size(), G, t0 - t_gather,
                            now_ms() - t0);
            }
            {
                std::lock_guard<std::mutex> lk(mu_);
                for (size_t i = 0; i < batch.size(); i++) {
                    if (released[i]) continue;
                    batch[i]->res = out[i];
                    batch[i]->done = true;
                    batch[i]->cv.notify_one();
                }
                if (counted) {
                    counted = false;
                    waiting_batches_--;
                }
            }
        }
    }
};

bool pre_answer(int algo, int dir, const jfs_iov &v, int64_t *res) {
    // Results the Go adapters produce before reaching the C codec.
    if (algo == JFS_ALGO_NONE) {  // compress.go:55-68
        if (v.dst_cap < v.src_len) { *res = JFS_ERR_SHORT_BUFFER; return true; }
        if (v.src_len > 0) memmove(v.dst, v.src, (size_t)v.src_len);
        *res = v.src_len;
        return true;
    }
    if (v.src_len < 0 || v.dst_cap < 0) { *res = JFS_ERR_INVALID; return true; }
    if (dir == DECOMPRESS && v.src_len == 0) { *res = JFS_ERR_EMPTY_INPUT; return true; }  // compress.go:121, ErrEmptySlice
    if (algo == JFS_ALGO_LZ4 && dir == COMPRESS && v.src_len > LZ4_MAX_INPUT) { *res = JFS_ERR_COMPRESS_FAIL; return true; }
    if (algo == JFS_ALGO_ZSTD && dir == COMPRESS && v.dst_cap < jfs_compress_bound(JFS_ALGO_ZSTD, v.src_len)) {
        *res = JFS_ERR_SHORT_BUFFER;  // compress.go:86-89 (DataDog checks cap(dst) against CompressBound)
        return true;
    }
    return false;
}

// Deal the todo blocks over the selected devices, size-balanced
// (plan_deal) and run them; ae_all (optional) is parallel to iov2.
int64_t deal(int algo, int dir, const std::vector<int> &todo, const std::vector<jfs_iov> &iov2, int64_t *out_n,
             uint32_t mask, const Aead *ae_all, uint32_t *crc = nullptr, uint8_t *const *csum = nullptr) {
    std::vector<DevCtx *> &all = devices();
    std::vector<DevCtx *> ds;
    for (DevCtx *d : all)
        if (mask == 0 || (d->id < 32 && (mask >> d->id) & 1u)) ds.push_back(d);
    if (ds.empty()) return JFS_ERR_NO_DEVICE;
    const size_t G = std::min(ds.size(), todo.size());
    struct Part {
        std::vector<jfs_iov> iov, orig;
        std::vector<const uint8_t *> key, nonce;
        std::vector<jfs_seal_param> sp;
        std::vector<int64_t> hdr, res;
        std::vector<uint32_t> crc;
        std::vector<uint8_t *> csum;
        std::vector<int> idx;
    };
    std::vector<Part> part(G);
    std::vector<int64_t> cost(todo.size());
    for (size_t k = 0; k < todo.size(); k++) cost[k] = block_cost(iov2[k]);
    std::vector<int32_t> where(todo.size(), 0);
    plan_deal(cost.data(), (int)todo.size(), (int)G, where.data());
    for (size_t k = 0; k < todo.size(); k++) {
        Part &p = part[where[k]];
        p.iov.push_back(iov2[k]);
        p.idx.push_back(todo[k]);
        if (csum) p.csum.push_back(csum[todo[k]]);
        if (ae_all) {
            p.orig.push_back(ae_all->orig[k]);
            p.key.push_back(ae_all->key[k]);
            p.nonce.push_back(ae_all->nonce[k]);
            if (ae_all->sp) p.sp.push_back(ae_all->sp[k]);
            if (ae_all->hdr) p.hdr.push_back(ae_all->hdr[k]);
        }
    }
    auto work = [&](size_t g) {
        Part &p = part[g];
        p.res.assign(p.iov.size(), 0);
        p.crc.assign(p.iov.size(), 0u);
        uint32_t *pc = crc ? p.crc.data() : nullptr;
        std::unique_lock<std::mutex> lk;
        Lane &ln = ds[g]->acquire_lane(lk, algo * 2 + dir);
        if (ae_all) {
            Aead a{ae_all->cipher, ae_all->seal, p.orig.data(), p.key.data(), p.nonce.data(),
                   ae_all->sp ? p.sp.data() : nullptr, ae_all->hdr ? p.hdr.data() : nullptr};
            run_isolated(ds[g], ln, algo, dir, (int)p.iov.size(), p.iov.data(), p.res.data(), &a, pc);
        } else {
            run_isolated(ds[g], ln, algo, dir, (int)p.iov.size(), p.iov.data(), p.res.data(), nullptr, pc,
                         csum ? p.csum.data() : nullptr);
        }
    };
    if (G == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (size_t g = 0; g < G; g++) th.emplace_back(work, g);
        for (auto &t : th) t.join();
    }
    for (size_t g = 0; g < G; g++)
        for (size_t k = 0; k < part[g].idx.size(); k++) {
            out_n[part[g].idx[k]] = part[g].res[k];
            if (crc) crc[part[g].idx[k]] = part[g].crc[k];
        }
    return JFS_OK;
}

int64_t envelope_parse(const uint8_t *src, int64_t n, int64_t *woff, int64_t *wlen, int64_t *noff, int64_t *nlen) {
    if (!src || n < 3) return JFS_ERR_CORRUPT;  // "received encrypted text length is less than 3"
    const int64_t kl = ((int64_t)src[0] << 8) + src[1], nl = src[2];
    if (3 + kl + nl >= n) return JFS_ERR_CORRUPT;  // "malformed ciphertext"
    if (woff) *woff = 3;
    if (wlen) *wlen = kl;
    if (noff) *noff = 3 + kl;
    if (nlen) *nlen = nl;
    return 3 + kl + nl;
}

// disk_cache_file.go checksum() of n bytes on the host (blocks answered
// without the GPU: the "none" codec)
void host_csum(const uint8_t *p, int64_t n, uint8_t *out) {
    const int64_t nw = n > 0 ? (n - 1) / CSUM_SEG + 1 : 1;
    for (int64_t w = 0; w < nw; w++) {
        const int64_t a = w * CSUM_SEG, e = std::min<int64_t>(n, a + CSUM_SEG);
        const uint32_t v = n > 0 ? host_crc32c(0, p + a, e - a) : 0u;
        out[4 * w] = (uint8_t)(v >> 24);
        out[4 * w + 1] = (uint8_t)(v >> 16);
        out[4 * w + 2] = (uint8_t)(v >> 8);
        out[4 * w + 3] = (uint8_t)v;
    }
}

int64_t batch_common(int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t mask,
                     uint32_t *crc = nullptr, uint8_t *const *csum = nullptr) {
    if (nblk < 0 || (nblk > 0 && (!iov || !out_n))) return JFS_ERR_INVALID;
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    std::vector<int> todo;
    for (int i = 0; i < nblk; i++) {
        if (!pre_answer(algo, dir, iov[i], &out_n[i])) {
            todo.push_back(i);
        } else {
            if (crc) crc[i] = out_n[i] >= 0 ? host_crc32c(0, iov[i].dst, out_n[i]) : 0u;  // "none": the payload is dst
            if (csum && csum[i] && out_n[i] >= 0) host_csum(iov[i].dst, out_n[i], csum[i]);
        }
    }
    if (todo.empty()) return JFS_OK;
    std::vector<jfs_iov> iov2(todo.size());
    for (size_t k = 0; k < todo.size(); k++) iov2[k] = iov[todo[k]];
    return deal(algo, dir, todo, iov2, out_n, mask, nullptr, crc, csum);
}

}  // namespace

extern "C" {

int jfs_codec_from_name(const char *name) {
    if (!name) return -1;
    std::string s(name);
    for (auto &ch : s) ch = (char)tolower((unsigned char)ch);
    if (s == "zstd") return JFS_ALGO_ZSTD;
    if (s == "lz4") return JFS_ALGO_LZ4;
    if (s == "none" || s.empty()) return JFS_ALGO_NONE;
    return -1;
}

const char *jfs_codec_name(int algo) {
    switch (algo) {
        case JFS_ALGO_NONE: return "Noop";
        case JFS_ALGO_LZ4: return "LZ4";
        case JFS_ALGO_ZSTD: return "Zstd";
        default: return nullptr;
    }
}

int64_t jfs_compress_bound(int algo, int64_t n) {
    switch (algo) {
        case JFS_ALGO_NONE: return n;
        case JFS_ALGO_LZ4:
            // LZ4_compressBound takes an int: (unsigned)n > LZ4_MAX_INPUT_SIZE -> 0
            if ((uint64_t)(uint32_t)n != (uint64_t)n && n >= 0) return 0;
            if ((uint32_t)n > (uint32_t)LZ4_MAX_INPUT) return 0;
            return n + n / 255 + 16;
        case JFS_ALGO_ZSTD: {
            int64_t low = 128 << 10;
            int64_t margin = n < low ? (low - n) >> 11 : 0;
            return n + (n >> 8) + margin;
        }
        default: return JFS_ERR_INVALID;
    }
}

static int64_t one_call(int algo, int dir, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n) {
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    const int64_t t0 = steady_ns();
    jfs_iov v{src, n, dst, dst_cap};
    int64_t r;
    if (!pre_answer(algo, dir, v, &r)) r = Coalescer::get().submit(algo, dir, v);
    OpStats *st = op_stats(algo, dir);
    st->calls.fetch_add(1, std::memory_order_relaxed);
    stat_block(st, n, r);
    st->nanos.fetch_add((uint64_t)(steady_ns() - t0), std::memory_order_relaxed);
    return r;
}

int64_t jfs_compress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n) {
    return one_call(algo, COMPRESS, dst, dst_cap, src, n);
}

int64_t jfs_decompress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n) {
    return one_call(algo, DECOMPRESS, dst, dst_cap, src, n);
}

static int64_t batch_call(int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask,
                          uint32_t *crc = nullptr, uint8_t *const *csum = nullptr) {
    const int64_t t0 = steady_ns();
    const int64_t r = batch_common(algo, dir, nblk, iov, out_n, device_mask, crc, csum);
    if (OpStats *st = op_stats(algo, dir)) {
        st->calls.fetch_add(1, std::memory_order_relaxed);
        if (r == JFS_OK)
            for (int i = 0; i < nblk; i++) stat_block(st, iov[i].src_len, out_n[i]);
        st->nanos.fetch_add((uint64_t)(steady_ns() - t0), std::memory_order_relaxed);
    }
    return r;
}

int64_t jfs_envelope_bound(int algo, int64_t n, int32_t wrapped_len) {
    if (n < 0 || wrapped_len < 0 || wrapped_len > 65535) return JFS_ERR_INVALID;
    const int64_t b = algo == JFS_ALGO_NONE ? n : jfs_compress_bound(algo, n);
    if (b < 0) return b;
    return 3 + wrapped_len + 12 + b + 16;
}

int64_t jfs_envelope_parse(const uint8_t *src, int64_t n, int64_t *wrapped_off, int64_t *wrapped_len,
                           int64_t *nonce_off, int64_t *nonce_len) {
    return envelope_parse(src, n, wrapped_off, wrapped_len, nonce_off, nonce_len);
}

int64_t jfs_compress_seal_batch(int algo, int cipher, int nblk, const jfs_iov *iov, const jfs_seal_param *p,
                                int64_t *out_n, uint32_t *crc, uint32_t device_mask) {
    if (nblk < 0 || (nblk > 0 && (!iov || !out_n || !p))) return JFS_ERR_INVALID;
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    if (jfs_cipher_key_size(cipher) < 0) return JFS_ERR_INVALID;
    const int64_t t0 = steady_ns();
    std::vector<int> todo;
    std::vector<jfs_iov> iov2, orig;
    std::vector<const uint8_t *> key, nonce;
    std::vector<jfs_seal_param> sp;
    std::vector<int64_t> hdr;
    for (int i = 0; i < nblk; i++) {
        if (crc) crc[i] = 0;
        const jfs_iov &v = iov[i];
        const jfs_seal_param &q = p[i];
        const int64_t bound = jfs_envelope_bound(algo, v.src_len, q.wrapped_len);
        if (v.src_len < 0 || v.dst_cap < 0 || !q.key || !q.nonce || bound < 0 || (q.wrapped_len > 0 && !q.wrapped) ||
            (v.src_len > 0 && !v.src)) {
            out_n[i] = JFS_ERR_INVALID;
            continue;
        }
        if (algo == JFS_ALGO_LZ4 && v.src_len > LZ4_MAX_INPUT) {
            out_n[i] = JFS_ERR_COMPRESS_FAIL;
            continue;
        }
        if (v.dst_cap < bound) {
            out_n[i] = JFS_ERR_SHORT_BUFFER;
            continue;
        }
        todo.push_back(i);
        const int64_t pay = bound - (3 + q.wrapped_len + 12);  // codec bound + tag
        iov2.push_back(jfs_iov{v.src, v.src_len, nullptr, pay});
        orig.push_back(v);
        key.push_back(q.key);
        nonce.push_back(q.nonce);
        sp.push_back(q);
        hdr.push_back(3 + q.wrapped_len + 12);
    }
    int64_t rc = JFS_OK;
    if (!todo.empty()) {
        Aead ae{cipher, true, orig.data(), key.data(), nonce.data(), sp.data(), hdr.data()};
        rc = deal(algo, COMPRESS, todo, iov2, out_n, device_mask, &ae, crc);
    }
    if (OpStats *st = op_stats(algo, COMPRESS)) {
        st->calls.fetch_add(1, std::memory_order_relaxed);
        if (rc == JFS_OK)
            for (int i = 0; i < nblk; i++) stat_block(st, iov[i].src_len, out_n[i]);
        st->nanos.fetch_add((uint64_t)(steady_ns() - t0), std::memory_order_relaxed);
    }
    return rc;
}

int64_t jfs_open_decompress_batch(int algo, int cipher, int nblk, const jfs_iov *iov, const uint8_t *const *keys,
                                  int64_t *out_n, uint32_t device_mask) {
    if (nblk < 0 || (nblk > 0 && (!iov || !out_n || !keys))) return JFS_ERR_INVALID;
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    if (jfs_cipher_key_size(cipher) < 0) return JFS_ERR_INVALID;
    const int64_t t0 = steady_ns();
    std::vector<int> todo;
    std::vector<jfs_iov> iov2, orig;
    std::vector<const uint8_t *> key, nonce;
    for (int i = 0; i < nblk; i++) {
        const jfs_iov &v = iov[i];
        int64_t noff = 0, nlen = 0;
        const int64_t off = envelope_parse(v.src, v.src_len, nullptr, nullptr, &noff, &nlen);
        if (v.dst_cap < 0 || !keys[i]) {
            out_n[i] = JFS_ERR_INVALID;
            continue;
        }
        if (off < 0 || nlen != 12) {  // the AEADs here all take 12-byte nonces
            out_n[i] = JFS_ERR_CORRUPT;
            continue;
        }
        const int64_t pay = v.src_len - off;  // ciphertext || tag
        if (pay < 16) {
            out_n[i] = JFS_ERR_AUTH;  // aead.Open rejects a payload shorter than the tag
            continue;
        }
        if (algo != JFS_ALGO_NONE && pay == 16) {  // the codec would see an empty input
            out_n[i] = JFS_ERR_EMPTY_INPUT;
            continue;
        }
        int64_t cap;
        if (algo == JFS_ALGO_NONE) {
            if (v.dst_cap < pay - 16) {  // noOp.Decompress: "buffer too short" (compress.go:63-65)
                out_n[i] = JFS_ERR_SHORT_BUFFER;
                continue;
            }
            cap = pay - 16;
        } else if (algo == JFS_ALGO_ZSTD) {
            // DataDog's size hint reads the frame header, which is still
            // ciphertext here: stage dst_cap (frames from pkg/compress carry
            // their content size, for which both rules agree)
            cap = std::min<int64_t>(v.dst_cap, INT32_MAX);
        } else {
            jfs_iov pv{v.src + off, pay - 16, v.dst, v.dst_cap};
            cap = staged_cap(algo, DECOMPRESS, pv);
        }
        todo.push_back(i);
        iov2.push_back(jfs_iov{v.src + off, pay, nullptr, cap});
        orig.push_back(v);
        key.push_back(keys[i]);
        nonce.push_back(v.src + noff);
    }
    int64_t rc = JFS_OK;
    if (!todo.empty()) {
        Aead ae{cipher, false, orig.data(), key.data(), nonce.data(), nullptr, nullptr};
        rc = deal(algo, DECOMPRESS, todo, iov2, out_n, device_mask, &ae);
    }
    if (OpStats *st = op_stats(algo, DECOMPRESS)) {
        st->calls.fetch_add(1, std::memory_order_relaxed);
        if (rc == JFS_OK)
            for (int i = 0; i < nblk; i++) stat_block(st, iov[i].src_len, out_n[i]);
        st->nanos.fetch_add((uint64_t)(steady_ns() - t0), std::memory_order_relaxed);
    }
    return rc;
}

int64_t jfs_compress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask) {
    return batch_call(algo, COMPRESS, nblk, iov, out_n, device_mask);
}

// Mixed-codec batches: the blocks of each codec form one batch call.  Decode
// calls run at once (a device has two lanes, so an LZ4 and a Zstd batch share
// every device instead of queueing one behind the other: config 4 decode
// 13.2 -> 21.9 GiB/s); encode calls run in turn (see below).
static int64_t batch_mixed(int dir, const int32_t *algo, int nblk, const jfs_iov *iov, int64_t *out_n,
                           uint32_t device_mask) {
    if (nblk < 0 || (nblk > 0 && (!algo || !iov || !out_n))) return JFS_ERR_INVALID;
    std::vector<int> idx[3];
    for (int i = 0; i < nblk; i++) {
        const int a = algo[i];
        if (a != JFS_ALGO_NONE && a != JFS_ALGO_LZ4 && a != JFS_ALGO_ZSTD) {
            out_n[i] = JFS_ERR_INVALID;
            continue;
        }
        idx[a].push_back(i);
    }
    struct Group {
        int algo;
        std::vector<jfs_iov> iov;
        std::vector<int64_t> out;
        int64_t rc = JFS_OK;
    };
    std::vector<Group> gs;
    for (int a = 0; a < 3; a++) {
        if (idx[a].empty()) continue;
        Group g;
        g.algo = a;
        for (int i : idx[a]) g.iov.push_back(iov[i]);
        g.out.assign(idx[a].size(), 0);
        gs.push_back(std::move(g));
    }
    auto run = [&](Group &g) {
        g.rc = batch_call(g.algo, dir, (int)g.iov.size(), g.iov.data(), g.out.data(), device_mask);
    };
    static const bool enc_together = [] {
        const char *e = getenv("JFS_MIXED_ENCODE_TOGETHER");
        return e && atoi(e) != 0;
    }();
    if (dir == DECOMPRESS || enc_together) {
        std::vector<std::thread> th;
        for (size_t k = 1; k < gs.size(); k++) th.emplace_back(run, std::ref(gs[k]));
        if (!gs.empty()) run(gs[0]);
        for (auto &t : th) t.join();
    } else {
        // encoders one codec after the other: measured on config 4's mix, the
        // LZ4 serial-parse kernels beside the Zstd encoder's host-synchronised
        // parse rounds ran 0.93 GiB/s against 1.47 in turn
        for (Group &g : gs) run(g);
    }
    // the first failing codec call's code is returned, and every block of a
    // failed call reports it in out_n (never a stale length)
    int64_t rc = JFS_OK;
    for (Group &g : gs) {
        const std::vector<int> &ix = idx[g.algo];
        if (g.rc != JFS_OK) {
            if (rc == JFS_OK) rc = g.rc;
            for (size_t k = 0; k < ix.size(); k++) out_n[ix[k]] = g.rc;
            continue;
        }
        for (size_t k = 0; k < ix.size(); k++) out_n[ix[k]] = g.out[k];
    }
    return rc;
}

int64_t jfs_compress_batch_mixed(const int32_t *algo, int nblk, const jfs_iov *iov, int64_t *out_n,
                                 uint32_t device_mask) {
    return batch_mixed(COMPRESS, algo, nblk, iov, out_n, device_mask);
}

int64_t jfs_decompress_batch_mixed(const int32_t *algo, int nblk, const jfs_iov *iov, int64_t *out_n,
                                   uint32_t device_mask) {
    return batch_mixed(DECOMPRESS, algo, nblk, iov, out_n, device_mask);
}

int64_t jfs_compress_batch_crc(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t *crc,
                               uint32_t device_mask) {
    if (nblk > 0 && !crc) return JFS_ERR_INVALID;
    return batch_call(algo, COMPRESS, nblk, iov, out_n, device_mask, crc);
}

int64_t jfs_decompress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask) {
    return batch_call(algo, DECOMPRESS, nblk, iov, out_n, device_mask);
}

int64_t jfs_decompress_batch_csum(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint8_t *const *csum,
                                  uint32_t device_mask) {
    if (nblk > 0 && !csum) return JFS_ERR_INVALID;
    return batch_call(algo, DECOMPRESS, nblk, iov, out_n, device_mask, nullptr, csum);
}

void jfs_deal_plan(const int64_t *cost, int n, int ndev, int32_t *out_dev) {
    if (!cost || !out_dev || n <= 0) return;
    plan_deal(cost, n, ndev, out_dev);
}

int64_t jfs_test_spread_locking(int ndev, int iters, int timeout_ms) {
    if (ndev < 1 || ndev > 32 || iters < 1) return -2;
    // fake devices (no GPU state: only their lane mutexes are used)
    struct Run {
        std::vector<DevCtx *> devs;
        std::atomic<int> finished{0};
        std::atomic<int64_t> spread{0};
    };
    auto *r = new Run;  // leaked on a deadlock (the stuck threads still use it)
    for (int d = 0; d < ndev; d++) {
        r->devs.push_back(new DevCtx);
        r->devs.back()->id = d;
    }
    const int nthr = ndev * NLANE;
    for (int t = 0; t < nthr; t++) {
        std::thread([r, t, iters, ndev] {
            DevCtx *dev = r->devs[t / NLANE];
            Lane &ln = dev->lane[t % NLANE];
            for (int i = 0; i < iters; i++) {
                SpreadLanes sl;
                spread_acquire(dev, ln, r->devs, ndev + 1, sl);
                if (!sl.hdev.empty()) r->spread.fetch_add(1);
                std::this_thread::yield();
                sl.release();
            }
            r->finished.fetch_add(1);
        }).detach();
    }
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    while (r->finished.load() < nthr) {
        if (std::chrono::steady_clock::now() > t_end) return -1;  // deadlocked
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
    const int64_t sp = r->spread.load();
    for (DevCtx *d : r->devs) delete d;
    delete r;
    return sp;
}

// The device-resident entry points launch on the caller's current device; it
// must be one the library selected (gfx950, in JFS_GPU_DEVICES).
static bool current_device_ok() {
    std::vector<DevCtx *> &ds = devices();
    int cur = -1;
    if (ds.empty() || hipGetDevice(&cur) != hipSuccess) return false;
    for (DevCtx *d : ds)
        if (d->id == cur) return true;
    return false;
}

int64_t jfs_lz4_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    stat_launch(JFS_ALGO_LZ4, DECOMPRESS, nblk);
    return jfs_launch_lz4_decode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

// Small-batch device decode: per-device scratch shared by every caller,
// ordered across streams by an event (like the Zstd device decoder's).
struct SplitScratch {
    std::mutex mu;
    uint8_t *p = nullptr;
    int64_t cap = 0;
    hipEvent_t ev_done = nullptr;
};
SplitScratch g_split[64];

int64_t jfs_lz4_decompress_device_small(const jfs_dev_block *d_blocks, const int32_t *src_len, const int32_t *dst_cap,
                                        int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0 || (nblk > 0 && (!src_len || !dst_cap))) return JFS_ERR_INVALID;
    if (nblk == 0) return JFS_OK;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return JFS_ERR_HIP;
    stat_launch(JFS_ALGO_LZ4, DECOMPRESS, nblk);
    int64_t nseg = 0, max_cap = 0, norg = 0;
    for (int k = 0; k < nblk; k++) {
        nseg += (std::max(src_len[k], 0) + JFS_LZ4_SPLIT_SEG - 1) / JFS_LZ4_SPLIT_SEG;
        max_cap = std::max<int64_t>(max_cap, dst_cap[k]);
        norg += (std::max<int64_t>(dst_cap[k], 0) + 3) & ~3ll;
    }
    const int64_t need = jfs_lz4_split_scratch_bytes(nblk, src_len, dst_cap);
    SplitScratch &z = g_split[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (!z.ev_done && hipEventCreateWithFlags(&z.ev_done, hipEventDisableTiming) != hipSuccess) return JFS_ERR_HIP;
    if (need > z.cap) {
        if (hipEventSynchronize(z.ev_done) != hipSuccess) return JFS_ERR_HIP;  // earlier launches may still use it
        if (z.p) (void)hipFree(z.p);
        z.p = nullptr;
        z.cap = 0;
        int64_t want = 64ll << 20;
        while (want < need) want <<= 1;
        if (hipMalloc((void **)&z.p, (size_t)want) != hipSuccess) return JFS_ERR_NO_MEMORY;
        z.cap = want;
    }
    hipStream_t st = (hipStream_t)stream;
    if (hipStreamWaitEvent(st, z.ev_done, 0) != hipSuccess) return JFS_ERR_HIP;
    if (jfs_launch_lz4_split(d_blocks, nblk, d_ret, z.p, nseg, max_cap, norg, st) != 0) return JFS_ERR_HIP;
    return hipEventRecord(z.ev_done, st) == hipSuccess ? JFS_OK : JFS_ERR_HIP;
}

SplitScratch g_eseg_scr[64];

int64_t jfs_lz4_compress_device_small(const jfs_dev_block *d_blocks, const int32_t *src_len, int nblk, int32_t *d_ret,
                                      void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0 || (nblk > 0 && !src_len)) return JFS_ERR_INVALID;
    if (nblk == 0) return JFS_OK;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return JFS_ERR_HIP;
    stat_launch(JFS_ALGO_LZ4, COMPRESS, nblk);
    const int64_t need = jfs_lz4_eseg_scratch_bytes(nblk, src_len);
    SplitScratch &z = g_eseg_scr[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (!z.ev_done && hipEventCreateWithFlags(&z.ev_done, hipEventDisableTiming) != hipSuccess) return JFS_ERR_HIP;
    if (need > z.cap) {
        if (hipEventSynchronize(z.ev_done) != hipSuccess) return JFS_ERR_HIP;
        if (z.p) (void)hipFree(z.p);
        z.p = nullptr;
        z.cap = 0;
        int64_t want = 64ll << 20;
        while (want < need) want <<= 1;
        if (hipMalloc((void **)&z.p, (size_t)want) != hipSuccess) return JFS_ERR_NO_MEMORY;
        z.cap = want;
    }
    hipStream_t st = (hipStream_t)stream;
    if (hipStreamWaitEvent(st, z.ev_done, 0) != hipSuccess) return JFS_ERR_HIP;
    if (jfs_launch_lz4_encode_seg(d_blocks, nblk, src_len, d_ret, z.p, z.cap, st) != 0) return JFS_ERR_HIP;
    return hipEventRecord(z.ev_done, st) == hipSuccess ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_lz4_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    stat_launch(JFS_ALGO_LZ4, COMPRESS, nblk);
    return jfs_launch_lz4_encode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_zstd_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    stat_launch(JFS_ALGO_ZSTD, COMPRESS, nblk);
    return jfs_launch_zstd_encode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_zstd_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    stat_launch(JFS_ALGO_ZSTD, DECOMPRESS, nblk);
    return jfs_launch_zstd_decode(d_blocks, nblk, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_crc32c_device(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes, uint32_t *d_crc,
                          int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0 || seg_bytes < 0 || (seg_bytes > 0 && seg_bytes % 4096 != 0)) return JFS_ERR_INVALID;
    return jfs_launch_crc32c(d_blocks, nblk, seg_bytes, d_crc, d_ret, (hipStream_t)stream) == 0 ? JFS_OK
                                                                                              : JFS_ERR_HIP;
}

int64_t jfs_aes256gcm_seal_device(const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0) return JFS_ERR_INVALID;
    return jfs_launch_aes256gcm(d_blocks, nblk, 0, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_aes256gcm_open_device(const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0) return JFS_ERR_INVALID;
    return jfs_launch_aes256gcm(d_blocks, nblk, 1, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int jfs_cipher_from_name(const char *name) {
    if (!name) return -1;
    std::string v(name);
    for (auto &ch : v) ch = (char)tolower((unsigned char)ch);
    if (v.empty() || v == "aes256gcm-rsa") return JFS_CIPHER_AES256GCM;  // encrypt.go:178
    if (v == "chacha20-rsa") return JFS_CIPHER_CHACHA20POLY1305;           // :190
    if (v == "sm4gcm") return JFS_CIPHER_SM4GCM;                            // :191
    return -1;
}

int jfs_cipher_key_size(int cipher) {
    switch (cipher) {
        case JFS_CIPHER_AES256GCM: return 32;
        case JFS_CIPHER_CHACHA20POLY1305: return 32;
        case JFS_CIPHER_SM4GCM: return 16;
        default: return -1;
    }
}

int64_t jfs_aead_seal_device(int cipher, const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0 || jfs_cipher_key_size(cipher) < 0) return JFS_ERR_INVALID;
    return jfs_launch_aead(cipher, d_blocks, nblk, 0, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_aead_open_device(int cipher, const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0 || jfs_cipher_key_size(cipher) < 0) return JFS_ERR_INVALID;
    return jfs_launch_aead(cipher, d_blocks, nblk, 1, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_lz4_compress_seal_device(const jfs_dev_block *d_comp, const jfs_aead_block *d_aead, int nblk,
                                     int32_t *d_ret_comp, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0) return JFS_ERR_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (jfs_launch_lz4_encode(d_comp, nblk, d_ret_comp, st) != 0) return JFS_ERR_HIP;
    return jfs_launch_aes256gcm(d_aead, nblk, 0, d_ret, d_ret_comp, st) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_open_lz4_decompress_device(const jfs_aead_block *d_aead, const jfs_dev_block *d_dec, int nblk,
                                       int32_t *d_ret_open, int32_t *d_ret, void *stream) {
    if (!current_device_ok()) return JFS_ERR_NO_DEVICE;
    if (nblk < 0) return JFS_ERR_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (jfs_launch_aes256gcm(d_aead, nblk, 1, d_ret_open, nullptr, st) != 0) return JFS_ERR_HIP;
    return jfs_launch_lz4_decode_lens(d_dec, nblk, d_ret, d_ret_open, st) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int jfs_device_count(void) { return (int)devices().size(); }

int jfs_gpu_mode(void) { return gpu_mode(); }

int jfs_stats(jfs_op_stats *out, int n) {
    for (int i = 0; out && i < n && i < JFS_STATS_N; i++) {
        const OpStats &g = g_stats[i];
        out[i].calls = g.calls.load(std::memory_order_relaxed);
        out[i].blocks = g.blocks.load(std::memory_order_relaxed);
        out[i].bytes_in = g.bytes_in.load(std::memory_order_relaxed);
        out[i].bytes_out = g.bytes_out.load(std::memory_order_relaxed);
        out[i].errors = g.errors.load(std::memory_order_relaxed);
        out[i].nanos = g.nanos.load(std::memory_order_relaxed);
        out[i].batches = g.batches.load(std::memory_order_relaxed);
    }
    return JFS_STATS_N;
}

void jfs_stats_reset(void) {
    for (OpStats &g : g_stats) {
        g.calls = 0;
        g.blocks = 0;
        g.bytes_in = 0;
        g.bytes_out = 0;
        g.errors = 0;
        g.nanos = 0;
        g.batches = 0;
    }
    for (DevCtx *d : devices()) {
        d->batches = 0;
        d->blocks = 0;
    }
}

int jfs_device_stats(jfs_device_stat *out, int n) {
    std::vector<DevCtx *> &ds = devices();
    for (int i = 0; out && i < n && i < (int)ds.size(); i++) {
        out[i].device = ds[i]->id;
        out[i].batches = ds[i]->batches.load(std::memory_order_relaxed);
        out[i].blocks = ds[i]->blocks.load(std::memory_order_relaxed);
    }
    return (int)ds.size();
}

void jfs_release_staging(void) {
    for (DevCtx *d : devices()) {
        DevGuard guard;
        for (Lane &ln : d->lane) {
            std::lock_guard<std::mutex> lk(ln.mu);
            release_lane_staging(d, ln);
        }
    }
}

const char *jfs_version(void) { return JFS_VERSION; }

int64_t jfs_gen_blocks_device(uint8_t *d_dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                          void *stream) {
    std::vector<DevCtx *> &ds = devices();
    if (ds.empty()) return JFS_ERR_NO_DEVICE;
    int cur = 0;
    (void)hipGetDevice(&cur);
    DevCtx *dev = nullptr;
    for (DevCtx *d : ds)
        if (d->id == cur) dev = d;
    if (!dev) return JFS_ERR_NO_DEVICE;
    {
        std::lock_guard<std::mutex> lk(dev->vocab_mu);
        if (!dev->d_vocab) {
            std::vector<uint8_t> v(JFS_VOCAB_WORDS * 16);
            jfs_build_vocab(v.data());
            if (hipMalloc((void **)&dev->d_vocab, v.size()) != hipSuccess) return JFS_ERR_HIP;
            if (hipMemcpy(dev->d_vocab, v.data(), v.size(), hipMemcpyHostToDevice) != hipSuccess) return JFS_ERR_HIP;
        }
    }
    return jfs_launch_gen(d_dst, nblk, block_bytes, cls, seed_base, dev->d_vocab, (hipStream_t)stream) == 0
               ? JFS_OK
               : JFS_ERR_HIP;
}

void jfs_gen_block_host(uint8_t *dst, int64_t n, char cls, uint64_t seed) {
    static std::once_flag once;
    static std::vector<uint8_t> vocab(JFS_VOCAB_WORDS * 16);
    std::call_once(once, [] { jfs_build_vocab(vocab.data()); });
    struct E {
        uint8_t *p;
        void operator()(uint8_t b) { *p++ = b; }
    } e{dst};
    jfs_gen_stream(vocab.data(), cls, seed, n, e);
}

}  // extern "C"
