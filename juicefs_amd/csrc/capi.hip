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
// coalescer; one worker thread per device drains the queue, so calls that
// arrive while a batch is running ride the next batch (no artificial delay).
// Batches go host -> pinned staging -> HBM -> kernel -> HBM -> pinned -> host.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "blockgen.h"
#include "jfs_internal.h"

#define JFS_VERSION "jfs-gpucodec 0.1.0 (gfx950)"

namespace {

constexpr int64_t LZ4_MAX_INPUT = 0x7E000000;

inline int64_t align16(int64_t x) { return (x + 15) & ~(int64_t)15; }

struct DevCtx {
    int id = -1;
    hipStream_t stream = nullptr;
    std::mutex mu;  // serialises use of the staging buffers below
    uint8_t *h_pin = nullptr;
    int64_t h_cap = 0;
    uint8_t *d_buf = nullptr;
    int64_t d_cap = 0;
    uint8_t *d_vocab = nullptr;

    bool ensure(int64_t host_bytes, int64_t dev_bytes) {
        (void)hipSetDevice(id);
        if (host_bytes > h_cap) {
            if (h_pin) (void)hipHostFree(h_pin);
            int64_t c = std::max<int64_t>(host_bytes, h_cap * 2);
            if (hipHostMalloc((void **)&h_pin, (size_t)c, hipHostMallocDefault) != hipSuccess) {
                h_pin = nullptr;
                h_cap = 0;
                return false;
            }
            h_cap = c;
        }
        if (dev_bytes > d_cap) {
            if (d_buf) (void)hipFree(d_buf);
            int64_t c = std::max<int64_t>(dev_bytes, d_cap * 2);
            if (hipMalloc((void **)&d_buf, (size_t)c) != hipSuccess) {
                d_buf = nullptr;
                d_cap = 0;
                return false;
            }
            d_cap = c;
        }
        return true;
    }
};

std::once_flag g_once;
std::vector<DevCtx *> g_devs;

void init_devices() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    for (int i = 0; i < n; i++) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
        if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) continue;
        DevCtx *d = new DevCtx();
        d->id = i;
        (void)hipSetDevice(i);
        if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
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

enum Dir { COMPRESS = 0, DECOMPRESS = 1 };

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

// Run blocks [0,nblk) of iov on one device, synchronously.  Blocks that the
// C-ABI answers without a kernel (empty input, noOp) are handled by the caller.
int64_t run_batch(DevCtx *dev, int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out) {
    if (nblk <= 0) return JFS_OK;
    std::lock_guard<std::mutex> lk(dev->mu);
    (void)hipSetDevice(dev->id);
    // layout: [inputs][outputs][descs][rets]
    std::vector<int64_t> in_off(nblk), out_off(nblk);
    int64_t tin = 0, tout = 0;
    for (int i = 0; i < nblk; i++) {
        in_off[i] = tin;
        tin += align16(iov[i].src_len);
        out_off[i] = tout;
        int64_t cap = iov[i].dst_cap;
        if (algo == JFS_ALGO_LZ4 && dir == COMPRESS) {
            // the kernel never writes at/after cap; stage the full bound so the
            // result can be copied out exactly
            cap = std::min<int64_t>(cap, iov[i].src_len + iov[i].src_len / 255 + 16);
        }
        if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS) {
            // cap(dst) < hint: DataDog decodes into a new hint-sized buffer
            cap = std::max<int64_t>(cap, zstd_size_hint(iov[i].src, iov[i].src_len));
        }
        if (algo == JFS_ALGO_ZSTD && dir == COMPRESS) cap = std::min<int64_t>(cap, jfs_compress_bound(JFS_ALGO_ZSTD, iov[i].src_len));
        tout += align16(std::max<int64_t>(cap, 0));
    }
    int64_t desc_bytes = align16((int64_t)nblk * (int64_t)sizeof(jfs_dev_block));
    int64_t ret_bytes = align16((int64_t)nblk * 4);
    int64_t host_bytes = tin + tout + desc_bytes + ret_bytes;
    if (!dev->ensure(host_bytes, host_bytes)) return JFS_ERR_HIP;
    uint8_t *h = dev->h_pin, *d = dev->d_buf;
    uint8_t *h_in = h, *h_out = h + tin;
    jfs_dev_block *h_desc = (jfs_dev_block *)(h + tin + tout);
    int32_t *h_ret = (int32_t *)(h + tin + tout + desc_bytes);
    uint8_t *d_in = d, *d_out = d + tin;
    jfs_dev_block *d_desc = (jfs_dev_block *)(d + tin + tout);
    int32_t *d_ret = (int32_t *)(d + tin + tout + desc_bytes);
    for (int i = 0; i < nblk; i++) {
        if (iov[i].src_len > 0) memcpy(h_in + in_off[i], iov[i].src, (size_t)iov[i].src_len);
        h_desc[i].src = d_in + in_off[i];
        h_desc[i].dst = d_out + out_off[i];
        h_desc[i].src_len = (int32_t)iov[i].src_len;
        int64_t cap = iov[i].dst_cap;
        if (algo == JFS_ALGO_LZ4 && dir == COMPRESS)
            cap = std::min<int64_t>(cap, iov[i].src_len + iov[i].src_len / 255 + 16);
        if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS)
            cap = std::max<int64_t>(cap, zstd_size_hint(iov[i].src, iov[i].src_len));
        if (algo == JFS_ALGO_ZSTD && dir == COMPRESS) cap = std::min<int64_t>(cap, jfs_compress_bound(JFS_ALGO_ZSTD, iov[i].src_len));
        h_desc[i].dst_cap = (int32_t)std::min<int64_t>(cap, INT32_MAX);
    }
    hipStream_t st = dev->stream;
    if (hipMemcpyAsync(d_in, h_in, (size_t)tin, hipMemcpyHostToDevice, st) != hipSuccess) return JFS_ERR_HIP;
    if (hipMemcpyAsync(d_desc, h_desc, (size_t)nblk * sizeof(jfs_dev_block), hipMemcpyHostToDevice, st) !=
        hipSuccess)
        return JFS_ERR_HIP;
    int rc = -1;
    if (algo == JFS_ALGO_LZ4 && dir == DECOMPRESS) rc = jfs_launch_lz4_decode(d_desc, nblk, d_ret, st);
    else if (algo == JFS_ALGO_LZ4 && dir == COMPRESS) rc = jfs_launch_lz4_encode(d_desc, nblk, d_ret, st);
    else if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS) rc = jfs_launch_zstd_decode(d_desc, nblk, d_ret, nullptr, st);
    else if (algo == JFS_ALGO_ZSTD && dir == COMPRESS) rc = jfs_launch_zstd_encode(d_desc, nblk, d_ret, st);
    else return JFS_ERR_UNSUPPORTED;
    if (rc != 0) return JFS_ERR_HIP;
    if (hipMemcpyAsync(h_ret, d_ret, (size_t)nblk * 4, hipMemcpyDeviceToHost, st) != hipSuccess) return JFS_ERR_HIP;
    if (hipMemcpyAsync(h_out, d_out, (size_t)tout, hipMemcpyDeviceToHost, st) != hipSuccess) return JFS_ERR_HIP;
    if (hipStreamSynchronize(st) != hipSuccess) return JFS_ERR_HIP;
    for (int i = 0; i < nblk; i++) {
        int64_t r = finish_result(algo, dir, h_ret[i]);
        if (algo == JFS_ALGO_ZSTD && dir == DECOMPRESS && r > 0 &&
            iov[i].dst_cap < zstd_size_hint(iov[i].src, iov[i].src_len)) {
            // decoded into DataDog's own buffer: compress.go:99-101 "buffer too short"
            r = JFS_ERR_SHORT_BUFFER;
        }
        if (r > 0) memcpy(iov[i].dst, h_out + out_off[i], (size_t)r);
        out[i] = r;
    }
    return JFS_OK;
}

// ---------------------------------------------------------------------------
// coalescer for the one-call-per-block API
// ---------------------------------------------------------------------------
struct Pending {
    int algo, dir;
    jfs_iov iov;
    int64_t res;
    bool done;
};

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
        Pending p{algo, dir, iov, 0, false};
        std::unique_lock<std::mutex> lk(mu_);
        q_.push_back(&p);
        cv_work_.notify_one();
        cv_done_.wait(lk, [&] { return p.done; });
        return p.res;
    }

   private:
    static constexpr int kMaxBlocks = 256;
    static constexpr int64_t kMaxBytes = 256ll << 20;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::deque<Pending *> q_;
    std::once_flag started_;

    void start(std::vector<DevCtx *> &ds) {
        std::call_once(started_, [&] {
            for (DevCtx *d : ds) std::thread([this, d] { worker(d); }).detach();
        });
    }
    void worker(DevCtx *dev) {
        std::vector<Pending *> batch;
        std::vector<jfs_iov> iov;
        std::vector<int64_t> out;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_work_.wait(lk, [&] { return !q_.empty(); });
                int algo = q_.front()->algo, dir = q_.front()->dir;
                int64_t bytes = 0;
                batch.clear();
                for (auto it = q_.begin(); it != q_.end() && (int)batch.size() < kMaxBlocks;) {
                    Pending *p = *it;
                    if (p->algo == algo && p->dir == dir && (batch.empty() || bytes + p->iov.src_len <= kMaxBytes)) {
                        batch.push_back(p);
                        bytes += p->iov.src_len + p->iov.dst_cap;
                        it = q_.erase(it);
                    } else {
                        ++it;
                    }
                }
            }
            iov.resize(batch.size());
            out.assign(batch.size(), 0);
            for (size_t i = 0; i < batch.size(); i++) iov[i] = batch[i]->iov;
            int64_t rc = run_batch(dev, batch[0]->algo, batch[0]->dir, (int)batch.size(), iov.data(), out.data());
            {
                std::lock_guard<std::mutex> lk(mu_);
                for (size_t i = 0; i < batch.size(); i++) {
                    batch[i]->res = rc == JFS_OK ? out[i] : rc;
                    batch[i]->done = true;
                }
            }
            cv_done_.notify_all();
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

int64_t batch_common(int algo, int dir, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t mask) {
    if (nblk < 0 || (nblk > 0 && (!iov || !out_n))) return JFS_ERR_INVALID;
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    std::vector<int> todo;
    for (int i = 0; i < nblk; i++) {
        if (!pre_answer(algo, dir, iov[i], &out_n[i])) todo.push_back(i);
    }
    if (todo.empty()) return JFS_OK;
    std::vector<DevCtx *> &all = devices();
    std::vector<DevCtx *> ds;
    for (DevCtx *d : all)
        if (mask == 0 || (d->id < 32 && (mask >> d->id) & 1u)) ds.push_back(d);
    if (ds.empty()) return JFS_ERR_NO_DEVICE;
    // round-robin deal of blocks to devices
    size_t G = std::min(ds.size(), todo.size());
    std::vector<std::vector<jfs_iov>> part(G);
    std::vector<std::vector<int>> idx(G);
    for (size_t k = 0; k < todo.size(); k++) {
        part[k % G].push_back(iov[todo[k]]);
        idx[k % G].push_back(todo[k]);
    }
    std::vector<int64_t> rc(G, JFS_OK);
    std::vector<std::vector<int64_t>> res(G);
    auto work = [&](size_t g) {
        res[g].assign(part[g].size(), 0);
        // bound each device batch to ~1 GiB of staging
        size_t s = 0;
        while (s < part[g].size() && rc[g] == JFS_OK) {
            size_t e = s;
            int64_t bytes = 0;
            while (e < part[g].size() && (e == s || bytes + part[g][e].src_len + part[g][e].dst_cap <= (1ll << 30))) {
                bytes += part[g][e].src_len + part[g][e].dst_cap;
                e++;
            }
            rc[g] = run_batch(ds[g], algo, dir, (int)(e - s), part[g].data() + s, res[g].data() + s);
            s = e;
        }
    };
    if (G == 1) work(0);
    else {
        std::vector<std::thread> th;
        for (size_t g = 0; g < G; g++) th.emplace_back(work, g);
        for (auto &t : th) t.join();
    }
    for (size_t g = 0; g < G; g++) {
        if (rc[g] != JFS_OK) return rc[g];
        for (size_t k = 0; k < idx[g].size(); k++) out_n[idx[g][k]] = res[g][k];
    }
    return JFS_OK;
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

int64_t jfs_compress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n) {
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    jfs_iov v{src, n, dst, dst_cap};
    int64_t r;
    if (pre_answer(algo, COMPRESS, v, &r)) return r;
    return Coalescer::get().submit(algo, COMPRESS, v);
}

int64_t jfs_decompress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n) {
    if (algo != JFS_ALGO_NONE && algo != JFS_ALGO_LZ4 && algo != JFS_ALGO_ZSTD) return JFS_ERR_INVALID;
    jfs_iov v{src, n, dst, dst_cap};
    int64_t r;
    if (pre_answer(algo, DECOMPRESS, v, &r)) return r;
    return Coalescer::get().submit(algo, DECOMPRESS, v);
}

int64_t jfs_compress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask) {
    return batch_common(algo, COMPRESS, nblk, iov, out_n, device_mask);
}

int64_t jfs_decompress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask) {
    return batch_common(algo, DECOMPRESS, nblk, iov, out_n, device_mask);
}

int64_t jfs_lz4_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (devices().empty()) return JFS_ERR_NO_DEVICE;
    return jfs_launch_lz4_decode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_lz4_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (devices().empty()) return JFS_ERR_NO_DEVICE;
    return jfs_launch_lz4_encode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_zstd_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (devices().empty()) return JFS_ERR_NO_DEVICE;
    return jfs_launch_zstd_encode(d_blocks, nblk, d_ret, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int64_t jfs_zstd_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream) {
    if (devices().empty()) return JFS_ERR_NO_DEVICE;
    return jfs_launch_zstd_decode(d_blocks, nblk, d_ret, nullptr, (hipStream_t)stream) == 0 ? JFS_OK : JFS_ERR_HIP;
}

int jfs_device_count(void) { return (int)devices().size(); }

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
        std::lock_guard<std::mutex> lk(dev->mu);
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
