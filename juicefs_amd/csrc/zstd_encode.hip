// Zstd frame encoder for gfx950 -- one wavefront per input.
//
// Replaces ZSTD_compress(level 1) reached from pkg/compress/compress.go:82-91
// (ZStandard.Compress -> zstd.CompressLevel(dst, src, ZSTD_LEVEL)).  The
// reference pins DataDog/zstd v1.5.6, whose encoder is not available offline,
// so byte parity with it is unpinnable; what this encoder
// guarantees is an RFC 8878 frame that libzstd and the GPU decoder both turn
// back into the input, no larger than ZSTD_COMPRESSBOUND (the capacity the Go
// adapter requires), with the frame layout libzstd uses (FCS always present,
// no checksum, no dictionary, raw blocks for incompressible data, smallest
// literal-header format).
//
// Per 128 KiB block:
//   1. greedy LZ77 parse (4-byte hash of the position, table of 4096 positions
//      in LDS, acceleration skip on misses like LZ4's, forward extension 64
//      bytes per step across the wave, backward catch-up); literals go
//      straight to the output, sequences to a per-input scratch list;
//   2. literals section: Raw_Literals_Block;
//   3. sequences section: Predefined_Mode for all three codes (no table
//      descriptions), FSE-encoded backwards exactly as RFC 8878 section 4.1.2
//      reads it (offsets are sent as offset + 3: no repeat codes);
//   4. if that is not smaller than the block, the block is stored raw.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
namespace zstde {

constexpr int32_t BLK = 128 << 10;          // Block_Maximum_Size
constexpr int64_t SEQ_CAP = BLK / 4 + 64;   // sequences per block (every match is >= 4 bytes)
constexpr int64_t SCR_PER = SEQ_CAP * 8;    // scratch bytes per input
constexpr int32_t HBITS = 12;               // hash table: 4096 positions

// RFC 8878 3.1.1.3.2.1 code tables and 3.1.1.3.2.2 predefined distributions
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

// FSE compression table (FSE_buildCTable semantics) of one code type
struct CTab {
    uint16_t st[64];   // state table: tableSize + spread position, by cumulative symbol rank
    int32_t dnb[53];   // deltaNbBits
    int32_t dfs[53];   // deltaFindState
};

struct Smem {
    uint32_t table[1 << HBITS];
    CTab ct[3];  // 0 LL (log 6), 1 ML (log 6), 2 OF (log 5)
    uint8_t lut_ll[64], lut_ml[128];
    uint8_t tsym[64];
    int32_t cumul[64];
};

__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

// Build the encoding table of a predefined distribution (lane 0 writes).
// Spread and state numbering are the decoder's (FSE_buildDTable): -1
// ("less than 1") symbols at the top, the others spread with step
// (size>>1)+(size>>3)+3 skipping the top; state table in symbol order.
__device__ void build_ctab(Smem &s, CTab &t, const int16_t *norm, int maxsv, int tlog) {
    if (lane_id() == 0) {
        const int size = 1 << tlog, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
        int high = size - 1;
        s.cumul[0] = 0;
        for (int u = 1; u <= maxsv + 1; u++) {
            if (norm[u - 1] == -1) {
                s.cumul[u] = s.cumul[u - 1] + 1;
                s.tsym[high--] = (uint8_t)(u - 1);
            } else {
                s.cumul[u] = s.cumul[u - 1] + norm[u - 1];
            }
        }
        int pos = 0;
        for (int sym = 0; sym <= maxsv; sym++) {
            for (int k = 0; k < norm[sym]; k++) {
                s.tsym[pos] = (uint8_t)sym;
                do { pos = (pos + step) & mask; } while (pos > high);
            }
        }
        for (int u = 0; u < size; u++) {
            const int sym = s.tsym[u];
            t.st[s.cumul[sym]++] = (uint16_t)(size + u);
        }
        int total = 0;
        for (int sym = 0; sym <= maxsv; sym++) {
            const int nc = norm[sym];
            if (nc == 0) {
                t.dnb[sym] = ((tlog + 1) << 16) - size;
                t.dfs[sym] = 0;
            } else if (nc == -1 || nc == 1) {
                t.dnb[sym] = (tlog << 16) - size;
                t.dfs[sym] = total - 1;
                total += 1;
            } else {
                const int mbo = tlog - (int)highbit((uint32_t)(nc - 1));
                t.dnb[sym] = (mbo << 16) - (nc << mbo);
                t.dfs[sym] = total - nc;
                total += nc;
            }
        }
    }
}

// ---------------------------------------------------------------------------
// byte access (the input is read-only; uniform addresses)
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t ld32u(const gc_u8 *p) {
    const uintptr_t a = (uintptr_t)p;
    const gc_u32 *w = (const gc_u32 *)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    const uint32_t w0 = w[0];
    if (sh == 0) return w0;
    return __builtin_amdgcn_alignbyte(w[1], w0, sh);
}

__device__ __forceinline__ uint32_t hash4(uint32_t v) { return (v * 2654435761u) >> (32 - HBITS); }

// ---------------------------------------------------------------------------
// backward bitstream writer (BIT_CStream semantics), uniform; bytes go to HBM
// ---------------------------------------------------------------------------
struct BitW {
    g_u8 *dst;
    int64_t wp, lim;  // next byte position; writes at or beyond lim are refused
    uint64_t bc;
    int bp;
    bool ovf;
};

__device__ __forceinline__ void bw_add(BitW &w, uint32_t v, int nb) {
    w.bc |= ((uint64_t)v & ((1ull << nb) - 1ull)) << w.bp;
    w.bp += nb;
}
__device__ __forceinline__ void bw_flush(BitW &w) {
    const int nbytes = w.bp >> 3;
    const int l = lane_id();
    if (w.wp + nbytes > w.lim) w.ovf = true;
    if (!w.ovf && l < nbytes) w.dst[w.wp + l] = (uint8_t)(w.bc >> (8 * l));
    w.wp += nbytes;
    w.bc = nbytes >= 8 ? 0ull : (w.bc >> (8 * nbytes));
    w.bp &= 7;
}

__device__ __forceinline__ uint32_t fse_init(const CTab &t, uint32_t sym) {
    const int32_t dnb = t.dnb[sym];
    const uint32_t nbo = (uint32_t)((dnb + (1 << 15)) >> 16);
    const uint32_t v = (nbo << 16) - (uint32_t)dnb;
    return t.st[(v >> nbo) + (uint32_t)t.dfs[sym]];
}
__device__ __forceinline__ void fse_enc(BitW &w, const CTab &t, uint32_t &st, uint32_t sym) {
    const uint32_t nbo = (uint32_t)(((int32_t)st + t.dnb[sym]) >> 16);
    bw_add(w, st, (int)nbo);
    st = t.st[(st >> nbo) + (uint32_t)t.dfs[sym]];
}
__device__ __forceinline__ void fse_fin(BitW &w, uint32_t st, int tlog) {
    bw_add(w, st, tlog);
    bw_flush(w);
}

__device__ __forceinline__ uint32_t ll_code(const Smem &s, uint32_t ll) { return ll < 64 ? s.lut_ll[ll] : highbit(ll) + 19; }
__device__ __forceinline__ uint32_t ml_code(const Smem &s, uint32_t mlb) {
    return mlb < 128 ? s.lut_ml[mlb] : highbit(mlb) + 36;
}

__device__ __forceinline__ void seq_fields(const uint64_t *seq, int64_t i, uint32_t &ll, uint32_t &ml, uint32_t &off) {
    const uint64_t r = seq[i];
    ll = (uint32_t)(r & 0x1FFFFu);
    ml = (uint32_t)((r >> 17) & 0x3FFFFu);
    off = (uint32_t)(r >> 35);
}

// Encode sequences [0, ns) (scratch records: ll | ml << 17 | off << 35 as
// u64) as the predefined-mode FSE bitstream at w.wp (ZSTD_encodeSequences
// order: last sequence first, states OF/ML/LL, extra bits LL/ML/OF).
__device__ void encode_sequences(const Smem &s, BitW &w, const uint64_t *seq, int64_t ns) {
    const CTab &TL = s.ct[0], &TM = s.ct[1], &TO = s.ct[2];
    uint32_t ll, ml, off;
    seq_fields(seq, ns - 1, ll, ml, off);
    uint32_t lc = ll_code(s, ll), mc = ml_code(s, ml - 3), ofv = off + 3, oc = highbit(ofv);
    uint32_t sML = fse_init(TM, mc), sOF = fse_init(TO, oc), sLL = fse_init(TL, lc);
    bw_add(w, ll - LL_BASE[lc], LL_BITS[lc]);
    bw_add(w, ml - ML_BASE[mc], ML_BITS[mc]);
    bw_flush(w);
    bw_add(w, ofv - (1u << oc), (int)oc);
    bw_flush(w);
    for (int64_t i = ns - 2; i >= 0; --i) {
        seq_fields(seq, i, ll, ml, off);
        lc = ll_code(s, ll);
        mc = ml_code(s, ml - 3);
        ofv = off + 3;
        oc = highbit(ofv);
        fse_enc(w, TO, sOF, oc);
        fse_enc(w, TM, sML, mc);
        fse_enc(w, TL, sLL, lc);
        bw_flush(w);
        bw_add(w, ll - LL_BASE[lc], LL_BITS[lc]);
        bw_add(w, ml - ML_BASE[mc], ML_BITS[mc]);
        bw_flush(w);
        bw_add(w, ofv - (1u << oc), (int)oc);
        bw_flush(w);
    }
    fse_fin(w, sML, 6);
    fse_fin(w, sOF, 5);
    fse_fin(w, sLL, 6);
    bw_add(w, 1, 1);  // end mark
    bw_flush(w);
    if (w.bp > 0) {   // last partial byte
        if (w.wp + 1 > w.lim) w.ovf = true;
        if (!w.ovf && lane_id() == 0) w.dst[w.wp] = (uint8_t)w.bc;
        w.wp++;
        w.bp = 0;
        w.bc = 0;
    }
}

// wave-parallel byte copy src[a, a+len) -> dst[o, o+len)
__device__ __forceinline__ void copy_bytes(g_u8 *dst, int64_t o, const gc_u8 *src, int64_t a, int64_t len) {
    const int l = lane_id();
    for (int64_t k = l; k < len; k += 64) dst[o + k] = src[a + k];
}

__device__ __forceinline__ void put3(g_u8 *dst, int64_t o, uint32_t v) {
    const int l = lane_id();
    if (l < 3) dst[o + l] = (uint8_t)(v >> (8 * l));
}

__global__ __launch_bounds__(64) void zstd_encode_kernel(const jfs_dev_block *__restrict__ blocks, int nblk,
                                                        int32_t *__restrict__ ret, uint64_t *__restrict__ scratch) {
    __shared__ Smem s;
    const int b = blockIdx.x;
    if (b >= nblk) return;
    const int l = lane_id();
    const jfs_dev_block d = ((const gc_blk *)blocks)[b];
    const gc_u8 *src = (const gc_u8 *)d.src;
    g_u8 *dst = (g_u8 *)d.dst;
    const int64_t n = d.src_len, cap = d.dst_cap;
    uint64_t *seq = scratch + (int64_t)b * SEQ_CAP;
    const int64_t bound = n + (n >> 8) + (n < BLK ? (BLK - n) >> 11 : 0);
    if (n < 0 || cap < bound) {  // compress.go:86-89: cap(dst) < CompressBound -> "buffer too short"
        if (l == 0) ret[b] = -2;
        return;
    }
    // tables
    for (int k = l; k < (1 << HBITS); k += 64) s.table[k] = 0;
    for (int v = l; v < 64; v += 64) {
        int c = 0;
        while (c + 1 < 36 && LL_BASE[c + 1] <= (uint32_t)v) c++;
        s.lut_ll[v] = (uint8_t)c;
    }
    for (int v = l; v < 128; v += 64) {
        int c = 0;
        while (c + 1 < 53 && ML_BASE[c + 1] - 3 <= (uint32_t)v) c++;
        s.lut_ml[v] = (uint8_t)c;
    }
    build_ctab(s, s.ct[0], LL_DEF, 35, 6);
    __builtin_amdgcn_wave_barrier();
    build_ctab(s, s.ct[1], ML_DEF, 52, 6);
    __builtin_amdgcn_wave_barrier();
    build_ctab(s, s.ct[2], OF_DEF, 28, 5);
    __syncthreads();

    // ---- frame header: magic, FHD, [Window_Descriptor], Frame_Content_Size
    int64_t op;
    {
        const bool single = n <= (1 << 19);
        int fcs_flag, fs;
        if (single) {
            if (n < 256) { fcs_flag = 0; fs = 1; }
            else if (n < 65536 + 256) { fcs_flag = 1; fs = 2; }
            else { fcs_flag = 2; fs = 4; }
        } else {
            fcs_flag = n < (1ll << 32) ? 2 : 3;
            fs = fcs_flag == 2 ? 4 : 8;
        }
        const uint32_t fhd = (uint32_t)((fcs_flag << 6) | (single ? 0x20 : 0));
        const int fpos = single ? 5 : 6;  // FCS position
        const uint64_t fv = (uint64_t)n - (fs == 2 ? 256 : 0);
        const int hn = fpos + fs;
        uint32_t byte = 0;
        if (l < 4) byte = (0xFD2FB528u >> (8 * l)) & 0xFFu;
        else if (l == 4) byte = fhd;
        else if (l == 5 && !single) byte = (19 - 10) << 3;  // windowLog 19 (512 KiB), like level 1
        else if (l >= fpos && l < hn) byte = (uint32_t)(fv >> (8 * (l - fpos))) & 0xFFu;
        if (l < hn) dst[l] = (uint8_t)byte;
        op = hn;
    }

    // ---- blocks
    int64_t bs = 0;
    do {
        const int64_t be = bs + BLK < n ? bs + BLK : n;
        const bool last = be == n;
        const int64_t raw = be - bs;
        const int64_t lit0 = op + 3 + 3;  // block header + largest literals header
        int64_t L = 0, ns = 0;
        bool ok = raw > 0;
        // 1. parse; literals straight to dst[lit0 + L]
        {
            int64_t ip = bs, anchor = bs;
            uint32_t miss = 0;
            while (ok && ip + 4 <= be) {
                const uint32_t v = ld32u(src + ip);
                const uint32_t h = hash4(v);
                const int64_t cand = (int64_t)s.table[h];
                s.table[h] = (uint32_t)ip;
                bool hit = cand < ip && ip - cand <= 65535;
                if (hit) hit = ld32u(src + cand) == v;
                if (!hit) {
                    ip += 1 + (miss++ >> 6);
                    continue;
                }
                miss = 0;
                // forward extension from +4, 64 bytes per step, up to the block end
                int64_t ml = 4;
                for (;;) {
                    const int64_t a = ip + ml + l;
                    const bool eq = a < be && src[a] == src[cand + ml + l];
                    const uint64_t ne = ~__ballot(eq);
                    const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                    ml += run;
                    if (run < 64) break;
                }
                // backward catch-up into the pending literals
                int64_t m0 = cand;
                {
                    int64_t lim = ip - anchor;
                    if (m0 < lim) lim = m0;
                    int64_t back = 0;
                    while (back < lim) {
                        const int64_t k = back + 1 + l;
                        const bool eq = k <= lim && src[ip - k] == src[m0 - k];
                        const uint64_t ne = ~__ballot(eq);
                        const int run = ne ? (int)__builtin_ctzll(ne) : 64;
                        back += run;
                        if (run < 64) break;
                    }
                    if (back > lim) back = lim;
                    ip -= back;
                    m0 -= back;
                    ml += back;
                }
                const int64_t ll = ip - anchor;
                copy_bytes(dst, lit0 + L, src, anchor, ll);
                L += ll;
                if (ns >= SEQ_CAP) { ok = false; break; }
                if (l == 0) seq[ns] = (uint64_t)ll | ((uint64_t)ml << 17) | ((uint64_t)(ip - m0) << 35);
                ns++;
                ip += ml;
                anchor = ip;
                if (ip - 2 >= bs && ip + 2 <= n) s.table[hash4(ld32u(src + ip - 2))] = (uint32_t)(ip - 2);
            }
            if (ok) {  // last literals of the block
                copy_bytes(dst, lit0 + L, src, anchor, be - anchor);
                L += be - anchor;
            }
        }
        __threadfence_block();
        // 2./3. headers and the sequences bitstream
        int64_t end = lit0 + L;
        if (ok) {
            // Raw_Literals_Block with the smallest Size_Format (1, 2 or 3 header
            // bytes, like libzstd); the literals move down to follow it
            const int hsz = L < 32 ? 1 : L < 4096 ? 2 : 3;
            const uint32_t lh = hsz == 1   ? (uint32_t)L << 3
                                : hsz == 2 ? (1u << 2) | ((uint32_t)L << 4)
                                           : (3u << 2) | ((uint32_t)L << 4);
            if (hsz < 3) {
                const int64_t to = op + 3 + hsz;
                for (int64_t k = 0; k < L; k += 64) {  // dst < src: ascending chunks are safe
                    uint8_t v = 0;
                    if (k + l < L) v = dst[lit0 + k + l];
                    __builtin_amdgcn_wave_barrier();
                    if (k + l < L) dst[to + k + l] = v;
                }
                end = to + L;
            }
            if (l < hsz) dst[op + 3 + l] = (uint8_t)(lh >> (8 * l));
            if (ns < 128) {
                if (l == 0) dst[end] = (uint8_t)ns;
                end += 1;
            } else if (ns < 0x7F00) {
                if (l == 0) dst[end] = (uint8_t)((ns >> 8) + 128);
                if (l == 1) dst[end + 1] = (uint8_t)(ns & 255);
                end += 2;
            } else {
                const int64_t r = ns - 0x7F00;
                if (l == 0) dst[end] = 255;
                if (l == 1) dst[end + 1] = (uint8_t)(r & 255);
                if (l == 2) dst[end + 2] = (uint8_t)(r >> 8);
                end += 3;
            }
            if (ns > 0) {
                if (l == 0) dst[end] = 0;  // Symbol_Compression_Modes: predefined x3
                end += 1;
                __threadfence_block();
                BitW w;
                w.dst = dst;
                w.wp = end;
                w.lim = op + 3 + raw;  // not smaller than raw -> stored raw anyway
                w.bc = 0;
                w.bp = 0;
                w.ovf = false;
                encode_sequences(s, w, seq, ns);
                end = w.wp;
                if (w.ovf) ok = false;
            }
        }
        const int64_t csize = end - (op + 3);
        __threadfence_block();
        if (ok && csize < raw) {
            put3(dst, op, (uint32_t)((csize << 3) | (2u << 1) | (last ? 1u : 0u)));
            op = end;
        } else {
            put3(dst, op, (uint32_t)((raw << 3) | (last ? 1u : 0u)));  // Raw_Block
            copy_bytes(dst, op + 3, src, bs, raw);
            op += 3 + raw;
        }
        __threadfence_block();
        bs = be;
    } while (bs < n);
    if (l == 0) ret[b] = op <= cap ? (int32_t)op : -2;
}

}  // namespace zstde
}  // namespace jfs

namespace {
struct ZEScratch {
    std::mutex mu;
    uint64_t *d = nullptr;
    size_t cap = 0;  // inputs
};
ZEScratch g_zes[16];
}  // namespace

extern "C" int jfs_launch_zstd_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream) {
    using namespace jfs::zstde;
    if (nblk <= 0) return 0;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 16) return -1;
    ZEScratch &z = g_zes[dev];
    std::lock_guard<std::mutex> lk(z.mu);
    if (z.cap < (size_t)nblk) {
        if (z.d) (void)hipFree(z.d);  // hipFree synchronises with work still using it
        z.d = nullptr;
        z.cap = 0;
        if (hipMalloc((void **)&z.d, (size_t)SCR_PER * (size_t)nblk) != hipSuccess) return -1;
        z.cap = (size_t)nblk;
    }
    hipLaunchKernelGGL(zstd_encode_kernel, dim3(nblk), dim3(64), 0, stream, d_blocks, nblk, d_ret, z.d);
    if (hipGetLastError() != hipSuccess) return -1;
    // the scratch is shared by every launch on this device: finish before it is reused
    return hipStreamSynchronize(stream) == hipSuccess ? 0 : -1;
}
