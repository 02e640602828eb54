/*
 * jfs_gpucodec.h -- C ABI of libjfsgpu.so, the MI355X block-compression engine
 * that drops in under JuiceFS's pkg/compress.
 *
 * Plain C types only (pointers + sizes); no torch / HIP types in signatures.
 * A stream argument is a hipStream_t passed as void* (0 = the library's own
 * per-device stream).
 *
 * Reference interface replaced (file:line in /root/reference):
 *   pkg/compress/compress.go:31-36   type Compressor interface {Name, CompressBound, Compress, Decompress}
 *   pkg/compress/compress.go:39-49   func NewCompressor(algr string) Compressor
 *   pkg/compress/compress.go:51-68   noOp            (Name "Noop")
 *   pkg/compress/compress.go:70-103  ZStandard{1}    (Name "Zstd", level ZSTD_LEVEL=1 :28)
 *   pkg/compress/compress.go:105-125 LZ4             (Name "LZ4")
 * Callers: pkg/chunk/cached_store.go:359,372 (upload), :764,814 (load),
 *          :827,846 (NewCachedStore), cmd/format.go:445 (validation).
 * The cgo binding a maintainer adds on the Go side is shown in INTEGRATION.md.
 */
#ifndef JFS_GPUCODEC_H
#define JFS_GPUCODEC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Codec ids (the three values NewCompressor can return). */
#define JFS_ALGO_NONE 0 /* noOp       compress.go:51  */
#define JFS_ALGO_LZ4 1  /* LZ4{}      compress.go:106 */
#define JFS_ALGO_ZSTD 2 /* ZStandard  compress.go:71  */

/* Status codes returned by the library (int64, all <= JFS_ERR_BASE).  LZ4
 * decompression failures return the raw LZ4_decompress_safe value instead (a
 * negative int32), because lz4.DecompressSafe passes it through to the Go
 * caller (compress.go:124); the two ranges never overlap. */
#define JFS_OK 0
#define JFS_ERR_BASE (-(1LL << 40))
#define JFS_ERR_SHORT_BUFFER (JFS_ERR_BASE - 1)  /* "buffer too short: %d < %d"   compress.go:57,64,88,100 */
#define JFS_ERR_EMPTY_INPUT (JFS_ERR_BASE - 2)   /* "decompress an empty input"   compress.go:122 / zstd ErrEmptySlice */
#define JFS_ERR_CORRUPT (JFS_ERR_BASE - 3)       /* malformed Zstd frame (ZSTD_decompress error) */
#define JFS_ERR_COMPRESS_FAIL (JFS_ERR_BASE - 4) /* LZ4_compress_default returned 0 */
#define JFS_ERR_UNSUPPORTED (JFS_ERR_BASE - 5)   /* operation not available in this build */
#define JFS_ERR_NO_DEVICE (JFS_ERR_BASE - 6)     /* no usable gfx950 device; the library never falls back to CPU */
#define JFS_ERR_INVALID (JFS_ERR_BASE - 7)       /* bad argument (unknown algo, negative size, ...) */
#define JFS_ERR_HIP (JFS_ERR_BASE - 8)           /* HIP runtime failure */
#define JFS_ERR_NO_MEMORY (JFS_ERR_BASE - 9)     /* pinned/HBM staging for this block could not be allocated */
#define JFS_ERR_AUTH (JFS_ERR_BASE - 10)         /* "cipher: message authentication failed" (aead.Open, encrypt.go:283) */

/* ---- Compressor surface (one synchronous call per block) ---------------- */

/* NewCompressor(algr): case-insensitive "zstd" | "lz4" | "none" | "" -> algo id,
 * anything else -> -1 (the Go factory's nil).                 compress.go:39-49 */
int jfs_codec_from_name(const char *name);

/* Name(): "Noop" / "LZ4" / "Zstd"; NULL for an unknown id.
 *                                                compress.go:53,76,109 */
const char *jfs_codec_name(int algo);

/* CompressBound(n).  LZ4: n>0x7E000000 ? 0 : n + n/255 + 16 (compress.go:112);
 * Zstd: n + n>>8 + (n < 128K ? (128K-n)>>11 : 0) (compress.go:79); none: n. */
int64_t jfs_compress_bound(int algo, int64_t n);

/* Compress(dst, src) -> bytes written (>=0) or a JFS_ERR_* code.
 * dst_cap is len(dst) for LZ4/none and cap(dst) for Zstd (DataDog/zstd writes
 * into dst[:cap]; compress.go:83-89).  LZ4 output is byte-identical to
 * LZ4_compress_default; a dst smaller than the compressed size fails
 * (JFS_ERR_COMPRESS_FAIL), like lz4.CompressDefault returning 0.  Zstd: one
 * RFC 8878 frame (FCS present, no checksum), never larger than
 * CompressBound; dst_cap < CompressBound(n) -> JFS_ERR_SHORT_BUFFER, the
 * "buffer too short" of compress.go:86-89. */
int64_t jfs_compress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n);

/* Decompress(dst, src) -> bytes written (>=0) or <0.
 * LZ4: empty src -> JFS_ERR_EMPTY_INPUT (compress.go:121-123); otherwise the
 * exact LZ4_decompress_safe(src, dst, n, dst_cap) result.
 * Zstd: empty src -> JFS_ERR_EMPTY_INPUT; frame(s) larger than dst_cap ->
 * JFS_ERR_SHORT_BUFFER (compress.go:99-101); malformed -> JFS_ERR_CORRUPT. */
int64_t jfs_decompress(int algo, uint8_t *dst, int64_t dst_cap, const uint8_t *src, int64_t n);

/* ---- Batch surface (host buffers; FillCache / compaction / aggregator) ----
 * Blocks are independent; they are dealt round-robin over the devices in
 * device_mask (bit d = device d; 0 = all visible devices) and staged through
 * pinned host memory with async copies.  out_n[i] receives what the
 * single-block call would have returned for block i.  Errors are per block: a
 * batch that fails as a whole (staging allocation, copy or launch failure) is
 * re-run block by block, so only the blocks that fail on their own report
 * JFS_ERR_NO_MEMORY / JFS_ERR_HIP.  Returns JFS_OK, or JFS_ERR_INVALID /
 * JFS_ERR_NO_DEVICE for a call that cannot run at all.  The calling thread's
 * current HIP device is unchanged on return. */
typedef struct jfs_iov {
    const uint8_t *src;
    int64_t src_len;
    uint8_t *dst;
    int64_t dst_cap;
} jfs_iov;

int64_t jfs_compress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask);
/* jfs_compress_batch plus crc[i] = crc32.Update(0, crc32c, dst[0:out_n[i]]) -- the
 * object checksum generateChecksum attaches to the PUT (pkg/object/checksum.go:
 * 30-45) -- computed on the GPU over the compressed payload before it leaves
 * HBM (0 for a block that failed).  For "none" the payload is the block itself. */
int64_t jfs_compress_batch_crc(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t *crc,
                               uint32_t device_mask);
int64_t jfs_decompress_batch(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint32_t device_mask);
/* Mixed-codec batches (algo[i] per block: a chunk store reading objects written
 * under different codecs).  Each codec's blocks form
 * one jfs_{de,}compress_batch call; decode calls run at once, so the codecs
 * share every device's lanes instead of queueing behind one another (encode
 * calls run in turn: the encoders slow each other down).  Per-block
 * results as jfs_{de,}compress_batch (JFS_ERR_INVALID for an unknown algo[i]);
 * returns JFS_OK or the first failing codec call's whole-call error, which is
 * then also written to out_n[i] of every block of that codec. */
int64_t jfs_compress_batch_mixed(const int32_t *algo, int nblk, const jfs_iov *iov, int64_t *out_n,
                                 uint32_t device_mask);
int64_t jfs_decompress_batch_mixed(const int32_t *algo, int nblk, const jfs_iov *iov, int64_t *out_n,
                                   uint32_t device_mask);
/* jfs_decompress_batch plus, for each block with csum[i] != NULL, the disk-cache
 * checksum of the decoded block -- what cacheStore.add writes beside it
 * (pkg/chunk/disk_cache.go:536-537, checksum() of disk_cache_file.go:139-152):
 * the big-endian CRC-32C of every 32 KiB piece, ((n-1)/32768+1)*4 bytes for
 * n = out_n[i] decoded bytes (4 zero bytes for n = 0), computed on the GPU
 * before the block leaves HBM.  csum[i] must hold ((dst_cap-1)/32768+1)*4
 * bytes; nothing is written for a block that fails. */
int64_t jfs_decompress_batch_csum(int algo, int nblk, const jfs_iov *iov, int64_t *out_n, uint8_t *const *csum,
                                  uint32_t device_mask);
/* The batch calls' device dealing policy, exposed for
 * schedulers and tests: out_dev[i] in [0, ndev) for blocks of cost[i] (the
 * library uses src_len + dst_cap + 4096): longest-first greedy onto the least
 * loaded device, so no device ends more than one block above another. */
void jfs_deal_plan(const int64_t *cost, int n, int ndev, int32_t *out_dev);

/* ---- Encrypted objects (host buffers): compress + seal, open + decompress --
 * The PUT path of an encrypted volume is Compress (cached_store.go:372) and
 * then dataEncryptor.Encrypt (pkg/object/encrypt.go:226-257), which writes
 *     be16(len(wrapped)) | u8(len(nonce)) | wrapped key | nonce | sealed
 * with sealed = aead.Seal(nonce, compressed, nil) = ciphertext || 16-byte tag.
 * jfs_compress_seal_batch does both on the GPU per block: iov[i].src is the raw
 * block, iov[i].dst receives the whole envelope (dst_cap must be at least
 * jfs_envelope_bound), out_n[i] = envelope bytes or the codec's error.  The
 * random data key and nonce and the key wrap (RSA / SM2, keyEncryptor) are
 * the caller's: p[i] carries them.  algo may be JFS_ALGO_NONE (encryption
 * without compression).
 * The GET path is Decrypt (:259-284) then Decompress (:814):
 * jfs_open_decompress_batch takes the envelope in iov[i].src and the data key
 * the caller unwrapped from its header (jfs_envelope_parse) in keys[i], and
 * writes the block to iov[i].dst: out_n[i] = what jfs_decompress returns, or
 * JFS_ERR_AUTH when the tag does not verify, or JFS_ERR_CORRUPT for a
 * malformed header.  Errors are per block; the call returns JFS_OK,
 * JFS_ERR_INVALID or JFS_ERR_NO_DEVICE like the plain batch calls. */
typedef struct jfs_seal_param {
    const uint8_t *key;     /* data key, jfs_cipher_key_size(cipher) bytes */
    const uint8_t *nonce;   /* 12 bytes */
    const uint8_t *wrapped; /* keyEncryptor.Encrypt(key) (encrypt.go:234) */
    int32_t wrapped_len;    /* 0 .. 65535 */
    int32_t reserved;
} jfs_seal_param;

/* 3 + wrapped_len + 12 + CompressBound(n) (n for "none") + 16 */
int64_t jfs_envelope_bound(int algo, int64_t n, int32_t wrapped_len);
/* Decrypt's header checks (encrypt.go:260-267): returns the offset of the sealed
 * payload and the wrapped key / nonce positions, or JFS_ERR_CORRUPT when
 * n < 3 or 3 + wrapped_len + nonce_len >= n. */
int64_t jfs_envelope_parse(const uint8_t *src, int64_t n, int64_t *wrapped_off, int64_t *wrapped_len,
                           int64_t *nonce_off, int64_t *nonce_len);
/* crc (optional, may be NULL): per block the CRC-32C of the whole envelope
 * (generateChecksum of the PUT payload), computed on the GPU. */
int64_t jfs_compress_seal_batch(int algo, int cipher, int nblk, const jfs_iov *iov, const jfs_seal_param *p,
                                int64_t *out_n, uint32_t *crc, uint32_t device_mask);
int64_t jfs_open_decompress_batch(int algo, int cipher, int nblk, const jfs_iov *iov, const uint8_t *const *keys,
                                  int64_t *out_n, uint32_t device_mask);

/* ---- Device-resident surface (inputs/outputs already in HBM) ------------
 * One descriptor per block; all pointers are device pointers on the calling
 * thread's current device, which must be a device this library selected
 * (gfx950, in JFS_GPU_DEVICES; else JFS_ERR_NO_DEVICE), and `stream`
 * (0 = the null stream) belongs to it.  ret[i] is written with the
 * single-block result -- exactly the value jfs_decompress/jfs_compress's
 * codec call would produce for that block (see each call below); no other
 * value is ever written.  The LZ4 calls only enqueue work on `stream`.
 * jfs_zstd_decompress_device enqueues too, but first waits on the host for
 * its header-scan kernels (microseconds after the work already on `stream`)
 * so it can size its scratch: it never asks the caller to resubmit.
 * jfs_zstd_compress_device is host-synchronous (per-device scratch, locked). */
typedef struct jfs_dev_block {
    const uint8_t *src;
    uint8_t *dst;
    int32_t src_len;
    int32_t dst_cap;
} jfs_dev_block;

/* ret[i] = LZ4_decompress_safe(src, dst, src_len, dst_cap): bytes written, or
 * its negative error value. */
int64_t jfs_lz4_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream);
/* The same result for a FEW blocks at low latency (cachedStore.load decodes one
 * block per cache miss, pkg/chunk/cached_store.go:755-823): every block is
 * spread over the whole GPU instead of one workgroup.  src_len / dst_cap are
 * HOST copies of the descriptors' sizes (they size the launch without a device
 * round trip) and must match d_blocks.  Asynchronous on `stream`; per-device
 * scratch of about 4 bytes per dst_cap byte, reused across calls.  Best below
 * ~128-192 blocks of 4 MiB; jfs_lz4_decompress_device is faster for large batches. */
int64_t jfs_lz4_decompress_device_small(const jfs_dev_block *d_blocks, const int32_t *src_len, const int32_t *dst_cap,
                                        int nblk, int32_t *d_ret, void *stream);
/* Diagnostics for the small-batch path (used by it, by jfs_decompress and by
 * small jfs_decompress_batch calls), six counters: out[0] = blocks it decoded
 * itself, out[1] = blocks it handed to the one-workgroup kernel (inputs outside
 * its proven cases), and why: out[2] the token-chain fix-up did not converge
 * (e.g. literal runs spanning many segments), out[3] the byte-origin pointer
 * jumping did not converge, out[4] a token outside the proven acceptance
 * conditions (malformed or edge-of-buffer), out[5] no final literal run; on
 * the current device since the last reset.  Synchronous; 0 on success. */
int jfs_lz4_split_counts(uint64_t *out, int reset);
/* ret[i] = LZ4_compress_default(src, dst, src_len, dst_cap): compressed size,
 * or 0 when it does not fit dst_cap. */
int64_t jfs_lz4_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream);
/* The same bytes as jfs_lz4_compress_device for few blocks (one-call
 * Compress under cachedStore.upload, pkg/chunk/cached_store.go:372): every
 * block is cut into segments that are parsed at once and re-parsed, each from
 * the state the segment before it stopped in, until nothing changes (then the
 * result is the serial parse, byte for byte); blocks that do not settle take
 * the serial kernel.  src_len = HOST copies of the descriptors' src_len.
 * Asynchronous on `stream`; per-device scratch of about 4 bytes per input
 * byte, reused across calls.  jfs_compress / small jfs_compress_batch calls use
 * it below JFS_LZ4E_SEG_MAX blocks (default 256). */
int64_t jfs_lz4_compress_device_small(const jfs_dev_block *d_blocks, const int32_t *src_len, int nblk, int32_t *d_ret,
                                      void *stream);
/* Diagnostics of the segment encoder: out[r] (r = 1..16) = blocks whose
 * segments settled after r rounds, out[0] = blocks handed to the serial kernel
 * (not settled within JFS_LZ4E_SEG_ROUNDS, default 8, or a segment with too
 * many sequences); on the current device since the last reset.  Synchronous. */
int jfs_lz4_eseg_counts(uint64_t *out, int reset);
/* ret[i]: decoded bytes, -1 malformed frame (ZSTD error), -2 output larger
 * than dst_cap ("Destination buffer is too small"), -3 src size incorrect
 * (truncated / trailing bytes). */
int64_t jfs_zstd_decompress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream);
/* Batches of at most JFS_ZSTD_SPLIT_MAX inputs (default 128; also the batch
 * ABI's staged chunks and jfs_decompress) decode one workgroup per Zstd block
 * with an origin-map replay; an input outside that path's proven cases (not
 * exactly one frame, a checksum, any error) is replayed by the exact one-wave
 * kernel -- same results either way.  Diagnostics: out[0] = inputs the
 * small-batch path replayed itself, out[1] = inputs it handed over; on the
 * current device since the last reset.  Synchronous; 0 on success. */
int jfs_zstd_split_counts(uint64_t *out, int reset);
/* Zstd frame per block; ret[i] = frame size, or -2 when dst_cap < CompressBound(src_len).
 * Synchronous with respect to `stream` (it uses per-device scratch). */
int64_t jfs_zstd_compress_device(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *stream);

/* CRC-32C (Castagnoli) of device-resident blocks.
 * d_blocks[i].src / src_len: the data.  d_crc[i] (if d_crc != NULL) receives
 * crc32.Update(0, crc32c, data), the object checksum of
 * pkg/object/checksum.go:30-45.  If seg_bytes > 0 (a multiple of 4096; JuiceFS
 * uses 32768), d_blocks[i].dst receives the disk-cache checksum layout of
 * pkg/chunk/disk_cache_file.go:139-152: the big-endian CRC-32C of every
 * seg_bytes piece, ((len-1)/seg_bytes+1)*4 bytes (4 zero bytes for len 0);
 * dst_cap must hold them.  d_ret[i] (if non-NULL) = bytes written to dst, or
 * -1 for a bad descriptor.  Asynchronous on `stream`. */
int64_t jfs_crc32c_device(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes, uint32_t *d_crc,
                          int32_t *d_ret, void *stream);

/* AES-256-GCM of device-resident blocks: the AEAD of
 * pkg/object/encrypt.go dataEncryptor for AES256GCM_RSA (aes.NewCipher(key) +
 * cipher.NewGCM, :178-189): 32-byte key, 12-byte nonce, 16-byte tag, no
 * additional data.  Seal (Encrypt :226-257): dst = ciphertext || tag,
 * ret = src_len + 16 (dst_cap must hold it).  Open (Decrypt :259-284):
 * src = ciphertext || tag, dst = plaintext, ret = src_len - 16, or -1 when the
 * tag does not verify ("cipher: message authentication failed"; dst[0, n)
 * is then zeroed, as Go's gcm.Open clears its output).  ret = -2 for a bad descriptor.  The random key/nonce, the
 * RSA wrap of the key and the object header (:230-252) are the caller's.
 * Asynchronous on `stream`; key and nonce are device pointers. */
typedef struct jfs_aead_block {
    const uint8_t *src;
    uint8_t *dst;
    int32_t src_len;
    int32_t dst_cap;
    const uint8_t *key;   /* 32 bytes */
    const uint8_t *nonce; /* 12 bytes */
} jfs_aead_block;

int64_t jfs_aes256gcm_seal_device(const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream);
int64_t jfs_aes256gcm_open_device(const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream);

/* The three data ciphers of NewDataEncryptor (pkg/object/encrypt.go:176-202).
 * Same seal/open contract as above (ret, zeroed dst on a failed open, no
 * additional data); the key is jfs_cipher_key_size(cipher) bytes. */
#define JFS_CIPHER_AES256GCM 0        /* "aes256gcm-rsa" (and ""), encrypt.go:179-188: 32-byte key */
#define JFS_CIPHER_CHACHA20POLY1305 1 /* "chacha20-rsa", encrypt.go:190: 32-byte key (RFC 8439) */
#define JFS_CIPHER_SM4GCM 2           /* "sm4gcm", encrypt.go:192-201: 16-byte key (GB/T 32907 + GCM) */
/* NewDataEncryptor's names -> cipher id, or -1 ("unsupport cipher") */
int jfs_cipher_from_name(const char *name);
/* keyLen of dataEncryptor (32 / 32 / 16), or -1 */
int jfs_cipher_key_size(int cipher);
int64_t jfs_aead_seal_device(int cipher, const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream);
int64_t jfs_aead_open_device(int cipher, const jfs_aead_block *d_blocks, int nblk, int32_t *d_ret, void *stream);

/* Fused object paths (compression runs before encryption on PUT and after
 * decryption on GET, cmd/format.go:289-302, docs internals.md:920), chained on
 * `stream` with no host round trip: the second kernel reads each block's
 * length from the first kernel's results on the device.
 *   compress -> seal: d_comp[i] LZ4-compresses into an intermediate buffer
 *     (d_ret_comp[i] = LZ4 result); d_aead[i].src must be that buffer (its
 *     src_len is ignored) and is sealed into d_aead[i].dst; d_ret[i] = sealed
 *     bytes, or JFS_CHAIN_FAILED (INT32_MIN) when the compression failed.
 *   open -> decompress: d_aead[i] opens into an intermediate buffer
 *     (d_ret_open[i] = plaintext length or -1); d_dec[i].src must be that
 *     buffer (its src_len is ignored); d_ret[i] = the LZ4_decompress_safe
 *     result, or INT32_MIN when the tag did not verify. */
int64_t jfs_lz4_compress_seal_device(const jfs_dev_block *d_comp, const jfs_aead_block *d_aead, int nblk,
                                     int32_t *d_ret_comp, int32_t *d_ret, void *stream);
int64_t jfs_open_lz4_decompress_device(const jfs_aead_block *d_aead, const jfs_dev_block *d_dec, int nblk,
                                       int32_t *d_ret_open, int32_t *d_ret, void *stream);

/* ---- Runtime / utilities ------------------------------------------------- */

/* Number of usable gfx950 devices (0 when none; never an error).  Only the
 * devices JFS_GPU_DEVICES selects count (a comma list of ordinals such as
 * "0,2,5", a mask such as "0x25", or "all" = the default). */
int jfs_device_count(void);

/* Codec selector, read once from JFS_GPU_CODEC:
 *   "off"   -> JFS_MODE_OFF: the library reports no device; every GPU entry
 *              point returns JFS_ERR_NO_DEVICE and the Go adapter keeps the
 *              CPU codecs of compress.go (NewCompressor unchanged);
 *   "auto"  -> JFS_MODE_AUTO (default, also for unknown values): the adapter
 *              uses this library when jfs_device_count() > 0, else the CPU
 *              codecs;
 *   "force" -> JFS_MODE_FORCE: the adapter must use this library and fail at
 *              start-up when jfs_device_count() == 0.
 * The library itself never runs a CPU codec in any mode. */
#define JFS_MODE_OFF 0
#define JFS_MODE_AUTO 1
#define JFS_MODE_FORCE 2
int jfs_gpu_mode(void);

/* Per-codec counters (the data behind cachedStore's object_request_data_bytes
 * and block-size metrics, cached_store.go:931-974).  Index algo * 2 + dir,
 * dir 0 = compress, 1 = decompress; 6 entries.  Host-path calls (one-call and
 * batch) count blocks, bytes and errors per block; device-resident launches
 * count only calls and blocks (their results stay in HBM). */
typedef struct jfs_op_stats {
    uint64_t calls;     /* API calls */
    uint64_t blocks;    /* blocks submitted */
    uint64_t bytes_in;  /* input bytes of host-path blocks that succeeded */
    uint64_t bytes_out; /* output bytes of host-path blocks that succeeded */
    uint64_t errors;    /* host-path blocks that returned an error code */
    uint64_t nanos;     /* wall time spent inside host-path calls */
    uint64_t batches;   /* device batches the host path ran (coalesced one-call
                           batches, or per-device parts of a jfs_*_batch call) */
} jfs_op_stats;
#define JFS_STATS_N 6
/* Copy min(n, JFS_STATS_N) entries to out; returns JFS_STATS_N. */
int jfs_stats(jfs_op_stats *out, int n);
void jfs_stats_reset(void);  /* also zeroes the per-device counters below */
/* Per-device host-path counters (where the round-robin deal put
 * the blocks): one entry per usable device, in jfs_device_count() order. */
typedef struct jfs_device_stat {
    int32_t device;   /* HIP device ordinal */
    int32_t pad_;
    uint64_t batches; /* device batches run */
    uint64_t blocks;  /* blocks in them */
} jfs_device_stat;
/* Copy min(n, devices) entries to out; returns the number of devices. */
int jfs_device_stats(jfs_device_stat *out, int n);
/* Free the batch path's pinned host + HBM staging now (it is also released
 * after JFS_STAGING_IDLE_MS, default 15000, of no batch activity). */
void jfs_release_staging(void);
/* Library version string. */
const char *jfs_version(void);

/* Synthetic benchmark input: block i of class cls
 * ('T','Z','R') with seed base+i, each `block_bytes` long, written
 * back-to-back at d_dst (device pointer) on `stream`.  Host twin below. */
int64_t jfs_gen_blocks_device(uint8_t *d_dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                              void *stream);
void jfs_gen_block_host(uint8_t *dst, int64_t n, char cls, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif /* JFS_GPUCODEC_H */
