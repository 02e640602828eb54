// Internal declarations shared by the HIP translation units of libjfsgpu.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/jfs_gpucodec.h"

// Explicit global (address space 1) pointer types: generic pointers compile to
// flat_* instructions, which count on both vmcnt and lgkmcnt and force the
// compiler to drain LDS traffic around every HBM access.
// (The host compilation pass of the same source sees plain types.)
#if defined(__HIP_DEVICE_COMPILE__)
#define JFS_GLOBAL __attribute__((address_space(1)))
#else
#define JFS_GLOBAL
#endif
typedef JFS_GLOBAL uint8_t g_u8;
typedef JFS_GLOBAL const uint8_t gc_u8;
typedef JFS_GLOBAL uint32_t g_u32;
typedef JFS_GLOBAL const uint32_t gc_u32;
typedef JFS_GLOBAL uint4 g_u4;
typedef JFS_GLOBAL const uint4 gc_u4;
typedef JFS_GLOBAL const uint2 gc_u2;
typedef JFS_GLOBAL const jfs_dev_block gc_blk;

extern "C" {
int jfs_launch_lz4_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream);
int jfs_launch_lz4_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream);
// segment-parallel LZ4 encode (same bytes as jfs_launch_lz4_encode); lens = the
// blocks' src_len on the host; scratch of jfs_lz4_eseg_scratch_bytes
int64_t jfs_lz4_eseg_scratch_bytes(int nblk, const int32_t *lens);
int jfs_launch_lz4_encode_seg(const jfs_dev_block *d_blocks, int nblk, const int32_t *lens, int32_t *d_ret,
                              void *scratch, int64_t scratch_cap, hipStream_t stream);
int jfs_launch_zstd_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream);
int jfs_launch_zstd_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, uint8_t *d_scratch,
                           hipStream_t stream);
// d_split: the small-batch path's scratch (jfs_zstd_split_bytes), or null;
// tot: jfs_zstd_plan_host's six totals
int jfs_launch_zstd_decode_planned(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, void *d_info,
                                   uint8_t *d_lit, uint16_t *d_tabs, void *d_items, void *d_split,
                                   const uint64_t *tot, hipStream_t stream);
size_t jfs_zstd_info_bytes(void);
// totals[6]: items, literal bytes, table cells, blocks, origin entries, largest dst_cap
void jfs_zstd_plan_host(const uint8_t *const *srcs, const int32_t *lens, const int32_t *caps, int nblk, void *info_out,
                        uint64_t *totals);
int jfs_zstd_split_ok(int nblk, const uint64_t *tot);  // the small-batch path takes this batch
int64_t jfs_zstd_split_bytes(int nblk, const uint64_t *tot);
int jfs_launch_crc32c(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes, uint32_t *d_crc, int32_t *d_ret,
                      hipStream_t stream);
int jfs_launch_crc32c_lens(const jfs_dev_block *d_blocks, int nblk, const int32_t *d_lens, const uint32_t *d_seeds,
                           uint32_t *d_crc, hipStream_t stream);
// per-seg_bytes checksums (jfs_crc32c_device's dst layout) of device blocks
// whose length the previous kernel wrote (lens; < 0: it failed, nothing written)
int jfs_launch_crc32c_segs_lens(const jfs_dev_block *d_blocks, int nblk, int32_t seg_bytes, const int32_t *d_lens,
                                hipStream_t stream);
int jfs_launch_aes256gcm(const jfs_aead_block *d_blocks, int nblk, int mode, int32_t *d_ret, const int32_t *d_lens,
                         hipStream_t stream);
int jfs_launch_aead(int cipher, const jfs_aead_block *d_blocks, int nblk, int mode, int32_t *d_ret,
                    const int32_t *d_lens, hipStream_t stream);
int jfs_launch_lz4_decode_lens(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, const int32_t *d_lens,
                               hipStream_t stream);
int jfs_launch_lz4_decode_todo(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, const int32_t *d_todo,
                               hipStream_t stream);
// small-batch LZ4 decode (lz4_split.hip): compressed bytes per segment (one
// lane each), scratch bytes for these blocks, and
// the launch (nseg_all = sum of ceil(src_len / 256), max_cap = largest dst_cap,
// norg_all = sum of dst_cap rounded up to 4: the host sizes the scratch with them)
#define JFS_LZ4_SPLIT_SEG 256
int64_t jfs_lz4_split_scratch_bytes(int nb, const int32_t *src_len, const int32_t *cap);
int jfs_launch_lz4_split(const jfs_dev_block *d_desc, int nb, int32_t *d_ret, void *d_scratch, int64_t nseg_all,
                         int64_t max_cap, int64_t norg_all, hipStream_t st);
// ret value of a fused chain's second step when its first step failed
#define JFS_CHAIN_FAILED (-2147483647 - 1)
int jfs_launch_gen(uint8_t *d_dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                   const uint8_t *d_vocab, hipStream_t stream);
}
