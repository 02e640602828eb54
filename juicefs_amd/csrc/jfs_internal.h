// Internal declarations shared by the HIP translation units of libjfsgpu.so.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/jfs_gpucodec.h"

extern "C" {
int jfs_launch_lz4_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream);
int jfs_launch_lz4_encode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, hipStream_t stream);
int jfs_launch_zstd_decode(const jfs_dev_block *d_blocks, int nblk, int32_t *d_ret, uint8_t *d_scratch,
                           hipStream_t stream);
int jfs_launch_gen(uint8_t *d_dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                   const uint8_t *d_vocab, hipStream_t stream);
}
