// Synthetic benchmark-input generator kernel.
// One thread per block (the text generator is a sequential stream), writing
// 16-byte chunks.  Input generation only -- not part of the codec path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "blockgen.h"
#include "jfs_internal.h"

namespace jfs {

struct Emit16 {
    uint8_t *out;
    uint32_t w[4];
    int k;
    int64_t pos;
    __device__ void operator()(uint8_t b) {
        int wi = k >> 2, sh = (k & 3) * 8;
        w[wi] = (k & 3) ? (w[wi] | ((uint32_t)b << sh)) : (uint32_t)b;
        if (++k == 16) {
            *(uint4 *)(out + pos) = make_uint4(w[0], w[1], w[2], w[3]);
            pos += 16;
            k = 0;
        }
    }
};

struct Emit1 {
    uint8_t *out;
    int64_t pos;
    __device__ void operator()(uint8_t b) { out[pos++] = b; }
};

__global__ void gen_kernel(uint8_t *dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                           const uint8_t *vocab) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    uint8_t *out = dst + (int64_t)b * block_bytes;
    if ((((uintptr_t)out) & 15) == 0 && (block_bytes & 15) == 0) {
        Emit16 e{out, {0, 0, 0, 0}, 0, 0};
        jfs_gen_stream(vocab, cls, seed_base + (uint64_t)b, block_bytes, e);
    } else {
        Emit1 e{out, 0};
        jfs_gen_stream(vocab, cls, seed_base + (uint64_t)b, block_bytes, e);
    }
}

}  // namespace jfs

extern "C" int jfs_launch_gen(uint8_t *d_dst, int nblk, int64_t block_bytes, char cls, uint64_t seed_base,
                              const uint8_t *d_vocab, hipStream_t stream) {
    if (nblk <= 0) return 0;
    int tpb = 1;  // one single-lane wave per block: the text stream is branchy, lanes would diverge
    hipLaunchKernelGGL(jfs::gen_kernel, dim3((nblk + tpb - 1) / tpb), dim3(tpb), 0, stream, d_dst, nblk, block_bytes,
                       cls, seed_base, d_vocab);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}
