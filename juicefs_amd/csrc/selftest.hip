// Self-test kernel for the wave64 primitives in wave.cuh (exported for the GPU
// test suite: tests/test_wave_gpu.py).  Not on the codec path.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jfs_internal.h"
#include "wave.cuh"

namespace jfs {
__global__ void wave_selftest_kernel(const uint32_t *in, uint32_t *out) {
    const int l = lane_id();
    uint32_t v = in[l];
    out[0 * 64 + l] = dpp_scan_add(v);
    out[1 * 64 + l] = dpp_scan_max(v);
    out[2 * 64 + l] = dpp_scan_min(v);
    out[3 * 64 + l] = dpp_shift_up(v, 12345u);
    out[4 * 64 + l] = dwave_min(v);
    out[5 * 64 + l] = dwave_max(v);
    out[6 * 64 + l] = dwave_sum(v);
    uint32_t tot;
    out[7 * 64 + l] = wave_scan_excl(v, &tot);
}
}  // namespace jfs

// in: 64 u32 (device), out: 8*64 u32 (device); synchronous
extern "C" int jfs_selftest_wave(const uint32_t *d_in, uint32_t *d_out) {
    hipLaunchKernelGGL(jfs::wave_selftest_kernel, dim3(1), dim3(64), 0, 0, d_in, d_out);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
