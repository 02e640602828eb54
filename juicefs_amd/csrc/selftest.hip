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

#ifdef JFS_DIAG  // diagnostic builds only (scripts/build_variant.sh diag -DJFS_DIAG), never in the product .so
// Probe: does this device honour unaligned LDS b128/b64 reads (SH_MEM_CONFIG
// alignment mode)?  out[l*4 + j] = dword j of ds_read_b128 at byte l (l < 16),
// out[64 + l*2 + j] = dword j of ds_read_b64 at byte 4*l.
namespace jfs {
__global__ void lds_align_probe_kernel(uint32_t *out) {
    __shared__ uint8_t buf[256];
    const int l = lane_id();
    for (int k = l; k < 256; k += 64) buf[k] = (uint8_t)k;
    __syncthreads();
    uint32_t base = (uint32_t)(uintptr_t)buf;
    if (l < 16) {
        uint4 v;
        uint32_t a = base + (uint32_t)l;
        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        out[l * 4 + 0] = v.x; out[l * 4 + 1] = v.y; out[l * 4 + 2] = v.z; out[l * 4 + 3] = v.w;
    }
    if (l < 16) {
        uint2 v;
        uint32_t a = base + 4u * (uint32_t)l;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        out[64 + l * 2] = v.x; out[64 + l * 2 + 1] = v.y;
    }
}
}  // namespace jfs

extern "C" int jfs_selftest_lds_align(uint32_t *d_out) {
    hipLaunchKernelGGL(jfs::lds_align_probe_kernel, dim3(1), dim3(64), 0, 0, d_out);
    if (hipGetLastError() != hipSuccess) return -1;
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}
#endif  // JFS_DIAG
