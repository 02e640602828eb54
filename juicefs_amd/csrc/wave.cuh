// Wave64 helpers shared by the codec kernels (gfx950: 64-lane wavefronts).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace jfs {

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
        v = w < v ? w : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
        v = w > v ? w : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
    return v;
}

// Exclusive prefix sum over lanes in lane order; *total = sum of all lanes.
__device__ __forceinline__ uint32_t wave_scan_excl(uint32_t v, uint32_t *total) {
    const int l = lane_id();
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
        if (l >= o) x += y;
    }
    *total = (uint32_t)__shfl((int)x, 63, 64);
    return x - v;
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

__device__ __forceinline__ uint32_t lane_read(uint32_t v, int lane) {
    return (uint32_t)__shfl((int)v, lane, 64);
}

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace jfs
