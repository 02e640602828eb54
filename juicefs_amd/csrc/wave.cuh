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

namespace jfs {
// ---- DPP (no LDS round trip) wave64 scans / reductions ---------------------
// row_shr:n = 0x110+n, row_bcast:15 = 0x142, row_bcast:31 = 0x143, wave_shr:1 = 0x138
__device__ __forceinline__ uint32_t dpp_scan_add(uint32_t v) {  // inclusive
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return v;
}
__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
__device__ __forceinline__ uint32_t dpp_scan_max(uint32_t v) {  // inclusive, identity 0
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, true));
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, true));
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, true));
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, true));
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false));
    v = umax32(v, __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false));
    return v;
}
__device__ __forceinline__ uint32_t dpp_scan_min(uint32_t v) {  // inclusive, identity ~0
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x111, 0xF, 0xF, false));
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x112, 0xF, 0xF, false));
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x114, 0xF, 0xF, false));
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x118, 0xF, 0xF, false));
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x142, 0xA, 0xF, false));
    v = umin32(v, __builtin_amdgcn_update_dpp(~0u, v, 0x143, 0xC, 0xF, false));
    return v;
}
// value of lane l-1 (lane 0 gets `first`): one DPP wave_shr:1 (GFX9 DPP;
// lane 0 has no source and keeps `old`)
__device__ __forceinline__ uint32_t dpp_shift_up(uint32_t v, uint32_t first) {
    return __builtin_amdgcn_update_dpp(first, v, 0x138, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t readlane(uint32_t v, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l); }
__device__ __forceinline__ uint32_t dwave_min(uint32_t v) { return readlane(dpp_scan_min(v), 63); }
__device__ __forceinline__ uint32_t dwave_max(uint32_t v) { return readlane(dpp_scan_max(v), 63); }
__device__ __forceinline__ uint32_t dwave_sum(uint32_t v) { return readlane(dpp_scan_add(v), 63); }
}  // namespace jfs
