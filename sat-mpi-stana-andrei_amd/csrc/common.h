// common.h -- shared host/device helpers for the satmi HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "satmi.h"

namespace satmi {

// ---------------------------------------------------------------- host side
void set_error(const std::string &msg);
int hip_fail(hipError_t e, const char *what);

#define SATMI_HIP(call)                                        \
    do {                                                       \
        hipError_t _e = (call);                                \
        if (_e != hipSuccess) return ::satmi::hip_fail(_e, #call); \
    } while (0)

// ---------------------------------------------------------------- wave64 helpers
// One CDNA wavefront = 64 lanes.  The DPLL kernel runs one instance per wave;
// control flow is wave-uniform and lanes cooperate on clause / variable scans.
__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Order LDS traffic between lanes of the same wave (the wave executes in
// order; this stops the compiler from caching/reordering across it).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int uniform_i32(int x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint32_t uniform_u32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)x);
}

__device__ __forceinline__ int wave_min_i32(int x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) x = min(x, __shfl_xor(x, o, 64));
    return uniform_i32(x);
}

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t x) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        uint64_t y = __shfl_xor(x, o, 64);
        x = x > y ? x : y;
    }
    uint32_t lo = uniform_u32((uint32_t)x), hi = uniform_u32((uint32_t)(x >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int x) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        int y = __shfl_up(x, o, 64);
        if (l >= o) x += y;
    }
    return x;
}

}  // namespace satmi
