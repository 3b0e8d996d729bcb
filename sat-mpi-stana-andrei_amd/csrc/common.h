// common.h -- shared host/device helpers for the satmi HIP library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <climits>
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
// The same, recomputed where it is written: for rarely taken paths inside hot
// loops, so the compiler cannot hoist lane-dependent addresses of the rare
// path out of the loop (hoisted, they hold VGPRs across the whole loop).
__device__ __forceinline__ int lane_id_here() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const int l = lane_id();
    return l == 0 ? 0ull : (~0ull >> (64 - l));
}

// Launch span of a persistent DPLL grid, kept beside its work counter
// (work[0] = counter, work_span = (uint64_t *)work + 1): span[0] = ~(earliest
// wave start), span[1] = latest wave end, both s_memrealtime ticks (the
// constant wall clock); zeroed with the counter before each launch.
__device__ __forceinline__ void span_begin(uint32_t *work) {
    if (lane_id() == 0) atomicMax((unsigned long long *)work + 1, ~(unsigned long long)__builtin_amdgcn_s_memrealtime());
}
__device__ __forceinline__ void span_end(uint32_t *work) {
    if (lane_id() == 0) atomicMax((unsigned long long *)work + 2, (unsigned long long)__builtin_amdgcn_s_memrealtime());
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

// ---- DPP (GFX9 data-parallel primitives): wave scans / reductions without an
// LDS round trip.  row_shr:n shifts within 16-lane rows; row_bcast:15 / :31
// carry a row's last lane into the following row(s).
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143;

#define SATMI_DPP(old, x, ctrl, rmask) __builtin_amdgcn_update_dpp((old), (x), (ctrl), (rmask), 0xf, false)

// inclusive prefix sum over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += SATMI_DPP(0, x, DPP_ROW_SHR1, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR2, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR4, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR8, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_BCAST15, 0xa);
    x += SATMI_DPP(0, x, DPP_ROW_BCAST31, 0xc);
    return x;
}

// the same within each 16-lane row (enough when only lanes 0..15 hold values)
__device__ __forceinline__ int row_incl_scan(int x) {
    x += SATMI_DPP(0, x, DPP_ROW_SHR1, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR2, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR4, 0xf);
    x += SATMI_DPP(0, x, DPP_ROW_SHR8, 0xf);
    return x;
}

// inclusive prefix max over the 64 lanes
__device__ __forceinline__ int wave_incl_max(int x) {
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_SHR1, 0xf));
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_SHR2, 0xf));
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_SHR4, 0xf));
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_SHR8, 0xf));
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_BCAST15, 0xa));
    x = max(x, SATMI_DPP(INT_MIN, x, DPP_ROW_BCAST31, 0xc));
    return x;
}

__device__ __forceinline__ int lane63(int x) { return __builtin_amdgcn_readlane(x, 63); }

// wave-uniform reductions (all 64 lanes must be active)
__device__ __forceinline__ int wave_min_i32(int x) {
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_SHR1, 0xf));
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_SHR2, 0xf));
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_SHR4, 0xf));
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_SHR8, 0xf));
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_BCAST15, 0xa));
    x = min(x, SATMI_DPP(INT_MAX, x, DPP_ROW_BCAST31, 0xc));
    return lane63(x);
}

__device__ __forceinline__ int wave_max_i32(int x) { return lane63(wave_incl_max(x)); }

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    // order-preserving map of u32 onto i32
    return (uint32_t)wave_min_i32((int)(x ^ 0x80000000u)) ^ 0x80000000u;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    return (uint32_t)wave_max_i32((int)(x ^ 0x80000000u)) ^ 0x80000000u;
}

}  // namespace satmi
