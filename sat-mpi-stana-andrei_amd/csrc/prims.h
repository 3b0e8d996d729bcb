// prims.h -- device-wide building blocks for the clause-set kernels (gfx950):
// grid sizing and the exclusive scan of int64 flags / counts (compaction in
// resolution.hip and dp.hip).  All launches go on the caller's stream; no host
// synchronisation happens here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace satmi {
namespace {   // internal linkage: every TU that includes this gets its own kernels

constexpr int PRIM_BLOCK = 256;

static inline int grid_for(int64_t n, int block = PRIM_BLOCK) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

// ---------------------------------------------------------------- exclusive scan
// Three phases over blocks of SCAN_TILE items: tile sums, a single-block scan
// of the tile sums (looping), then per-tile scans plus the tile offset.
constexpr int SCAN_TILE = 1024;

__device__ __forceinline__ int64_t block_excl_scan(int64_t x, int64_t *sh, int64_t *total) {
    // blockDim.x == 256, 4 items per thread handled by the caller
    const int t = threadIdx.x;
    sh[t] = x;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const int64_t y = t >= o ? sh[t - o] : 0;
        __syncthreads();
        sh[t] += y;
        __syncthreads();
    }
    const int64_t incl = sh[t];
    *total = sh[255];
    __syncthreads();
    return incl - x;
}

__global__ void __launch_bounds__(256) scan_tiles_kernel(const int64_t *in, int64_t *tile_sum, int64_t n) {
    __shared__ int64_t sh[256];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t s = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + threadIdx.x * 4 + k;
        if (i < n) s += in[i];
    }
    int64_t tot;
    block_excl_scan(s, sh, &tot);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(256) scan_sums_kernel(int64_t *tile_sum, int64_t ntiles, int64_t *grand) {
    __shared__ int64_t sh[256];
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < ntiles; b0 += 256) {
        const int64_t i = b0 + threadIdx.x;
        const int64_t x = i < ntiles ? tile_sum[i] : 0;
        int64_t tot;
        const int64_t ex = block_excl_scan(x, sh, &tot);
        if (i < ntiles) tile_sum[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0 && grand) *grand = carry;
}

__global__ void __launch_bounds__(256) scan_apply_kernel(const int64_t *in, int64_t *out, const int64_t *tile_off,
                                                         int64_t n) {
    __shared__ int64_t sh[256];
    const int64_t base = (int64_t)blockIdx.x * SCAN_TILE;
    int64_t v[4], s = 0;
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + threadIdx.x * 4 + k;
        v[k] = i < n ? in[i] : 0;
        s += v[k];
    }
    int64_t tot;
    int64_t ex = block_excl_scan(s, sh, &tot) + tile_off[blockIdx.x];
    for (int k = 0; k < 4; ++k) {
        const int64_t i = base + threadIdx.x * 4 + k;
        if (i < n) out[i] = ex;
        ex += v[k];
    }
}

// out[i] = sum(in[0..i)), *grand = sum(in) (device).  tiles: ceil(n/1024) int64 scratch.
static inline int exclusive_scan(const int64_t *in, int64_t *out, int64_t n, int64_t *tiles, int64_t *grand,
                                 hipStream_t s) {
    const int64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
    if (n == 0) {
        if (grand) SATMI_HIP(hipMemsetAsync(grand, 0, sizeof(int64_t), s));
        return SATMI_OK;
    }
    hipLaunchKernelGGL(scan_tiles_kernel, dim3((unsigned)nt), dim3(256), 0, s, in, tiles, n);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(256), 0, s, tiles, nt, grand);
    hipLaunchKernelGGL(scan_apply_kernel, dim3((unsigned)nt), dim3(256), 0, s, in, out, tiles, n);
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
}

}  // namespace
}  // namespace satmi
