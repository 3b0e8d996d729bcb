// prims.h -- device-wide building blocks for the clause-set kernels (gfx950):
// exclusive scan of int64 counts, stable merge sort of an index array under a
// key comparator, rank-merge of two sorted key arrays.  All launches go on the
// caller's stream; no host synchronisation happens here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace satmi {
namespace {   // internal linkage: every TU that includes this gets its own kernels

constexpr int PRIM_BLOCK = 256;

// ---------------------------------------------------------------- multiword keys
// A clause key is K uint64 words: positive-literal bitset words then negative
// ones over the formula's dense variable index.  Order: lexicographic.
struct KeyView {
    const uint64_t *w;
    int K;
    __device__ __forceinline__ const uint64_t *at(int64_t i) const { return w + i * K; }
};

__device__ __forceinline__ int key_cmp(const uint64_t *a, const uint64_t *b, int K) {
    for (int k = 0; k < K; ++k) {
        if (a[k] != b[k]) return a[k] < b[k] ? -1 : 1;
    }
    return 0;
}

// number of elements of sorted idx[lo, hi) whose key is < x (strict) or <= x
template <bool UPPER>
__device__ int64_t rank_in(const KeyView &kv, const int64_t *idx, int64_t lo, int64_t hi, const uint64_t *x) {
    int64_t a = lo, b = hi;
    while (a < b) {
        const int64_t mid = (a + b) >> 1;
        const int c = key_cmp(kv.at(idx ? idx[mid] : mid), x, kv.K);
        if (c < 0 || (UPPER && c == 0)) a = mid + 1;
        else b = mid;
    }
    return a - lo;
}

// one pass of a stable bottom-up merge sort of idx by key: runs of `width`
__global__ void merge_pass_kernel(KeyView kv, const int64_t *in, int64_t *out, int64_t n, int64_t width) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a0 = (i / (2 * width)) * (2 * width);
        const int64_t a1 = min(a0 + width, n), b1 = min(a0 + 2 * width, n);
        const int64_t x = in[i];
        int64_t pos;
        if (i < a1) pos = i + rank_in<false>(kv, in, a1, b1, kv.at(x));          // A before equal B
        else pos = a0 + (i - a1) + rank_in<true>(kv, in, a0, a1, kv.at(x));
        out[pos] = x;
    }
}

__global__ void iota_kernel(int64_t *a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        a[i] = i;
}

static inline int grid_for(int64_t n, int block = PRIM_BLOCK) {
    int64_t g = (n + block - 1) / block;
    if (g < 1) g = 1;
    if (g > 65536) g = 65536;
    return (int)g;
}

// Sort indices 0..n-1 by key; result in *result (== a or tmp).  a, tmp: n int64 each.
static inline int sort_indices(KeyView kv, int64_t n, int64_t *a, int64_t *tmp, int64_t **result, hipStream_t s) {
    hipLaunchKernelGGL(iota_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, a, n);
    int64_t *src = a, *dst = tmp;
    for (int64_t w = 1; w < n; w *= 2) {
        hipLaunchKernelGGL(merge_pass_kernel, dim3(grid_for(n)), dim3(PRIM_BLOCK), 0, s, kv, src, dst, n, w);
        int64_t *t = src;
        src = dst;
        dst = t;
    }
    *result = src;
    SATMI_HIP(hipGetLastError());
    return SATMI_OK;
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
