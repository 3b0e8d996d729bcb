// issue_probe.hip -- measure the per-CU issue rates that bound dpll_scan_kernel
// on gfx950: integer VALU (v_add_u32, v_bfe_u32), SALU (s_add_u32) and LDS
// byte gathers (ds_read_u8, conflict-free and random), at 1..8 waves per SIMD.
// Prints one JSON line per case: wave-instructions per CU-cycle.
//
//   hipcc -O3 --offload-arch=gfx950 -o tools/issue_probe tools/issue_probe.hip
//   tools/issue_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <vector>

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e_ = (x);                                                              \
        if (e_ != hipSuccess) {                                                           \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

enum { K_VADD = 0, K_VBFE = 1, K_SADD = 2, K_LDS_SEQ = 3, K_LDS_RND = 4, K_MIX = 5 };

template <int KIND>
__global__ void __launch_bounds__(64) probe(int iters, uint32_t *out, uint64_t *span) {
    __shared__ uint8_t lds[1024];
    for (int i = threadIdx.x; i < 1024; i += 64) lds[i] = (uint8_t)(i * 7);
    __syncthreads();
    uint32_t a[8];
    for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * (j + 3) + j;
    uint32_t s0 = blockIdx.x, s1 = 3, s2 = 5, s3 = 7;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (KIND == K_VADD) {
#pragma unroll
                for (int j = 0; j < 8; ++j) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
            } else if constexpr (KIND == K_VBFE) {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    asm volatile("v_bfe_u32 %0, %0, %1, 10" : "+v"(a[j]) : "v"(a[(j + 1) & 7]));
            } else if constexpr (KIND == K_SADD) {
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(s2));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s2) : "s"(s3));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s3) : "s"(s0));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(s2));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s2) : "s"(s3));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s3) : "s"(s0));
            } else if constexpr (KIND == K_LDS_SEQ || KIND == K_LDS_RND) {
                // 8 independent byte gathers: lane l reads byte l*4 (one dword per
                // bank, conflict-free) or a pseudo-random byte of 1 KiB
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    uint32_t addr = KIND == K_LDS_SEQ ? (threadIdx.x * 4u + (uint32_t)j * 256u) & 1023u
                                                     : (a[j] * 2654435761u >> 22) & 1023u;
                    uint32_t v;
                    asm volatile("ds_read_u8 %0, %1" : "=v"(v) : "v"(addr));
                    a[j] += v;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            } else {
                // dpll_scan-like mix: 1 word + 3 byte gathers, ~6 VALU per clause slot
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    uint32_t w;
                    uint32_t wa = (threadIdx.x * 4u + (uint32_t)j * 256u) & 1023u;
                    asm volatile("ds_read_b32 %0, %1" : "=v"(w) : "v"(wa));
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    w ^= a[j];
                    uint32_t x0, x1, x2;
                    uint32_t c0 = w & 1023u, c1 = (w >> 10) & 1023u, c2 = (w >> 20) & 1023u;
                    asm volatile("ds_read_u8 %0, %1" : "=v"(x0) : "v"(c0));
                    asm volatile("ds_read_u8 %0, %1" : "=v"(x1) : "v"(c1));
                    asm volatile("ds_read_u8 %0, %1" : "=v"(x2) : "v"(c2));
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    a[j] += x0 + x1 + x2;
                }
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint32_t acc = s0 + s1 + s2 + s3;
    for (int j = 0; j < 8; ++j) acc += a[j];
    out[blockIdx.x * 64 + threadIdx.x] = acc;
    if (threadIdx.x == 0) span[blockIdx.x] = t1 - t0;
}

template <int KIND>
int run(const char *name, double insts_per_iter, int cus, int waves_per_simd) {
    const int iters = 4096;
    const int blocks = cus * 4 * waves_per_simd;   // one-wave workgroups
    uint32_t *out;
    uint64_t *span;
    CHECK(hipMalloc(&out, sizeof(uint32_t) * blocks * 64));
    CHECK(hipMalloc(&span, sizeof(uint64_t) * blocks));
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(64), 0, 0, iters, out, span);   // warm
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL(probe<KIND>, dim3(blocks), dim3(64), 0, 0, iters, out, span);
    CHECK(hipDeviceSynchronize());
    std::vector<uint64_t> h(blocks);
    CHECK(hipMemcpy(h.data(), span, sizeof(uint64_t) * blocks, hipMemcpyDeviceToHost));
    double mean = 0;
    uint64_t mx = 0;
    for (auto v : h) {
        mean += (double)v;
        mx = v > mx ? v : mx;
    }
    mean /= blocks;
    // wave-instructions per CU-cycle: all waves of a CU over the mean wave span
    const double per_cu = 4.0 * waves_per_simd * insts_per_iter * iters / mean;
    std::printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"inst_per_cu_cycle\": %.3f, \"mean_span\": %.0f, \"max_span\": %llu}\n",
                name, waves_per_simd, per_cu, mean, (unsigned long long)mx);
    CHECK(hipFree(out));
    CHECK(hipFree(span));
    return 0;
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    for (int w : {1, 2, 4, 8}) {
        run<K_VADD>("v_add_u32", 32, cus, w);
        run<K_VBFE>("v_bfe_u32", 32, cus, w);
        run<K_SADD>("s_add_u32", 32, cus, w);
        run<K_LDS_SEQ>("ds_read_u8 conflict-free", 32, cus, w);
        run<K_LDS_RND>("ds_read_u8 random 1KiB", 32, cus, w);
        run<K_MIX>("mix: ds_read_b32 + 3 ds_read_u8 (LDS insts)", 32, cus, w);
    }
    return 0;
}
