// capi.hip -- process-level entry points of libsatmi (errors, devices, memory).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>

#include "common.h"

namespace satmi {

static thread_local std::string g_last_error;

void set_error(const std::string &msg) { g_last_error = msg; }

int hip_fail(hipError_t e, const char *what) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return SATMI_ERR_HIP;
}

// One link of an empty dependent chain (satmi_launch_chain_floor): a single
// vector load + store keeps the launch from being trivially empty.
__global__ void chain_link_kernel(uint32_t *p) {
    if (threadIdx.x == 0) p[0] += 1u;
}

}  // namespace satmi

using namespace satmi;

extern "C" {

int satmi_abi_version(void) { return SATMI_ABI_VERSION; }

const char *satmi_last_error(void) { return g_last_error.c_str(); }

int satmi_device_count(int *count) {
    if (!count) { set_error("count is NULL"); return SATMI_ERR_ARG; }
    SATMI_HIP(hipGetDeviceCount(count));
    return SATMI_OK;
}

int satmi_set_device(int device) {
    SATMI_HIP(hipSetDevice(device));
    return SATMI_OK;
}

int satmi_synchronize(void) {
    SATMI_HIP(hipDeviceSynchronize());
    return SATMI_OK;
}

int satmi_malloc(void **d_ptr, uint64_t bytes) {
    if (!d_ptr) { set_error("d_ptr is NULL"); return SATMI_ERR_ARG; }
    SATMI_HIP(hipMalloc(d_ptr, bytes ? bytes : 16));
    return SATMI_OK;
}

int satmi_free(void *d_ptr) {
    if (d_ptr) SATMI_HIP(hipFree(d_ptr));
    return SATMI_OK;
}

int satmi_memcpy_h2d(void *d_dst, const void *h_src, uint64_t bytes, void *stream) {
    if (!bytes) return SATMI_OK;
    SATMI_HIP(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, (hipStream_t)stream));
    return SATMI_OK;
}

int satmi_memcpy_d2h(void *h_dst, const void *d_src, uint64_t bytes, void *stream) {
    if (!bytes) return SATMI_OK;
    SATMI_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, (hipStream_t)stream));
    SATMI_HIP(hipStreamSynchronize((hipStream_t)stream));
    return SATMI_OK;
}

int satmi_stream_synchronize(void *stream) {
    SATMI_HIP(hipStreamSynchronize((hipStream_t)stream));
    return SATMI_OK;
}

int satmi_launch_chain_floor(int launches, int reps, double *us_per_launch) {
    if (launches < 1 || reps < 1 || !us_per_launch) {
        set_error("satmi_launch_chain_floor: bad arguments");
        return SATMI_ERR_ARG;
    }
    hipStream_t s = nullptr;
    hipGraph_t g = nullptr;
    hipGraphExec_t ge = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    uint32_t *d = nullptr;
    int rc = SATMI_OK;
    hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&d, 256);
    if (e == hipSuccess) e = hipMemsetAsync(d, 0, 256, s);
    if (e == hipSuccess) e = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    if (e == hipSuccess) {
        for (int i = 0; i < launches; ++i) hipLaunchKernelGGL(chain_link_kernel, dim3(1), dim3(64), 0, s, d);
        e = hipStreamEndCapture(s, &g);
    }
    if (e == hipSuccess) e = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    if (e == hipSuccess) e = hipGraphLaunch(ge, s);   // warm-up replay
    if (e == hipSuccess) e = hipEventRecord(e0, s);
    for (int r = 0; e == hipSuccess && r < reps; ++r) e = hipGraphLaunch(ge, s);
    if (e == hipSuccess) e = hipEventRecord(e1, s);
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e == hipSuccess) *us_per_launch = (double)ms * 1e3 / ((double)launches * reps);
    else rc = hip_fail(e, "satmi_launch_chain_floor");
    if (e1) (void)hipEventDestroy(e1);
    if (e0) (void)hipEventDestroy(e0);
    if (ge) (void)hipGraphExecDestroy(ge);
    if (g) (void)hipGraphDestroy(g);
    if (s) (void)hipStreamSynchronize(s);
    if (d) (void)hipFree(d);
    if (s) (void)hipStreamDestroy(s);
    return rc;
}

}  // extern "C"
