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

}  // extern "C"
