// lib.hip — library-level entry points: version, thread-local error, arch probe.
#include "common.h"
#include <cstring>
#include <mutex>

namespace sfmhip {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s) {
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev >= 0 && dev < kMaxDev) {
        std::call_once(once[dev], [dev] {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
                uint64_t thr = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
            }
            (void)hipGetLastError();
        });
    }
    return hipMallocAsync(p, bytes, s);
}
}  // namespace sfmhip

extern "C" int sfmhip_version(void) { return (0 << 16) | (1 << 8) | 0; }

extern "C" const char* sfmhip_last_error(void) { return sfmhip::g_err; }

extern "C" int sfmhip_device_arch(char* buf, int len) {
    SFMHIP_REQUIRE(buf != nullptr && len > 0, "sfmhip_device_arch: null buffer");
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, 0);
    if (e != hipSuccess) {
        sfmhip::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
        return SFMHIP_E_HIP;
    }
    std::strncpy(buf, prop.gcnArchName, (size_t)len - 1);
    buf[len - 1] = '\0';
    return SFMHIP_OK;
}
