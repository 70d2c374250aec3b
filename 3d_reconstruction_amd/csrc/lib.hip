// lib.hip — library-level entry points: version, thread-local error, arch probe.
#include "common.h"
#include <cstring>

namespace sfmhip {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
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
