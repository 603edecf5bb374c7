// capi.hip -- error plumbing and ABI version of libuavhip.so (see include/uavhip.h).
#include <cstdarg>
#include <cstdio>

#include "common.hpp"

namespace uavhip {
static thread_local char g_err[1024] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

int check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return UAVHIP_EHIP;
    }
    return UAVHIP_OK;
}
}  // namespace uavhip

extern "C" const char* uavhip_last_error(void) { return uavhip::g_err; }
extern "C" int32_t uavhip_abi_version(void) { return 4; }
