// Error reporting of the C ABI (include/nerf_hip.h): per-thread last-error message.
#include <stdarg.h>
#include <stdio.h>

#include "../../include/nerf_hip.h"

namespace nerf {

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

}  // namespace nerf

extern "C" const char* nerf_last_error(void) { return nerf::g_last_error; }

extern "C" int nerf_abi_version(void) { return 12; }
