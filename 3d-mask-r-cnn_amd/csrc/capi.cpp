// Non-kernel parts of the C-ABI: error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace m3d {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}
}  // namespace m3d

extern "C" const char* m3d_last_error(void) { return m3d::g_err; }
extern "C" int m3d_abi_version(void) { return 1; }
