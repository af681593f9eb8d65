// Non-kernel parts of the C-ABI: error string, version.
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

namespace m3d {
static thread_local char g_err[512] = "";
static DetState g_det = {0, nullptr, 0};

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

const DetState& det() { return g_det; }
}  // namespace m3d

extern "C" const char* m3d_last_error(void) { return m3d::g_err; }
extern "C" int m3d_abi_version(void) { return 1; }

extern "C" int m3d_set_deterministic(int32_t on, void* scratch, size_t bytes) {
    if (on && (!scratch || bytes < 4096 || (reinterpret_cast<uintptr_t>(scratch) & 15)))
        return m3d::einval("set_deterministic: needs a 16-byte aligned device scratch of >= 4096 bytes");
    m3d::g_det = on ? m3d::DetState{1, scratch, bytes} : m3d::DetState{0, nullptr, 0};
    return M3D_OK;
}

extern "C" int32_t m3d_get_deterministic(void) { return m3d::g_det.on; }
