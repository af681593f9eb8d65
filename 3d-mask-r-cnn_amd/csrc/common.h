// Shared helpers for the libm3d HIP sources (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>

#include "../../include/m3d.h"

namespace m3d {

// Thread-local last-error text (the reference's InvalidArgument strings).
void set_error(const char* fmt, ...);

inline int einval(const char* msg) {
    set_error("%s", msg);
    return M3D_EINVAL;
}

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return M3D_EHIP;
    }
    return M3D_OK;
}

inline hipStream_t st(m3d_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Deterministic mode (m3d_set_deterministic): the reductions that would add
// fp32 partial sums with atomics in arrival order (weight-gradient m-splits,
// per-tensor clip norms) write the partials into the registered scratch and
// sum them in a fixed order instead.
struct DetState {
    int on;
    void* scratch;
    size_t bytes;
};
const DetState& det();

inline unsigned grid_for(int64_t n, int per_block, int64_t cap = 1 << 30) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// std::min / std::max semantics (NaN behaviour identical to the reference's
// TF 2.2 CPU kernels).
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }

}  // namespace m3d
