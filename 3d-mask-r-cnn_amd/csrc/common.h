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

// Deterministic reductions (m3d_det_t, include/m3d.h): the reductions that
// would add fp32 partial sums with atomics in arrival order (weight-gradient
// m-splits, per-tensor clip norms) write the partials into the call's scratch
// and sum them in a fixed order instead.  The entry points taking a det open a
// DetScope for the duration of the call (M3D_DET_SCOPE): the launch helpers
// below them read it through det().  The scope is thread-local and ends with
// the call, so the library holds no mode between calls (reentrant).
struct DetState {
    int on;
    void* scratch;
    size_t bytes;
};
DetState det();
int det_check(const m3d_det_t* d);
struct DetScope {
    const m3d_det_t* prev;
    explicit DetScope(const m3d_det_t* d);
    ~DetScope();
    DetScope(const DetScope&) = delete;
    DetScope& operator=(const DetScope&) = delete;
};
#define M3D_DET_SCOPE(d)                                   \
    if (int det_rc_ = ::m3d::det_check(d)) return det_rc_; \
    ::m3d::DetScope det_scope_(d)

inline unsigned grid_for(int64_t n, int per_block, int64_t cap = 1 << 30) {
    int64_t g = (n + per_block - 1) / per_block;
    if (g < 1) g = 1;
    if (g > cap) g = cap;
    return (unsigned)g;
}

// std::min / std::max semantics (NaN behaviour identical to the reference's
// TF 2.2 CPU kernels).
// Workgroup barrier over LDS only: waits for this wave's LDS operations, then
// s_barrier.  __syncthreads() also fences global memory (s_waitcnt vmcnt(0)
// before the barrier), which drains every prefetch in flight -- a serial
// kernel that loads the next step's global operands before a barrier pays a
// full memory round trip per step with it.  Use only where the barrier orders
// LDS traffic alone (global results are not read by other waves after it).
// A workgroup barrier with release / acquire fences limited to LDS ("local"
// MMRA): the compiler knows it as a convergent barrier and orders LDS accesses
// around it, and it emits only lgkmcnt(0) + s_barrier (no vmcnt wait).
__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
__device__ __forceinline__ float smin(float a, float b) { return (b < a) ? b : a; }
__device__ __forceinline__ float smax(float a, float b) { return (a < b) ? b : a; }

// elementwise.hip: fold [3][rows][C] channel partials into s0 / s1 / s2 (+=)
int bn_sums_reduce(const float* part, int64_t rows, int64_t C, float* s0, float* s1, float* s2, hipStream_t s);
int64_t bn_act_bwd_rows(int64_t M, int64_t C);
int bn_act_bwd_splitk(const float* slices, int splits, int64_t M, int64_t C, const m3d_bn_bwd_t* bn,
                      float* dx, int accumulate, void* ws, size_t ws_bytes, hipStream_t s);

// topk.hip: stable sort of n uint64 keys (ascending / descending) with their
// positions (pos[i], or i when pos is NULL) through rank_sort_scratch_bytes(n)
// of device scratch; signed_out: write key ^ 2^63 (int64 order)
size_t rank_sort_scratch_bytes(int64_t n);
int rank_sort_u64(const uint64_t* u, const int64_t* pos, int64_t n, bool desc, bool signed_out, uint32_t* scratch,
                  uint64_t* out_u, int64_t* out_pos, hipStream_t s);

}  // namespace m3d

// ---- tuning constants -------------------------------------------------------
// Every kernel-variant choice of the product library is a compile-time constant
// holding its measured-best value (DESIGN.md 5 lists the A/B runs).  An A/B
// build overrides one:  make ab AB_DEFS=-DM3D_TUNE_ROI_SLICES=16  (libm3d_ab.so,
// loaded with M3D_LIB_FILE=libm3d_ab.so).  Variants measured slower are compiled
// only in such builds (if constexpr on these values).  The one runtime switch
// left is M3D_OPERAND_LIMIT (conv3d.hip: lowers the 32-bit operand bound so the
// per-batch-item path runs at test sizes; tests/test_gpu_conv.py).
// GEMM forms on the exact bf16 split (bit mask, conv3d.hip x3_mask); 31 = all,
// the implicit-GEMM convs included since round 4 (same-box step A/B with the
// fused BN backward: 27.33 -> 27.08 ms, profiles/r04v_cx3_step_ab.txt)
#ifndef M3D_TUNE_GEMM_X3
#define M3D_TUNE_GEMM_X3 31
#endif
#ifndef M3D_TUNE_WGRAD_MINM
#define M3D_TUNE_WGRAD_MINM 512
#endif
#ifndef M3D_TUNE_X3W_TR
#define M3D_TUNE_X3W_TR 1
#endif
#ifndef M3D_TUNE_X3W_TR_MINM
#define M3D_TUNE_X3W_TR_MINM 256
#endif
// stream-K x3_wgrad_tr_kernel in non-deterministic mode (one balanced round
// of workgroups instead of tiles x splits; 0: the split grid in both modes)
#ifndef M3D_TUNE_X3W_SK
#define M3D_TUNE_X3W_SK 1
#endif
// ... for weight-gradient GEMMs whose tiles have at least this many 16-row steps
#ifndef M3D_TUNE_X3W_SK_MIN_STEPS
#define M3D_TUNE_X3W_SK_MIN_STEPS 32
#endif
// (Measured-slower variants and their switches were removed in round 6:
// DESIGN.md section 8 lists them, docs/DESIGN_HISTORY.md has their numbers.)
// Winograd output tile along y: F(2,3) (2) or F(4,3) (4), as NZ is along z.
// 4 (round 4): 4x2x4 tiles, 144 points per 32 outputs instead of 96 per 16 --
// 25 % fewer point-GEMM FLOPs and transform bytes; step 26.9 -> 25.0 ms at
// 128^3 (same box, r04ny4_ab), parity suite green (profiles/r04ny4_parity_tests.log)
#ifndef M3D_TUNE_WINO_NY
#define M3D_TUNE_WINO_NY 4
#endif
#ifndef M3D_TUNE_WINO_NZ
#define M3D_TUNE_WINO_NZ 4
#endif
#ifndef M3D_TUNE_WINO_WGRAD_NZ
#define M3D_TUNE_WINO_WGRAD_NZ 4
#endif
// the data gradient's y tile (conv3d.hip wino_dgrad_ny): 2 = F(2x2x4) data
// gradients beside F(4x2x4) forwards / weight gradients (round 5, accuracy);
// 0 = the forward's
#ifndef M3D_TUNE_WINO_DGRAD_NY
#define M3D_TUNE_WINO_DGRAD_NY 2
#endif
#ifndef M3D_TUNE_WGRAD1_X3_MIN_N
#define M3D_TUNE_WGRAD1_X3_MIN_N 65   // 64 (x3_wgrad64_kernel for 256 -> 64, 64 -> 64): step-neutral, 64 -> 64 slower alone (r06c64b)
#endif
#ifndef M3D_TUNE_BN_BLOCKS
#define M3D_TUNE_BN_BLOCKS 1024
#endif
#ifndef M3D_TUNE_ROI_SLICES
#define M3D_TUNE_ROI_SLICES 8
#endif
