// Bandwidth-bound kernels of the backbone/FPN/RPN graph (gfx950).
//   maxpool3d fwd/bwd   KL.MaxPooling3D (core/models.py:245 stem pool, 3211 P6)
//   upsample221 bwd     KL.UpSampling3D((2,2,1)) adjoint (core/models.py:3193-3204)
//   subsample221        P6 = MaxPool(1, strides (2,2,1)) (core/models.py:3211)
//   bn_act_bwd          backward of act(BN_frozen(z) [+ residual]) with the
//                       per-channel reductions for gamma/beta/bias
//   sgd_keras           Keras 2.3.1 SGD + clipnorm + decay + the RPN L2 term
//                       (core/models.py:3340-3387)
// All channels-last with C innermost; threads map to consecutive channels so
// every access is coalesced; float4 where C % 4 == 0.
#include "common.h"

namespace m3d {

__global__ void maxpool_fwd_kernel(const float* __restrict__ x, int B, int H, int W, int D, int C,
                                   int kh, int kw, int kd, int sy, int sx, int sz, int py, int px,
                                   int pz, int OH, int OW, int OD, float* __restrict__ y,
                                   uint8_t* __restrict__ am) {
    const int64_t total = (int64_t)B * OH * OW * OD * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        int64_t t = i / C;
        const int oz = (int)(t % OD); t /= OD;
        const int ox = (int)(t % OW); t /= OW;
        const int oy = (int)(t % OH);
        const int b = (int)(t / OH);
        float best = -INFINITY;
        int bi = 0;
        bool any = false;
        for (int ky = 0; ky < kh; ++ky) {
            const int iy = oy * sy - py + ky;
            if (iy < 0 || iy >= H) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int ix = ox * sx - px + kx;
                if (ix < 0 || ix >= W) continue;
                for (int kz = 0; kz < kd; ++kz) {
                    const int iz = oz * sz - pz + kz;
                    if (iz < 0 || iz >= D) continue;
                    const float v = x[((((int64_t)b * H + iy) * W + ix) * D + iz) * C + c];
                    if (!any || v > best) { best = v; bi = (ky * kw + kx) * kd + kz; any = true; }
                }
            }
        }
        y[i] = best;
        if (am) am[i] = (uint8_t)bi;
    }
}

__global__ void maxpool_bwd_kernel(const float* __restrict__ dy, const uint8_t* __restrict__ am,
                                   int B, int H, int W, int D, int C, int kh, int kw, int kd,
                                   int sy, int sx, int sz, int py, int px, int pz, int OH, int OW,
                                   int OD, float* __restrict__ dx) {
    const int64_t total = (int64_t)B * H * W * D * C;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C);
        int64_t t = i / C;
        const int iz = (int)(t % D); t /= D;
        const int ix = (int)(t % W); t /= W;
        const int iy = (int)(t % H);
        const int b = (int)(t / H);
        float acc = 0.0f;
        // outputs o with o*s - p <= i <= o*s - p + k - 1
        const int oy_lo = max(0, (iy + py - kh + 1 + sy - 1) / sy), oy_hi = min(OH - 1, (iy + py) / sy);
        const int ox_lo = max(0, (ix + px - kw + 1 + sx - 1) / sx), ox_hi = min(OW - 1, (ix + px) / sx);
        const int oz_lo = max(0, (iz + pz - kd + 1 + sz - 1) / sz), oz_hi = min(OD - 1, (iz + pz) / sz);
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const int ky = iy - (oy * sy - py);
            if (ky < 0 || ky >= kh) continue;
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int kx = ix - (ox * sx - px);
                if (kx < 0 || kx >= kw) continue;
                for (int oz = oz_lo; oz <= oz_hi; ++oz) {
                    const int kz = iz - (oz * sz - pz);
                    if (kz < 0 || kz >= kd) continue;
                    const int64_t o = ((((int64_t)b * OH + oy) * OW + ox) * OD + oz) * C + c;
                    if (am[o] == (uint8_t)((ky * kw + kx) * kd + kz)) acc += dy[o];
                }
            }
        }
        dx[i] = acc;
    }
}

// C % 4 == 0 and < 2^31 float4s per tensor: one float4 of channels per
// thread and 32-bit index math (the generic kernels above pay a 64-bit
// division chain per element: the stem pool ran at 0.8 TB/s).  Per channel
// the window order, the first-valid initialisation and the strict '>' (so the
// argmax byte and NaN behaviour) and the backward summation order are the
// scalar kernels' own, so results are bit-identical.
// Depth-slab halo planes beside the slab (m3d.slab.halo_planes): the pool runs on
// the virtual z grid [lower halo (nlo planes) | slab (Dl) | upper halo], D =
// nlo + Dl + nhi; plane zl = z - nlo < 0 reads halo plane zl + r, zl >= Dl
// reads halo plane r + zl - Dl ([B,H,W,2r,C]: [0,r) from below, [r,2r) from
// above).  Same values and order as the pool over the halo-extended copy.
struct PoolHalo {
    const float4* h;     // [B,H,W,2r,C/4]
    float4* dh;          // backward: gradient of the halo planes, same layout
    int nlo, Dl, r;
};
template <bool HALO>
__device__ __forceinline__ uint32_t pool_zoff(const PoolHalo& hz, uint32_t bhw, int D, int iz, int C4,
                                              bool& in_halo) {
    if (!HALO) {
        in_halo = false;
        return (bhw * (uint32_t)D + iz) * (uint32_t)C4;
    }
    const int zl = iz - hz.nlo;
    in_halo = zl < 0 || zl >= hz.Dl;
    if (!in_halo) return (bhw * (uint32_t)hz.Dl + zl) * (uint32_t)C4;
    const int pl = zl < 0 ? zl + hz.r : hz.r + zl - hz.Dl;
    return (bhw * (uint32_t)(2 * hz.r) + pl) * (uint32_t)C4;
}

template <bool HALO>
__global__ __launch_bounds__(256) void maxpool_fwd4_kernel(const float4* __restrict__ x, int H, int W, int D,
                                                           int C4, int kh, int kw, int kd, int sy, int sx,
                                                           int sz, int py, int px, int pz, int OH, int OW,
                                                           int OD, uint32_t total, float4* __restrict__ y,
                                                           uchar4* __restrict__ am, PoolHalo hz) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int oz = (int)(t % (uint32_t)OD); t /= (uint32_t)OD;
        const int ox = (int)(t % (uint32_t)OW); t /= (uint32_t)OW;
        const int oy = (int)(t % (uint32_t)OH);
        const uint32_t b = t / (uint32_t)OH;
        float best[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        int bi[4] = {0, 0, 0, 0};
        bool any = false;
        for (int ky = 0; ky < kh; ++ky) {
            const int iy = oy * sy - py + ky;
            if (iy < 0 || iy >= H) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int ix = ox * sx - px + kx;
                if (ix < 0 || ix >= W) continue;
                const uint32_t bhw = (b * (uint32_t)H + iy) * (uint32_t)W + ix;
                for (int kz = 0; kz < kd; ++kz) {
                    const int iz = oz * sz - pz + kz;
                    if (iz < 0 || iz >= D) continue;
                    bool hal;
                    const uint32_t zo = pool_zoff<HALO>(hz, bhw, D, iz, C4, hal);
                    const float4 v = (HALO && hal ? hz.h : x)[zo + c];
                    const float vv[4] = {v.x, v.y, v.z, v.w};
                    const int id = (ky * kw + kx) * kd + kz;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (!any || vv[q] > best[q]) { best[q] = vv[q]; bi[q] = id; }
                    any = true;
                }
            }
        }
        y[i] = make_float4(best[0], best[1], best[2], best[3]);
        if (am) am[i] = make_uchar4((unsigned char)bi[0], (unsigned char)bi[1], (unsigned char)bi[2],
                                    (unsigned char)bi[3]);
    }
}

template <bool HALO>
__global__ __launch_bounds__(256) void maxpool_bwd4_kernel(const float4* __restrict__ dy,
                                                           const uchar4* __restrict__ am, int H, int W,
                                                           int D, int C4, int kh, int kw, int kd, int sy,
                                                           int sx, int sz, int py, int px, int pz, int OH,
                                                           int OW, int OD, uint32_t total,
                                                           float4* __restrict__ dx, PoolHalo hz) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int iz = (int)(t % (uint32_t)D); t /= (uint32_t)D;
        const int ix = (int)(t % (uint32_t)W); t /= (uint32_t)W;
        const int iy = (int)(t % (uint32_t)H);
        const uint32_t b = t / (uint32_t)H;
        float acc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        const int oy_lo = max(0, (iy + py - kh + 1 + sy - 1) / sy), oy_hi = min(OH - 1, (iy + py) / sy);
        const int ox_lo = max(0, (ix + px - kw + 1 + sx - 1) / sx), ox_hi = min(OW - 1, (ix + px) / sx);
        const int oz_lo = max(0, (iz + pz - kd + 1 + sz - 1) / sz), oz_hi = min(OD - 1, (iz + pz) / sz);
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const int ky = iy - (oy * sy - py);
            if (ky < 0 || ky >= kh) continue;
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int kx = ix - (ox * sx - px);
                if (kx < 0 || kx >= kw) continue;
                const uint32_t row = ((b * (uint32_t)OH + oy) * (uint32_t)OW + ox) * (uint32_t)OD;
                for (int oz = oz_lo; oz <= oz_hi; ++oz) {
                    const int kz = iz - (oz * sz - pz);
                    if (kz < 0 || kz >= kd) continue;
                    const uint32_t o = (row + oz) * (uint32_t)C4 + c;
                    const uchar4 a = am[o];
                    const float4 g = dy[o];
                    const unsigned char id = (unsigned char)((ky * kw + kx) * kd + kz);
                    if (a.x == id) acc[0] += g.x;
                    if (a.y == id) acc[1] += g.y;
                    if (a.z == id) acc[2] += g.z;
                    if (a.w == id) acc[3] += g.w;
                }
            }
        }
        const float4 r = make_float4(acc[0], acc[1], acc[2], acc[3]);
        if (HALO) {     // i runs over the virtual grid: the slab's planes go to dx, the halo's to dh
            bool hal;
            const uint32_t zo = pool_zoff<true>(hz, (b * (uint32_t)H + iy) * (uint32_t)W + ix, D, iz, C4, hal);
            (hal ? hz.dh : dx)[zo + c] = r;
        } else {
            dx[i] = r;
        }
    }
}

// z-stride-1 pools (the stem's MaxPooling3D((3,3,3),(2,2,1),'same'),
// core/models.py:245) over runs of R consecutive output (fwd) / input (bwd) z
// planes per thread: the windows of neighbouring z overlap in all but one
// plane, so each input plane (fwd) or dy / argmax plane (bwd) is loaded once
// per run instead of up to kd times (the per-element forms re-read every
// window: 27 float4 loads per output, L2-bound at 2.3 TB/s of HBM bytes at
// 256^3).  Per output the window is visited in the same (ky, kx, kz) order with
// the same first-valid / strict '>' rule, and per input the backward adds its
// windows in the same (oy, ox, oz) order: bit-identical to the kernels above.
template <bool HALO, int R>
__global__ __launch_bounds__(256) void maxpool_fwd4z_kernel(const float4* __restrict__ x, int H, int W, int D,
                                                            int C4, int kh, int kw, int kd, int sy, int sx,
                                                            int py, int px, int pz, int OH, int OW, int OD,
                                                            int nrun, uint32_t total, float4* __restrict__ y,
                                                            uchar4* __restrict__ am, PoolHalo hz) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int run = (int)(t % (uint32_t)nrun); t /= (uint32_t)nrun;
        const int ox = (int)(t % (uint32_t)OW); t /= (uint32_t)OW;
        const int oy = (int)(t % (uint32_t)OH);
        const uint32_t b = t / (uint32_t)OH;
        const int oz0 = run * R;
        const int nr = OD - oz0 < R ? OD - oz0 : R;
        float best[R][4];
        int bi[R][4];
        bool any[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            any[r] = false;
#pragma unroll
            for (int q = 0; q < 4; ++q) { best[r][q] = -INFINITY; bi[r][q] = 0; }
        }
        for (int ky = 0; ky < kh; ++ky) {
            const int iy = oy * sy - py + ky;
            if (iy < 0 || iy >= H) continue;
            for (int kx = 0; kx < kw; ++kx) {
                const int ix = ox * sx - px + kx;
                if (ix < 0 || ix >= W) continue;
                const uint32_t bhw = (b * (uint32_t)H + iy) * (uint32_t)W + ix;
                const int base = (ky * kw + kx) * kd;
                const int iz_lo = oz0 - pz < 0 ? 0 : oz0 - pz;
                const int iz_end = oz0 + nr - 1 - pz + kd;
                for (int iz = iz_lo; iz < iz_end && iz < D; ++iz) {
                    bool hal;
                    const uint32_t zo = pool_zoff<HALO>(hz, bhw, D, iz, C4, hal);
                    const float4 v = (HALO && hal ? hz.h : x)[zo + c];
                    const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int kz = iz - (oz0 + r - pz);
                        if (r < nr && kz >= 0 && kz < kd) {
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                if (!any[r] || vv[q] > best[r][q]) { best[r][q] = vv[q]; bi[r][q] = base + kz; }
                            any[r] = true;
                        }
                    }
                }
            }
        }
        const uint32_t o0 = ((b * (uint32_t)OH + oy) * (uint32_t)OW + ox) * (uint32_t)OD + oz0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r >= nr) break;
            const uint32_t o = (o0 + r) * (uint32_t)C4 + c;
            y[o] = make_float4(best[r][0], best[r][1], best[r][2], best[r][3]);
            if (am) am[o] = make_uchar4((unsigned char)bi[r][0], (unsigned char)bi[r][1], (unsigned char)bi[r][2],
                                        (unsigned char)bi[r][3]);
        }
    }
}

// maxpool_fwd4z_kernel specialised to the stem's pool (KL.MaxPooling3D((3,3,3),
// (2,2,1), 'same'): core/models.py:244), no halo.  Per (y, x) tap column the
// R + 2 input planes of the run are loaded as one unrolled batch (independent
// loads in flight; the general kernel's runtime-bounded z loop issued them one
// at a time behind its compares), clamped in range and masked; the compares
// then run in the general kernel's order (ky, kx, iz ascending, first maximum
// wins): bit-identical values and argmax.
template <int R>
__global__ __launch_bounds__(256) void maxpool_fwd333_kernel(const float4* __restrict__ x, int H, int W, int D,
                                                             int C4, int OH, int OW, int nrun, uint32_t total,
                                                             float4* __restrict__ y, uchar4* __restrict__ am) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int run = (int)(t % (uint32_t)nrun); t /= (uint32_t)nrun;
        const int ox = (int)(t % (uint32_t)OW); t /= (uint32_t)OW;
        const int oy = (int)(t % (uint32_t)OH);
        const uint32_t b = t / (uint32_t)OH;
        const int oz0 = run * R;                       // OD == D ('same', stride 1 along z)
        const int nr = D - oz0 < R ? D - oz0 : R;
        float best[R][4];
        int bi[R][4];
        bool any[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            any[r] = false;
#pragma unroll
            for (int q = 0; q < 4; ++q) { best[r][q] = -INFINITY; bi[r][q] = 0; }
        }
        // 'same' padding of a 3-window, stride 2: pad-before (k - 1 - (H - 1) % 2) / 2
        const int py = (2 - (H - 1) % 2) / 2, px = (2 - (W - 1) % 2) / 2;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int iy = oy * 2 - py + ky;
            if (iy < 0 || iy >= H) continue;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int ix = ox * 2 - px + kx;
                if (ix < 0 || ix >= W) continue;
                const uint32_t col = ((b * (uint32_t)H + iy) * (uint32_t)W + ix) * (uint32_t)D;
                const int base = (ky * 3 + kx) * 3;
                float4 v[R + 2];
#pragma unroll
                for (int p = 0; p < R + 2; ++p) {          // plane iz = oz0 - 1 + p
                    int iz = oz0 - 1 + p;
                    iz = iz < 0 ? 0 : (iz >= D ? D - 1 : iz);
                    v[p] = x[(col + (uint32_t)iz) * (uint32_t)C4 + c];
                }
#pragma unroll
                for (int p = 0; p < R + 2; ++p) {
                    const int iz = oz0 - 1 + p;
                    if (iz < 0 || iz >= D) continue;
                    const float vv[4] = {v[p].x, v[p].y, v[p].z, v[p].w};
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int kz = p - r;
                        if (r < nr && kz >= 0 && kz < 3) {
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                if (!any[r] || vv[q] > best[r][q]) { best[r][q] = vv[q]; bi[r][q] = base + kz; }
                            any[r] = true;
                        }
                    }
                }
            }
        }
        const uint32_t o0 = ((b * (uint32_t)OH + oy) * (uint32_t)OW + ox) * (uint32_t)D + oz0;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r >= nr) break;
            const uint32_t o = (o0 + r) * (uint32_t)C4 + c;
            y[o] = make_float4(best[r][0], best[r][1], best[r][2], best[r][3]);
            if (am) am[o] = make_uchar4((unsigned char)bi[r][0], (unsigned char)bi[r][1], (unsigned char)bi[r][2],
                                        (unsigned char)bi[r][3]);
        }
    }
}

// maxpool_bwd4z_kernel specialised as maxpool_fwd333_kernel: per (oy, ox)
// output column the R + 2 (argmax, gradient) rows of the run are loaded as one
// unrolled batch, then added in the general kernel's order (oy, ox, oz
// ascending): bit-identical sums.
template <int R>
__global__ __launch_bounds__(256) void maxpool_bwd333_kernel(const float4* __restrict__ dy,
                                                             const uchar4* __restrict__ am, int H, int W, int D,
                                                             int C4, int OH, int OW, int nrun, uint32_t total,
                                                             float4* __restrict__ dx) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int run = (int)(t % (uint32_t)nrun); t /= (uint32_t)nrun;
        const int ix = (int)(t % (uint32_t)W); t /= (uint32_t)W;
        const int iy = (int)(t % (uint32_t)H);
        const uint32_t b = t / (uint32_t)H;
        const int iz0 = run * R;
        const int nr = D - iz0 < R ? D - iz0 : R;
        float acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] = 0.0f;
        const int py = (2 - (H - 1) % 2) / 2, px = (2 - (W - 1) % 2) / 2;
        const int oy_lo = max(0, (iy + py - 1) / 2), oy_hi = min(OH - 1, (iy + py) / 2);
        const int ox_lo = max(0, (ix + px - 1) / 2), ox_hi = min(OW - 1, (ix + px) / 2);
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const int ky = iy - (oy * 2 - py);
            if (ky < 0 || ky >= 3) continue;
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int kx = ix - (ox * 2 - px);
                if (kx < 0 || kx >= 3) continue;
                const uint32_t row = ((b * (uint32_t)OH + oy) * (uint32_t)OW + ox) * (uint32_t)D;
                const int base = (ky * 3 + kx) * 3;
                uchar4 a[R + 2];
                float4 g[R + 2];
#pragma unroll
                for (int p = 0; p < R + 2; ++p) {          // output plane oz = iz0 - 1 + p
                    int oz = iz0 - 1 + p;
                    oz = oz < 0 ? 0 : (oz >= D ? D - 1 : oz);
                    const uint32_t o = (row + (uint32_t)oz) * (uint32_t)C4 + c;
                    a[p] = am[o];
                    g[p] = dy[o];
                }
#pragma unroll
                for (int p = 0; p < R + 2; ++p) {
                    const int oz = iz0 - 1 + p;
                    if (oz < 0 || oz >= D) continue;
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int kz = r - p + 2;           // iz0 + r - (oz - 1)
                        if (r < nr && kz >= 0 && kz < 3) {
                            const unsigned char id = (unsigned char)(base + kz);
                            if (a[p].x == id) acc[r][0] += g[p].x;
                            if (a[p].y == id) acc[r][1] += g[p].y;
                            if (a[p].z == id) acc[r][2] += g[p].z;
                            if (a[p].w == id) acc[r][3] += g[p].w;
                        }
                    }
                }
            }
        }
        const uint32_t bhw = (b * (uint32_t)H + iy) * (uint32_t)W + ix;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r >= nr) break;
            dx[(bhw * (uint32_t)D + iz0 + r) * (uint32_t)C4 + c] =
                make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
        }
    }
}

template <bool HALO, int R>
__global__ __launch_bounds__(256) void maxpool_bwd4z_kernel(const float4* __restrict__ dy,
                                                            const uchar4* __restrict__ am, int H, int W, int D,
                                                            int C4, int kh, int kw, int kd, int sy, int sx, int py,
                                                            int px, int pz, int OH, int OW, int OD, int nrun,
                                                            uint32_t total, float4* __restrict__ dx, PoolHalo hz) {
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
        const uint32_t c = i % (uint32_t)C4;
        uint32_t t = i / (uint32_t)C4;
        const int run = (int)(t % (uint32_t)nrun); t /= (uint32_t)nrun;
        const int ix = (int)(t % (uint32_t)W); t /= (uint32_t)W;
        const int iy = (int)(t % (uint32_t)H);
        const uint32_t b = t / (uint32_t)H;
        const int iz0 = run * R;
        const int nr = D - iz0 < R ? D - iz0 : R;
        float acc[R][4];
#pragma unroll
        for (int r = 0; r < R; ++r)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[r][q] = 0.0f;
        const int oy_lo = max(0, (iy + py - kh + 1 + sy - 1) / sy), oy_hi = min(OH - 1, (iy + py) / sy);
        const int ox_lo = max(0, (ix + px - kw + 1 + sx - 1) / sx), ox_hi = min(OW - 1, (ix + px) / sx);
        // outputs oz with oz - pz <= iz <= oz - pz + kd - 1 for some iz of the run
        const int oz_lo = max(0, iz0 + pz - kd + 1), oz_hi = min(OD - 1, iz0 + nr - 1 + pz);
        for (int oy = oy_lo; oy <= oy_hi; ++oy) {
            const int ky = iy - (oy * sy - py);
            if (ky < 0 || ky >= kh) continue;
            for (int ox = ox_lo; ox <= ox_hi; ++ox) {
                const int kx = ix - (ox * sx - px);
                if (kx < 0 || kx >= kw) continue;
                const uint32_t row = ((b * (uint32_t)OH + oy) * (uint32_t)OW + ox) * (uint32_t)OD;
                const int base = (ky * kw + kx) * kd;
                for (int oz = oz_lo; oz <= oz_hi; ++oz) {
                    const uint32_t o = (row + oz) * (uint32_t)C4 + c;
                    const uchar4 a = am[o];
                    const float4 g = dy[o];
#pragma unroll
                    for (int r = 0; r < R; ++r) {
                        const int kz = iz0 + r - (oz - pz);
                        if (r < nr && kz >= 0 && kz < kd) {
                            const unsigned char id = (unsigned char)(base + kz);
                            if (a.x == id) acc[r][0] += g.x;
                            if (a.y == id) acc[r][1] += g.y;
                            if (a.z == id) acc[r][2] += g.z;
                            if (a.w == id) acc[r][3] += g.w;
                        }
                    }
                }
            }
        }
        const uint32_t bhw = (b * (uint32_t)H + iy) * (uint32_t)W + ix;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (r >= nr) break;
            const float4 v = make_float4(acc[r][0], acc[r][1], acc[r][2], acc[r][3]);
            if (HALO) {
                bool hal;
                const uint32_t zo = pool_zoff<true>(hz, bhw, D, iz0 + r, C4, hal);
                (hal ? hz.dh : dx)[zo + c] = v;
            } else {
                dx[(bhw * (uint32_t)D + iz0 + r) * (uint32_t)C4 + c] = v;
            }
        }
    }
}

constexpr int POOL_ZRUN = 8;

// IDX: the index type of the element loop (uint32_t when the source has < 2^32
// float4s: the 64-bit div/mod of the decomposition are software sequences)
template <typename IDX>
__global__ void upsample221_bwd_kernel(const float4* __restrict__ dup, int B, int H, int W, int D,
                                       int C4, float4* __restrict__ dsrc, int accumulate) {
    const IDX total = (IDX)B * H * W * D * C4;
    for (IDX i = (IDX)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (IDX)gridDim.x * blockDim.x) {
        const int c = (int)(i % (IDX)C4);
        IDX t = i / (IDX)C4;
        const int z = (int)(t % (IDX)D); t /= (IDX)D;
        const int x = (int)(t % (IDX)W); t /= (IDX)W;
        const int y = (int)(t % (IDX)H);
        const int b = (int)(t / (IDX)H);
        float4 acc = accumulate ? dsrc[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        for (int a = 0; a < 2; ++a)
            for (int q = 0; q < 2; ++q) {
                const float4 v = dup[((((int64_t)b * 2 * H + 2 * y + a) * 2 * W + 2 * x + q) * D + z) * C4 + c];
                acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
            }
        dsrc[i] = acc;
    }
}

__global__ void subsample221_kernel(const float4* __restrict__ src, int B, int H, int W, int D,
                                    int C4, float4* __restrict__ dst, int bwd) {
    const int OH = (H + 1) / 2, OW = (W + 1) / 2;
    const int64_t total = (int64_t)B * OH * OW * D * C4;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(i % C4);
        int64_t t = i / C4;
        const int z = (int)(t % D); t /= D;
        const int x = (int)(t % OW); t /= OW;
        const int y = (int)(t % OH);
        const int b = (int)(t / OH);
        const int64_t full = ((((int64_t)b * H + 2 * y) * W + 2 * x) * D + z) * C4 + c;
        if (!bwd) {
            dst[i] = src[full];
        } else {
            float4 a = dst[full];
            const float4 v = src[i];
            a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
            dst[full] = a;
        }
    }
}

// rows per loop iteration with all their loads first (A/B builds: 2 and 4
// measured 28.42-28.46 / 28.57-28.59 ms per 128^3 step against 28.31-28.42
// for 1, scripts/gpu_bn_unroll.sh -- the kernel is not latency-bound there)
#ifndef BN_UNROLL
#define BN_UNROLL 1
#endif
// Thread layout: T threads per row cover T channel quads; R = 256/T rows per
// block pass; gridDim.y channel groups of 4*T channels.  Each block writes its
// per-channel partial sums to part[3][gridDim.x][C] (no contended atomics);
// bn_sums_reduce_kernel then folds them in a fixed order (deterministic).
// splits > 1: dy is the K-slice partials of a split-K data gradient (slice k
// at dy + k * plane), summed in slice order as splitk_epi_kernel does; acc_dz:
// dz holds the data gradient's earlier contribution, added after the slices
// (the accumulated store's order) and overwritten in place by dz -- the fused
// split-K form of m3d_conv3d_bwd_data_splitk + this kernel.
__global__ __launch_bounds__(256) void bn_act_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ y, const float* __restrict__ z,
    int64_t M, int C, int T, int relu, const float* __restrict__ scale,
    const float* __restrict__ mean, const float* __restrict__ rstd, float* dz,
    float* __restrict__ dres, int accumulate_res, int want_xhat, float* __restrict__ part,
    int splits = 1, int64_t plane = 0, int acc_dz = 0) {
    const int R = 256 / T;
    const int tx = threadIdx.x % T, ty = threadIdx.x / T;
    const int c = (blockIdx.y * T + tx) * 4;
    float s_p[4] = {0, 0, 0, 0}, s_x[4] = {0, 0, 0, 0}, s_z[4] = {0, 0, 0, 0};
    if (c < C) {
        float sc[4] = {1, 1, 1, 1}, mu[4] = {0, 0, 0, 0}, rs[4] = {1, 1, 1, 1};
        if (scale) { const float4 v = *(const float4*)(scale + c); sc[0] = v.x; sc[1] = v.y; sc[2] = v.z; sc[3] = v.w; }
        if (mean) { const float4 v = *(const float4*)(mean + c); mu[0] = v.x; mu[1] = v.y; mu[2] = v.z; mu[3] = v.w; }
        if (rstd) { const float4 v = *(const float4*)(rstd + c); rs[0] = v.x; rs[1] = v.y; rs[2] = v.z; rs[3] = v.w; }
        // BN_UNROLL rows per iteration, all their loads issued before any use
        const int64_t step = (int64_t)gridDim.x * R;
        for (int64_t r0 = (int64_t)blockIdx.x * R + ty; r0 < M; r0 += BN_UNROLL * step) {
            float4 g4[BN_UNROLL], y4[BN_UNROLL], z4[BN_UNROLL], a4[BN_UNROLL];
#pragma unroll
            for (int u = 0; u < BN_UNROLL; ++u) {
                const int64_t r = r0 + u * step;
                const bool in = r < M;
                const int64_t off = (in ? r : r0) * C + c;
                g4[u] = *(const float4*)(dy + off);
                for (int k = 1; k < splits; ++k) {
                    const float4 t = *(const float4*)(dy + k * plane + off);
                    g4[u].x += t.x; g4[u].y += t.y; g4[u].z += t.z; g4[u].w += t.w;
                }
                if (acc_dz) {
                    const float4 t = *(const float4*)(dz + off);
                    g4[u].x += t.x; g4[u].y += t.y; g4[u].z += t.z; g4[u].w += t.w;
                }
                y4[u] = relu ? *(const float4*)(y + off) : make_float4(1.f, 1.f, 1.f, 1.f);
                z4[u] = want_xhat ? *(const float4*)(z + off) : make_float4(0.f, 0.f, 0.f, 0.f);
                a4[u] = (dres && accumulate_res) ? *(const float4*)(dres + off) : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < BN_UNROLL; ++u) {
                const int64_t r = r0 + u * step;
                if (r >= M) break;
                const int64_t off = r * C + c;
                float g[4] = {g4[u].x, g4[u].y, g4[u].z, g4[u].w};
                if (relu) {
                    if (!(y4[u].x > 0.f)) g[0] = 0.f;
                    if (!(y4[u].y > 0.f)) g[1] = 0.f;
                    if (!(y4[u].z > 0.f)) g[2] = 0.f;
                    if (!(y4[u].w > 0.f)) g[3] = 0.f;
                }
                const float zz[4] = {z4[u].x, z4[u].y, z4[u].z, z4[u].w};
                float d[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    d[q] = g[q] * sc[q];
                    s_p[q] += g[q];
                    s_x[q] += g[q] * ((zz[q] - mu[q]) * rs[q]);
                    s_z[q] += d[q];
                }
                if (dz) *(float4*)(dz + off) = make_float4(d[0], d[1], d[2], d[3]);
                if (dres) {
                    float4 o = make_float4(g[0], g[1], g[2], g[3]);
                    if (accumulate_res) { o.x += a4[u].x; o.y += a4[u].y; o.z += a4[u].z; o.w += a4[u].w; }
                    *(float4*)(dres + off) = o;
                }
            }
        }
    }
    if (!part) return;          // elementwise only (block-uniform): no channel sums
    __shared__ float red[3][256][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        red[0][threadIdx.x][q] = s_p[q];
        red[1][threadIdx.x][q] = s_x[q];
        red[2][threadIdx.x][q] = s_z[q];
    }
    __syncthreads();
    for (int step = R / 2; step > 0; step >>= 1) {
        if (ty < step) {
            const int o = threadIdx.x + step * T;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                red[0][threadIdx.x][q] += red[0][o][q];
                red[1][threadIdx.x][q] += red[1][o][q];
                red[2][threadIdx.x][q] += red[2][o][q];
            }
        }
        __syncthreads();
    }
    if (ty == 0 && c < C) {
        const int64_t gx = gridDim.x;
#pragma unroll
        for (int a = 0; a < 3; ++a)
            *(float4*)(part + ((int64_t)a * gx + blockIdx.x) * C + c) =
                make_float4(red[a][tx][0], red[a][tx][1], red[a][tx][2], red[a][tx][3]);
    }
}

// out_a[c] += sum_b part[a][b][c].  grid (ceil(C/16), 3); 256 threads =
// 4 channel quads (float4) x 64 row groups, each with 4 independent
// accumulators, folded by a fixed LDS tree (deterministic).  64 row groups keep
// the serial chain short for the 2048-block partials of bn_act_bwd_kernel.
// The fold of one [gx][C] partial array into dst (block blockIdx.x's 16
// channels); every thread of the block calls it.
__device__ __forceinline__ void bn_sums_fold(const float* __restrict__ part, int gx, int C, float* __restrict__ dst) {
    const int tq = threadIdx.x & 3, rg = threadIdx.x >> 2;
    const int c = blockIdx.x * 16 + tq * 4;
    float4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    if (c < C) {
        const float* p = part + c;
        int b = rg;
        for (; b + 192 < gx; b += 256) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const float4 v = *(const float4*)(p + (int64_t)(b + 64 * u) * C);
                acc[u].x += v.x; acc[u].y += v.y; acc[u].z += v.z; acc[u].w += v.w;
            }
        }
        for (; b < gx; b += 64) {
            const float4 v = *(const float4*)(p + (int64_t)b * C);
            acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
        }
    }
    __shared__ float4 red[64][4];
    red[rg][tq] = make_float4((acc[0].x + acc[1].x) + (acc[2].x + acc[3].x),
                              (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y),
                              (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z),
                              (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w));
    __syncthreads();
    for (int step = 32; step > 0; step >>= 1) {
        if (rg < step) {
            const float4 o = red[rg + step][tq];
            float4 m = red[rg][tq];
            m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
            red[rg][tq] = m;
        }
        __syncthreads();
    }
    if (rg == 0 && c < C) {
        const float4 r = red[0][tq];
        dst[c] += r.x; dst[c + 1] += r.y; dst[c + 2] += r.z; dst[c + 3] += r.w;
    }
}

__global__ __launch_bounds__(256) void bn_sums_reduce_kernel(const float* __restrict__ part, int gx,
                                                             int C, float* __restrict__ s0,
                                                             float* __restrict__ s1,
                                                             float* __restrict__ s2) {
    const int a = blockIdx.y;
    float* dst = a == 0 ? s0 : (a == 1 ? s1 : s2);
    if (!dst) return;
    bn_sums_fold(part + (int64_t)a * gx * C, gx, C, dst);
}

// ---- Keras SGD over a flat parameter buffer split into segments padded to
// multiples of 1024 floats; chunk c (1024 floats) belongs to seg_of_chunk[c].
// Each block folds SGD_NORM_CHUNKS consecutive chunks and issues one atomic
// per segment it touches (was one per 1024-float chunk: ~57k atomics onto
// ~160 addresses per step).  The segment of a chunk is block-uniform.
constexpr int SGD_NORM_CHUNKS = 16;
__global__ __launch_bounds__(256) void sgd_norm_kernel(const float* __restrict__ w,
                                                       const float* __restrict__ g,
                                                       const int32_t* __restrict__ seg_of_chunk,
                                                       const float* __restrict__ l2, int64_t n_chunks,
                                                       float* __restrict__ norms) {
    __shared__ float red[4];
    const int64_t ch0 = (int64_t)blockIdx.x * SGD_NORM_CHUNKS;
    const int64_t ch1 = ch0 + SGD_NORM_CHUNKS < n_chunks ? ch0 + SGD_NORM_CHUNKS : n_chunks;
    int cur = seg_of_chunk[ch0];
    float s = 0.0f;
    auto flush = [&]() {
        float r = s;
        for (int o = 32; o > 0; o >>= 1) r += __shfl_xor(r, o);
        if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = r;
        __syncthreads();
        if (threadIdx.x == 0) unsafeAtomicAdd(norms + cur, red[0] + red[1] + red[2] + red[3]);
        __syncthreads();
        s = 0.0f;
    };
    for (int64_t ch = ch0; ch < ch1; ++ch) {
        const int seg = seg_of_chunk[ch];
        if (seg != cur) {
            flush();
            cur = seg;
        }
        const float lc = l2[seg];
        const int64_t off = ch * 1024 + threadIdx.x * 4;
        const float4 wv = *(const float4*)(w + off), gv = *(const float4*)(g + off);
        const float a = gv.x + lc * wv.x, b = gv.y + lc * wv.y, c = gv.z + lc * wv.z, d = gv.w + lc * wv.w;
        s += a * a + b * b + c * c + d * d;
    }
    flush();
}

// Deterministic mode: chunk_norm_kernel writes each chunk's sum of squares
// (fixed reduction tree) to part[chunk]; seg_norm_kernel (one block per
// segment) adds the chunks of its segment in chunk order per thread and a
// fixed tree across threads.  No assumption on the chunk -> segment order.
__device__ __forceinline__ float block_sum256(float v, float* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    const float r = (red[0] + red[1]) + (red[2] + red[3]);
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(256) void chunk_norm_kernel(const float* __restrict__ w,
                                                         const float* __restrict__ g,
                                                         const int32_t* __restrict__ seg_of_chunk,
                                                         const float* __restrict__ l2,
                                                         float* __restrict__ part) {
    __shared__ float red[4];
    const int64_t ch = blockIdx.x;
    const float lc = l2[seg_of_chunk[ch]];
    const int64_t off = ch * 1024 + threadIdx.x * 4;
    const float4 wv = *(const float4*)(w + off), gv = *(const float4*)(g + off);
    const float a = gv.x + lc * wv.x, b = gv.y + lc * wv.y, c = gv.z + lc * wv.z, d = gv.w + lc * wv.w;
    const float r = block_sum256(a * a + b * b + c * c + d * d, red);
    if (threadIdx.x == 0) part[ch] = r;
}

__global__ __launch_bounds__(256) void seg_norm_kernel(const int32_t* __restrict__ seg_of_chunk,
                                                       const float* __restrict__ part, int64_t n_chunks,
                                                       float* __restrict__ norms) {
    __shared__ float red[4];
    const int seg = blockIdx.x;
    float s = 0.0f;
    for (int64_t c = threadIdx.x; c < n_chunks; c += 256)
        if (seg_of_chunk[c] == seg) s += part[c];
    const float r = block_sum256(s, red);
    if (threadIdx.x == 0) norms[seg] = r;
}

__global__ __launch_bounds__(256) void sgd_update_kernel(float* __restrict__ w,
                                                         const float* __restrict__ g,
                                                         float* __restrict__ v,
                                                         const int32_t* __restrict__ seg_of_chunk,
                                                         const float* __restrict__ l2,
                                                         const float* __restrict__ norms, float lr,
                                                         float momentum, float clipnorm) {
    const int64_t ch = blockIdx.x;
    const int seg = seg_of_chunk[ch];
    const float lc = l2[seg];
    const float nrm = clipnorm > 0.f ? sqrtf(norms[seg]) : 0.0f;
    const float den = clipnorm > 0.f ? (nrm > clipnorm ? nrm : clipnorm) : 1.0f;
    const float num = clipnorm > 0.f ? clipnorm : 1.0f;
    const int64_t off = ch * 1024 + threadIdx.x * 4;
    float4 wv = *(float4*)(w + off), vv = *(float4*)(v + off);
    const float4 gv = *(const float4*)(g + off);
    float gg[4] = {gv.x + lc * wv.x, gv.y + lc * wv.y, gv.z + lc * wv.z, gv.w + lc * wv.w};
    float* wp = &wv.x;
    float* vp = &vv.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float gc = (gg[q] * num) / den;          // tf.clip_by_norm
        vp[q] = momentum * vp[q] - lr * gc;            // Keras SGD velocity
        wp[q] = wp[q] + vp[q];
    }
    *(float4*)(w + off) = wv;
    *(float4*)(v + off) = vv;
}

// ---- Keras 2.3.1 Adam / Adadelta over the same flat, chunked buffers
// (core/models.py:3349-3357 picks them by OPTIMIZER.name).  Per element, in
// the op order of keras/optimizers.py (compiled -ffp-contract=off):
//   Adam:     m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*(g*g);
//             [amsgrad: vh = max(vh, v), v' = vh]   p -= (lr_t*m) / (sqrt(v') + eps)
//             (lr_t = lr*sqrt(1-b2^t)/(1-b1^t) is a host scalar)
//   Adadelta: a = rho*a + (1-rho)*(g*g);  u = (g*sqrt(d+eps)) / sqrt(a+eps);
//             p -= lr*u;  d = rho*d + (1-rho)*(u*u)
// where g is the tf.clip_by_norm'd gradient plus the L2 term, as for SGD.
template <int MODE>
__global__ __launch_bounds__(256) void adaptive_update_kernel(
        float* __restrict__ w, const float* __restrict__ g, float* __restrict__ s1,
        float* __restrict__ s2, float* __restrict__ s3, const int32_t* __restrict__ seg_of_chunk,
        const float* __restrict__ l2, const float* __restrict__ norms, float lr, float c1,
        float c1m, float c2, float c2m, float eps, float clipnorm) {
    const int64_t ch = blockIdx.x;
    const int seg = seg_of_chunk[ch];
    const float lc = l2[seg];
    const float nrm = clipnorm > 0.f ? sqrtf(norms[seg]) : 0.0f;
    const float den = clipnorm > 0.f ? (nrm > clipnorm ? nrm : clipnorm) : 1.0f;
    const float num = clipnorm > 0.f ? clipnorm : 1.0f;
    const int64_t off = ch * 1024 + threadIdx.x * 4;
    float4 wv = *(float4*)(w + off), av = *(float4*)(s1 + off), bv = *(float4*)(s2 + off);
    float4 hv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (MODE == 1) hv = *(float4*)(s3 + off);
    const float4 gv = *(const float4*)(g + off);
    const float gg[4] = {gv.x + lc * wv.x, gv.y + lc * wv.y, gv.z + lc * wv.z, gv.w + lc * wv.w};
    float* wp = &wv.x;
    float* ap = &av.x;
    float* bp = &bv.x;
    float* hp = &hv.x;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float gc = (gg[q] * num) / den;                  // tf.clip_by_norm
        if (MODE <= 1) {                                       // Adam (1: amsgrad)
            const float m = c1 * ap[q] + c1m * gc;
            const float v = c2 * bp[q] + c2m * (gc * gc);
            float vd = v;
            if (MODE == 1) {
                hp[q] = hp[q] > v ? hp[q] : v;
                vd = hp[q];
            }
            wp[q] = wp[q] - (lr * m) / (sqrtf(vd) + eps);
            ap[q] = m;
            bp[q] = v;
        } else {                                               // Adadelta
            const float a = c1 * ap[q] + c1m * (gc * gc);
            const float u = (gc * sqrtf(bp[q] + eps)) / sqrtf(a + eps);
            wp[q] = wp[q] - lr * u;
            ap[q] = a;
            bp[q] = c1 * bp[q] + c1m * (u * u);
        }
    }
    *(float4*)(w + off) = wv;
    *(float4*)(s1 + off) = av;
    *(float4*)(s2 + off) = bv;
    if (MODE == 1) *(float4*)(s3 + off) = hv;
}

}  // namespace m3d

using namespace m3d;

static unsigned ew_grid(int64_t n) { return grid_for(n, 256, 256 * 32); }

// KL.MaxPooling3D argument checks (the kernels index with 32-bit ints)
static int check_pool_args(int64_t B, int64_t H, int64_t W, int64_t D, int64_t C, int kh, int kw, int kd,
                           int sy, int sx, int sz, int py, int px, int pz, int64_t OH, int64_t OW, int64_t OD) {
    if (B < 0 || H <= 0 || W <= 0 || D <= 0 || C <= 0 || OH <= 0 || OW <= 0 || OD <= 0)
        return einval("maxpool3d: dimensions must be positive");
    if (kh <= 0 || kw <= 0 || kd <= 0) return einval("maxpool3d: pool size must be positive");
    if (kh * kw * kd > 255) return einval("maxpool3d: window larger than 255");
    if (sy <= 0 || sx <= 0 || sz <= 0) return einval("maxpool3d: strides must be positive");
    if (py < 0 || px < 0 || pz < 0) return einval("maxpool3d: padding must be non-negative");
    if (B * H * W * D * C > 0x7FFFFFFFll || B * OH * OW * OD * C > 0x7FFFFFFFll)
        return einval("maxpool3d: tensor larger than 2^31 elements");
    return M3D_OK;
}

static int check_resample_args(const char* what, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C) {
    if (B < 0 || H < 0 || W < 0 || D < 0 || C < 0) return einval(what);
    if (C % 4) return einval("C must be a multiple of 4");
    if (B * H * W * D * C > 0x7FFFFFFFll) return einval("tensor larger than 2^31 elements");
    return M3D_OK;
}

extern "C" int m3d_maxpool3d_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                 int64_t C, int32_t kh, int32_t kw, int32_t kd, int32_t sy,
                                 int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                                 int64_t OH, int64_t OW, int64_t OD, float* y, uint8_t* argmax,
                                 m3d_stream_t s) {
    int rc = check_pool_args(B, H, W, D, C, kh, kw, kd, sy, sx, sz, py, px, pz, OH, OW, OD);
    if (rc) return rc;
    const int64_t total = B * OH * OW * OD * C;
    if (total == 0) return M3D_OK;
    if (C % 4 == 0 && B * H * W * D * C / 4 < 0x7FFFFFFF && total / 4 < 0x7FFFFFFF &&
        ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0 && ((uintptr_t)argmax & 3) == 0) {
        if (sz == 1 && kh == 3 && kw == 3 && kd == 3 && sy == 2 && sx == 2 && OD == D && pz == 1 &&
            py == (2 - (H - 1) % 2) / 2 && px == (2 - (W - 1) % 2) / 2 && OH == (H + 1) / 2 && OW == (W + 1) / 2) {
            const int nrun = (int)((OD + POOL_ZRUN - 1) / POOL_ZRUN);
            const int64_t nt = B * OH * OW * nrun * (C / 4);
            hipLaunchKernelGGL((maxpool_fwd333_kernel<POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                               (const float4*)x, (int)H, (int)W, (int)D, (int)(C / 4), (int)OH, (int)OW, nrun,
                               (uint32_t)nt, (float4*)y, (uchar4*)argmax);
            return check_launch("maxpool_fwd333_kernel");
        }
        if (sz == 1) {
            const int nrun = (int)((OD + POOL_ZRUN - 1) / POOL_ZRUN);
            const int64_t nt = B * OH * OW * nrun * (C / 4);
            hipLaunchKernelGGL((maxpool_fwd4z_kernel<false, POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                               (const float4*)x, (int)H, (int)W, (int)D, (int)(C / 4), kh, kw, kd, sy, sx, py, px,
                               pz, (int)OH, (int)OW, (int)OD, nrun, (uint32_t)nt, (float4*)y, (uchar4*)argmax,
                               PoolHalo{});
            return check_launch("maxpool_fwd4z_kernel");
        }
        hipLaunchKernelGGL(maxpool_fwd4_kernel<false>, dim3(ew_grid(total / 4)), dim3(256), 0, st(s),
                           (const float4*)x, (int)H, (int)W, (int)D, (int)(C / 4), kh, kw, kd, sy, sx, sz,
                           py, px, pz, (int)OH, (int)OW, (int)OD, (uint32_t)(total / 4), (float4*)y,
                           (uchar4*)argmax, PoolHalo{});
        return check_launch("maxpool_fwd4_kernel");
    }
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(ew_grid(total)), dim3(256), 0, st(s), x, (int)B,
                       (int)H, (int)W, (int)D, (int)C, kh, kw, kd, sy, sx, sz, py, px, pz, (int)OH,
                       (int)OW, (int)OD, y, argmax);
    return check_launch("maxpool_fwd_kernel");
}

extern "C" int m3d_maxpool3d_bwd(const float* dy, const uint8_t* argmax, int64_t B, int64_t H,
                                 int64_t W, int64_t D, int64_t C, int32_t kh, int32_t kw,
                                 int32_t kd, int32_t sy, int32_t sx, int32_t sz, int32_t py,
                                 int32_t px, int32_t pz, int64_t OH, int64_t OW, int64_t OD,
                                 float* dx, m3d_stream_t s) {
    int rc = check_pool_args(B, H, W, D, C, kh, kw, kd, sy, sx, sz, py, px, pz, OH, OW, OD);
    if (rc) return rc;
    const int64_t total = B * H * W * D * C;
    if (total == 0) return M3D_OK;
    if (C % 4 == 0 && total / 4 < 0x7FFFFFFF && B * OH * OW * OD * C / 4 < 0x7FFFFFFF &&
        ((uintptr_t)dy & 15) == 0 && ((uintptr_t)dx & 15) == 0 && ((uintptr_t)argmax & 3) == 0) {
        if (sz == 1 && kh == 3 && kw == 3 && kd == 3 && sy == 2 && sx == 2 && OD == D && pz == 1 &&
            py == (2 - (H - 1) % 2) / 2 && px == (2 - (W - 1) % 2) / 2 && OH == (H + 1) / 2 && OW == (W + 1) / 2) {
            const int nrun = (int)((D + POOL_ZRUN - 1) / POOL_ZRUN);
            const int64_t nt = B * H * W * nrun * (C / 4);
            hipLaunchKernelGGL((maxpool_bwd333_kernel<POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                               (const float4*)dy, (const uchar4*)argmax, (int)H, (int)W, (int)D, (int)(C / 4),
                               (int)OH, (int)OW, nrun, (uint32_t)nt, (float4*)dx);
            return check_launch("maxpool_bwd333_kernel");
        }
        if (sz == 1) {
            const int nrun = (int)((D + POOL_ZRUN - 1) / POOL_ZRUN);
            const int64_t nt = B * H * W * nrun * (C / 4);
            hipLaunchKernelGGL((maxpool_bwd4z_kernel<false, POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                               (const float4*)dy, (const uchar4*)argmax, (int)H, (int)W, (int)D, (int)(C / 4), kh,
                               kw, kd, sy, sx, py, px, pz, (int)OH, (int)OW, (int)OD, nrun, (uint32_t)nt,
                               (float4*)dx, PoolHalo{});
            return check_launch("maxpool_bwd4z_kernel");
        }
        hipLaunchKernelGGL(maxpool_bwd4_kernel<false>, dim3(ew_grid(total / 4)), dim3(256), 0, st(s),
                           (const float4*)dy, (const uchar4*)argmax, (int)H, (int)W, (int)D, (int)(C / 4),
                           kh, kw, kd, sy, sx, sz, py, px, pz, (int)OH, (int)OW, (int)OD,
                           (uint32_t)(total / 4), (float4*)dx, PoolHalo{});
        return check_launch("maxpool_bwd4_kernel");
    }
    hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(ew_grid(total)), dim3(256), 0, st(s), dy, argmax,
                       (int)B, (int)H, (int)W, (int)D, (int)C, kh, kw, kd, sy, sx, sz, py, px, pz,
                       (int)OH, (int)OW, (int)OD, dx);
    return check_launch("maxpool_bwd_kernel");
}

// Depth-slab form (core/models.py:246 MaxPooling3D on the slab): x is the
// local slab [B,H,W,Dl,C], halo [B,H,W,2r,C] the neighbours' r boundary planes
// (has_lo / has_hi: present), z window kd = 2r + 1 at z-stride 1 with the 'same'
// z pad r only where the volume ends; y / argmax [B,OH,OW,Dl,C].
static int pool_halo_args(const float* x, const float* h, int64_t B, int64_t H, int64_t W, int64_t Dl,
                          int64_t C, int32_t kd, int32_t sz, int32_t pz, int32_t r, int64_t OD) {
    if (!x || !h) return einval("maxpool3d_halo: null slab or halo");
    if (C % 4 || ((uintptr_t)x & 15) || ((uintptr_t)h & 15))
        return einval("maxpool3d_halo: C % 4 == 0 and 16-B aligned tensors required");
    if (r <= 0 || kd != 2 * r + 1 || sz != 1 || pz != r || OD != Dl || Dl < r)
        return einval("maxpool3d_halo: z window must be 'same' 2r+1 at stride 1 on a slab of >= r planes");
    if (B * H * W * (Dl + 2 * r) * C / 4 >= 0x7FFFFFFF) return einval("maxpool3d_halo: tensor too large");
    return M3D_OK;
}

extern "C" int m3d_maxpool3d_fwd_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi,
                                      int32_t r, int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t C,
                                      int32_t kh, int32_t kw, int32_t kd, int32_t sy, int32_t sx, int32_t sz,
                                      int32_t py, int32_t px, int32_t pz, int64_t OH, int64_t OW, int64_t OD,
                                      float* y, uint8_t* argmax, m3d_stream_t s) {
    const int nlo = has_lo ? r : 0, nhi = has_hi ? r : 0;
    const int64_t D = Dl + nlo + nhi;
    int rc = check_pool_args(B, H, W, D, C, kh, kw, kd, sy, sx, sz, py, px, pz - nlo, OH, OW, OD);
    if (rc) return rc;
    if ((rc = pool_halo_args(x, halo, B, H, W, Dl, C, kd, sz, pz, r, OD))) return rc;
    if (!y || !argmax || ((uintptr_t)y & 15) || ((uintptr_t)argmax & 3))
        return einval("maxpool3d_halo: y / argmax must be aligned");
    const int64_t total = B * OH * OW * OD * C;
    if (total == 0) return M3D_OK;
    PoolHalo hz{(const float4*)halo, nullptr, nlo, (int)Dl, r};
    const int nrun = (int)((OD + POOL_ZRUN - 1) / POOL_ZRUN);      // (sz == 1: pool_halo_args)
    const int64_t nt = B * OH * OW * nrun * (C / 4);
    hipLaunchKernelGGL((maxpool_fwd4z_kernel<true, POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                       (const float4*)x, (int)H, (int)W, (int)D, (int)(C / 4), kh, kw, kd, sy, sx, py, px,
                       pz - nlo, (int)OH, (int)OW, (int)OD, nrun, (uint32_t)nt, (float4*)y, (uchar4*)argmax, hz);
    return check_launch("maxpool_fwd4z_kernel<halo>");
}

// Backward of m3d_maxpool3d_fwd_halo: dx [B,H,W,Dl,C] (the slab's own planes)
// and dhalo [B,H,W,2r,C] (the gradient of the neighbours' planes, to be sent
// back: m3d.slab.return_halo_grads); planes of an absent neighbour are not written.
extern "C" int m3d_maxpool3d_bwd_halo(const float* dy, const uint8_t* argmax, int32_t has_lo, int32_t has_hi,
                                      int32_t r, int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t C,
                                      int32_t kh, int32_t kw, int32_t kd, int32_t sy, int32_t sx, int32_t sz,
                                      int32_t py, int32_t px, int32_t pz, int64_t OH, int64_t OW, int64_t OD,
                                      float* dx, float* dhalo, m3d_stream_t s) {
    const int nlo = has_lo ? r : 0, nhi = has_hi ? r : 0;
    const int64_t D = Dl + nlo + nhi;
    int rc = check_pool_args(B, H, W, D, C, kh, kw, kd, sy, sx, sz, py, px, pz - nlo, OH, OW, OD);
    if (rc) return rc;
    if ((rc = pool_halo_args(dx, dhalo, B, H, W, Dl, C, kd, sz, pz, r, OD))) return rc;
    if (!dy || !argmax || ((uintptr_t)dy & 15) || ((uintptr_t)argmax & 3))
        return einval("maxpool3d_halo: dy / argmax must be aligned");
    const int64_t total = B * H * W * D * C;
    if (total == 0) return M3D_OK;
    PoolHalo hz{nullptr, (float4*)dhalo, nlo, (int)Dl, r};
    const int nrun = (int)((D + POOL_ZRUN - 1) / POOL_ZRUN);       // the virtual grid [lo halo | slab | hi halo]
    const int64_t nt = B * H * W * nrun * (C / 4);
    hipLaunchKernelGGL((maxpool_bwd4z_kernel<true, POOL_ZRUN>), dim3(ew_grid(nt)), dim3(256), 0, st(s),
                       (const float4*)dy, (const uchar4*)argmax, (int)H, (int)W, (int)D, (int)(C / 4), kh, kw, kd,
                       sy, sx, py, px, pz - nlo, (int)OH, (int)OW, (int)OD, nrun, (uint32_t)nt, (float4*)dx, hz);
    return check_launch("maxpool_bwd4z_kernel<halo>");
}

extern "C" int m3d_upsample221_bwd(const float* d_up, int64_t B, int64_t H, int64_t W, int64_t D,
                                   int64_t C, float* d_src, int32_t accumulate, m3d_stream_t s) {
    if (int rc = check_resample_args("upsample221_bwd: negative dimension", B, H, W, D, C)) return rc;
    if (C == 0) return einval("upsample221_bwd: C must be a positive multiple of 4");
    const int64_t total = B * H * W * D * (C / 4);
    if (total == 0) return M3D_OK;
    if (total + (int64_t)ew_grid(total) * 256 < ((int64_t)1 << 32))
        hipLaunchKernelGGL(upsample221_bwd_kernel<uint32_t>, dim3(ew_grid(total)), dim3(256), 0, st(s),
                           (const float4*)d_up, (int)B, (int)H, (int)W, (int)D, (int)(C / 4),
                           (float4*)d_src, accumulate);
    else
        hipLaunchKernelGGL(upsample221_bwd_kernel<int64_t>, dim3(ew_grid(total)), dim3(256), 0, st(s),
                           (const float4*)d_up, (int)B, (int)H, (int)W, (int)D, (int)(C / 4),
                           (float4*)d_src, accumulate);
    return check_launch("upsample221_bwd_kernel");
}

extern "C" int m3d_subsample221_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                    int64_t C, float* y, m3d_stream_t s) {
    if (int rc = check_resample_args("subsample221: negative dimension", B, H, W, D, C)) return rc;
    const int64_t total = B * ((H + 1) / 2) * ((W + 1) / 2) * D * (C / 4);
    if (total == 0) return M3D_OK;
    hipLaunchKernelGGL(subsample221_kernel, dim3(ew_grid(total)), dim3(256), 0, st(s),
                       (const float4*)x, (int)B, (int)H, (int)W, (int)D, (int)(C / 4), (float4*)y, 0);
    return check_launch("subsample221_kernel");
}

extern "C" int m3d_subsample221_bwd(const float* dy, int64_t B, int64_t H, int64_t W, int64_t D,
                                    int64_t C, float* dx, m3d_stream_t s) {
    if (int rc = check_resample_args("subsample221: negative dimension", B, H, W, D, C)) return rc;
    const int64_t total = B * ((H + 1) / 2) * ((W + 1) / 2) * D * (C / 4);
    if (total == 0) return M3D_OK;
    hipLaunchKernelGGL(subsample221_kernel, dim3(ew_grid(total)), dim3(256), 0, st(s),
                       (const float4*)dy, (int)B, (int)H, (int)W, (int)D, (int)(C / 4), (float4*)dx, 1);
    return check_launch("subsample221_kernel(bwd)");
}

// total bn_act_bwd blocks (M3D_BN_BLOCKS, default 1024 = 4 per CU).  Alone the
// kernel streams best at 2048 (512 reached ~2.7 TB/s); inside the training
// step, beside the weight-gradient stream, 1024 is faster (step 32.1 -> 31.9 ms
// at 128^3, 512: 32.4 ms; scripts/gpu_step_ab.sh, round 2) and halves the
// partial rows bn_sums_reduce_kernel folds.
static int bn_blocks_env() {
    static constexpr int v = M3D_TUNE_BN_BLOCKS;
    return v > 0 ? v : 1024;
}
static void bn_grid(int64_t M, int64_t C, int& T, int& groups, int64_t& gx) {
    const int quads = (int)(C / 4);
    T = 1;
    while (T < quads && T < 256) T <<= 1;
    groups = (quads + T - 1) / T;
    const int R = 256 / T;
    gx = (M + R - 1) / R;
    const int64_t cap = bn_blocks_env() / groups > 0 ? bn_blocks_env() / groups : 1;
    if (gx > cap) gx = cap;
    if (gx < 1) gx = 1;
}

namespace m3d {
// Frozen-BN affine of one layer in one launch: rstd = 1/sqrt(var + eps),
// scale = gamma * rstd, shift = beta - mean * scale (BatchNorm inference,
// core/models.py:102-114; replaces five elementwise launches per layer).
__global__ void bn_affine_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                 const float* __restrict__ mean, const float* __restrict__ var,
                                 float eps, int C, float* __restrict__ scale,
                                 float* __restrict__ shift, float* __restrict__ rstd) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float r = 1.0f / sqrtf(var[c] + eps);
    const float sc = gamma[c] * r;
    rstd[c] = r;
    scale[c] = sc;
    shift[c] = beta[c] - mean[c] * sc;
}
}  // namespace m3d

namespace m3d {
// one grid row per BN layer (bn_affine_kernel's expressions)
__global__ void bn_affine_batched_kernel(const m3d_bn_affine_item_t* __restrict__ items) {
    const m3d_bn_affine_item_t it = items[blockIdx.y];
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= it.C) return;
    const float r = 1.0f / sqrtf(it.var[c] + it.eps);
    const float sc = it.gamma[c] * r;
    it.out[c] = r;
    it.out[it.C + c] = sc;
    it.out[2 * it.C + c] = it.beta[c] - it.mean[c] * sc;
}
}  // namespace m3d

extern "C" int m3d_bn_affine_batched(const m3d_bn_affine_item_t* items, int32_t n, int64_t max_c,
                                     m3d_stream_t s) {
    if (n <= 0 || n > 65535 || max_c <= 0 || !items) return einval("bn_affine_batched: bad arguments");
    hipLaunchKernelGGL(bn_affine_batched_kernel, dim3(grid_for(max_c, 256), (unsigned)n), dim3(256), 0, st(s),
                       items);
    return check_launch("bn_affine_batched_kernel");
}

extern "C" int m3d_bn_affine(const float* gamma, const float* beta, const float* mean,
                             const float* var, float eps, int64_t C, float* scale, float* shift,
                             float* rstd, m3d_stream_t s) {
    if (C <= 0) return einval("bn_affine: C must be positive");
    hipLaunchKernelGGL(bn_affine_kernel, dim3(grid_for(C, 256)), dim3(256), 0, st(s), gamma, beta,
                       mean, var, eps, (int)C, scale, shift, rstd);
    return check_launch("bn_affine_kernel");
}

namespace m3d {
// bn_act_bwd_kernel's partial rows for M rows of C channels
int64_t bn_act_bwd_rows(int64_t M, int64_t C) {
    int T, groups;
    int64_t gx;
    bn_grid(M, C, T, groups, gx);
    return gx;
}

// The split-K data gradient's reduce with the fused BN-ReLU backward: dx =
// sum of the K-slice partials (+ dx when accumulating), then bn_act_bwd_kernel's
// maths -- dz into dx, dpre into bn->dres, the channel sums via the workspace.
int bn_act_bwd_splitk(const float* slices, int splits, int64_t M, int64_t C, const m3d_bn_bwd_t* bn,
                      float* dx, int accumulate, void* ws, size_t ws_bytes, hipStream_t s) {
    int T, groups;
    int64_t gx;
    bn_grid(M, C, T, groups, gx);
    const bool sums = bn->sum_dpre || bn->sum_dpre_xhat || bn->sum_dz;
    if (sums && ws_bytes < sizeof(float) * 3 * (size_t)gx * (size_t)C)
        return einval("bwd-data split-K (fused BN backward): workspace too small");
    hipLaunchKernelGGL(bn_act_bwd_kernel, dim3((unsigned)gx, (unsigned)groups), dim3(256), 0, s, slices, bn->y,
                       bn->z, M, (int)C, T, bn->relu ? 1 : 0, bn->scale, bn->mean, bn->rstd, dx, bn->dres, 0,
                       bn->sum_dpre_xhat ? 1 : 0, sums ? (float*)ws : nullptr, splits, M * C, accumulate ? 1 : 0);
    int rc = check_launch("bn_act_bwd_kernel(split-K)");
    if (rc || !sums) return rc;
    return bn_sums_reduce((const float*)ws, gx, C, bn->sum_dpre, bn->sum_dpre_xhat, bn->sum_dz, s);
}

// fold [3][rows][C] channel partials into s0 / s1 / s2 (+=, fixed order; NULL: skipped)
int bn_sums_reduce(const float* part, int64_t rows, int64_t C, float* s0, float* s1, float* s2, hipStream_t s) {
    if (!(s0 || s1 || s2) || rows <= 0) return M3D_OK;
    hipLaunchKernelGGL(bn_sums_reduce_kernel, dim3((unsigned)((C + 15) / 16), 3), dim3(256), 0, s, part,
                       (int)rows, (int)C, s0, s1, s2);
    return check_launch("bn_sums_reduce_kernel(fused)");
}
}  // namespace m3d

extern "C" size_t m3d_bn_act_bwd_workspace_bytes(int64_t M, int64_t C) {
    int T, groups;
    int64_t gx;
    bn_grid(M, C, T, groups, gx);
    return sizeof(float) * 3 * (size_t)gx * (size_t)C;
}

extern "C" int m3d_bn_act_bwd(const float* dy, const float* y, const float* z, int64_t M,
                              int64_t C, int32_t relu, const float* scale, const float* mean,
                              const float* rstd, float* dz, float* dres, int32_t accumulate_res,
                              float* sum_dpre, float* sum_dpre_xhat, float* sum_dz,
                              void* workspace, size_t ws_bytes, m3d_stream_t s) {
    if (C % 4) return einval("bn_act_bwd: C must be a multiple of 4");
    if (relu && !y) return einval("bn_act_bwd: relu needs y");
    if (sum_dpre_xhat && !z) return einval("bn_act_bwd: xhat sums need z");
    if (M == 0) return M3D_OK;
    int T, groups;
    int64_t gx;
    bn_grid(M, C, T, groups, gx);
    const bool sums = sum_dpre || sum_dpre_xhat || sum_dz;
    if (sums && ws_bytes < sizeof(float) * 3 * (size_t)gx * (size_t)C)
        return einval("bn_act_bwd: workspace too small");
    if (!sums && !dz && !dres) return M3D_OK;
    hipLaunchKernelGGL(bn_act_bwd_kernel, dim3((unsigned)gx, (unsigned)groups), dim3(256), 0, st(s),
                       dy, y, z, M, (int)C, T, relu, scale, mean, rstd, dz, dres, accumulate_res,
                       sum_dpre_xhat ? 1 : 0, sums ? (float*)workspace : nullptr);
    int rc = check_launch("bn_act_bwd_kernel");
    if (rc || !sums) return rc;
    hipLaunchKernelGGL(bn_sums_reduce_kernel, dim3((unsigned)((C + 15) / 16), 3), dim3(256), 0, st(s),
                       (const float*)workspace, (int)gx, (int)C, sum_dpre, sum_dpre_xhat, sum_dz);
    return check_launch("bn_sums_reduce_kernel");
}

// ---- batched column sums (m3d_col_sums_batched): every item with
// bn_act_bwd_kernel's block geometry (bn_grid) and summation order, one sum
// instead of three, all items in one launch; then bn_sums_reduce_kernel's fold
// per item, all items in a second launch.  The item table travels by value in
// the kernel arguments (no device copy; capturable in a HIP graph).
struct ColSumsBatch {
    const float* x[M3D_COL_SUMS_MAX];
    float* out[M3D_COL_SUMS_MAX];
    int64_t M[M3D_COL_SUMS_MAX];
    int64_t part[M3D_COL_SUMS_MAX];        // float offset of the item's [gx][C] partial rows
    int C[M3D_COL_SUMS_MAX], T[M3D_COL_SUMS_MAX], gx[M3D_COL_SUMS_MAX];
    int block0[M3D_COL_SUMS_MAX + 1];      // first block of each item in the flat grid
    int n;
};

__global__ __launch_bounds__(256) void col_sums_batched_kernel(const ColSumsBatch b, float* __restrict__ ws) {
    int i = 0;
    while (i + 1 < b.n && (int)blockIdx.x >= b.block0[i + 1]) ++i;
    const int local = (int)blockIdx.x - b.block0[i];
    const int gx = b.gx[i], T = b.T[i], C = b.C[i];
    const int bx = local % gx, by = local / gx;
    const int R = 256 / T;
    const int tx = threadIdx.x % T, ty = threadIdx.x / T;
    const int c = (by * T + tx) * 4;
    const float* __restrict__ x = b.x[i];
    const int64_t M = b.M[i];
    float s[4] = {0, 0, 0, 0};
    if (c < C) {
        const int64_t step = (int64_t)gx * R;
        for (int64_t r = (int64_t)bx * R + ty; r < M; r += step) {
            const float4 v = *(const float4*)(x + r * C + c);
            s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
        }
    }
    __shared__ float red[256][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) red[threadIdx.x][q] = s[q];
    __syncthreads();
    for (int st_ = R / 2; st_ > 0; st_ >>= 1) {
        if (ty < st_) {
            const int o = threadIdx.x + st_ * T;
#pragma unroll
            for (int q = 0; q < 4; ++q) red[threadIdx.x][q] += red[o][q];
        }
        __syncthreads();
    }
    if (ty == 0 && c < C)
        *(float4*)(ws + b.part[i] + (int64_t)bx * C + c) =
            make_float4(red[tx][0], red[tx][1], red[tx][2], red[tx][3]);
}

// grid (ceil(max C / 16), n): item blockIdx.y's partial rows folded into its out
__global__ __launch_bounds__(256) void col_sums_reduce_kernel(const ColSumsBatch b, const float* __restrict__ ws) {
    const int i = blockIdx.y;
    const int C = b.C[i];
    if ((int)blockIdx.x * 16 >= C) return;                 // block-uniform
    bn_sums_fold(ws + b.part[i], b.gx[i], C, b.out[i]);
}

static int col_sums_plan(const m3d_col_sums_item_t* items, int32_t n, ColSumsBatch& b, size_t& ws_floats,
                         int& max_c) {
    if (n < 0 || n > M3D_COL_SUMS_MAX || (n > 0 && !items)) return einval("col_sums_batched: bad item count");
    b = ColSumsBatch{};
    b.n = n;
    ws_floats = 0;
    max_c = 0;
    int blocks = 0;
    for (int i = 0; i < n; ++i) {
        const m3d_col_sums_item_t& it = items[i];
        if (!it.x || !it.out || it.M <= 0 || it.C <= 0 || it.C % 4 || it.C > (1 << 20))
            return einval("col_sums_batched: an item needs x, out, M > 0, C > 0 and C % 4 == 0");
        for (int j = 0; j < i; ++j)
            if (items[j].out == it.out) return einval("col_sums_batched: two items share out");
        int T, groups;
        int64_t gx;
        bn_grid(it.M, it.C, T, groups, gx);
        b.x[i] = it.x;
        b.out[i] = it.out;
        b.M[i] = it.M;
        b.C[i] = (int)it.C;
        b.T[i] = T;
        b.gx[i] = (int)gx;
        b.part[i] = (int64_t)ws_floats;
        b.block0[i] = blocks;
        blocks += (int)gx * groups;
        ws_floats += (size_t)gx * (size_t)it.C;
        if ((int)it.C > max_c) max_c = (int)it.C;
    }
    b.block0[n] = blocks;
    return M3D_OK;
}

extern "C" size_t m3d_col_sums_batched_workspace_bytes(const m3d_col_sums_item_t* items, int32_t n) {
    ColSumsBatch b{};
    size_t f;
    int mc;
    if (col_sums_plan(items, n, b, f, mc) != M3D_OK) return 0;
    return sizeof(float) * f;
}

extern "C" int m3d_col_sums_batched(const m3d_col_sums_item_t* items, int32_t n, void* workspace, size_t ws_bytes,
                                    m3d_stream_t s) {
    ColSumsBatch b{};
    size_t f;
    int max_c;
    int rc = col_sums_plan(items, n, b, f, max_c);
    if (rc) return rc;
    if (n == 0) return M3D_OK;
    if (!workspace || ws_bytes < sizeof(float) * f) return einval("col_sums_batched: workspace too small");
    hipLaunchKernelGGL(col_sums_batched_kernel, dim3((unsigned)b.block0[n]), dim3(256), 0, st(s), b,
                       (float*)workspace);
    rc = check_launch("col_sums_batched_kernel");
    if (rc) return rc;
    hipLaunchKernelGGL(col_sums_reduce_kernel, dim3((unsigned)((max_c + 15) / 16), (unsigned)n), dim3(256), 0, st(s),
                       b, (const float*)workspace);
    return check_launch("col_sums_reduce_kernel");
}

// per-segment squared norms of (grad + l2 * w) for tf.clip_by_norm
static int clip_norms(const float* params, const float* grads, int64_t n_chunks,
                      const int32_t* seg_of_chunk, const float* l2_coef, int32_t n_segments,
                      float clipnorm, float* norms, m3d_stream_t s) {
    if (!(clipnorm > 0.f)) return M3D_OK;
    const DetState d = det();
    if (d.on) {
        if (d.bytes < sizeof(float) * (size_t)n_chunks)
            return einval("clip norms (deterministic mode): scratch smaller than n_chunks floats");
        float* part = static_cast<float*>(d.scratch);
        hipLaunchKernelGGL(chunk_norm_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st(s), params, grads,
                           seg_of_chunk, l2_coef, part);
        int rc = check_launch("chunk_norm_kernel");
        if (rc || n_segments == 0) return rc;
        hipLaunchKernelGGL(seg_norm_kernel, dim3((unsigned)n_segments), dim3(256), 0, st(s), seg_of_chunk,
                           (const float*)part, (int64_t)n_chunks, norms);
        return check_launch("seg_norm_kernel");
    }
    if (hipMemsetAsync(norms, 0, sizeof(float) * n_segments, st(s)) != hipSuccess)
        return check_launch("memset norms");
    hipLaunchKernelGGL(sgd_norm_kernel, dim3((unsigned)((n_chunks + SGD_NORM_CHUNKS - 1) / SGD_NORM_CHUNKS)),
                       dim3(256), 0, st(s), params, grads, seg_of_chunk, l2_coef, (int64_t)n_chunks, norms);
    return check_launch("sgd_norm_kernel");
}

extern "C" int m3d_sgd_keras(float* params, const float* grads, float* moments, int64_t n_chunks,
                             const int32_t* seg_of_chunk, const float* l2_coef, int32_t n_segments,
                             float lr, float momentum, float clipnorm, float* norms,
                             const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    if (n_chunks < 0 || n_segments < 0) return einval("sgd: negative chunk or segment count");
    if (n_chunks == 0) return M3D_OK;
    if (!params || !grads || !moments || !seg_of_chunk || !l2_coef || (clipnorm > 0.f && !norms))
        return einval("sgd: null pointer");
    int rc = clip_norms(params, grads, n_chunks, seg_of_chunk, l2_coef, n_segments, clipnorm, norms, s);
    if (rc) return rc;
    hipLaunchKernelGGL(sgd_update_kernel, dim3((unsigned)n_chunks), dim3(256), 0, st(s), params,
                       grads, moments, seg_of_chunk, l2_coef, norms, lr, momentum, clipnorm);
    return check_launch("sgd_update_kernel");
}

extern "C" int m3d_adam_keras(float* params, const float* grads, float* m, float* v, float* vhat,
                              int64_t n_chunks, const int32_t* seg_of_chunk, const float* l2_coef,
                              int32_t n_segments, float lr_t, float beta_1, float beta_2,
                              float epsilon, float clipnorm, float* norms, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    if (n_chunks < 0 || n_segments < 0) return einval("adam: negative chunk or segment count");
    if (n_chunks == 0) return M3D_OK;
    if (!params || !grads || !m || !v || !seg_of_chunk || !l2_coef || (clipnorm > 0.f && !norms))
        return einval("adam: null pointer");
    int rc = clip_norms(params, grads, n_chunks, seg_of_chunk, l2_coef, n_segments, clipnorm, norms, s);
    if (rc) return rc;
    const float c1m = 1.0f - beta_1, c2m = 1.0f - beta_2;
    if (vhat)
        hipLaunchKernelGGL(adaptive_update_kernel<1>, dim3((unsigned)n_chunks), dim3(256), 0, st(s),
                           params, grads, m, v, vhat, seg_of_chunk, l2_coef, norms, lr_t, beta_1, c1m,
                           beta_2, c2m, epsilon, clipnorm);
    else
        hipLaunchKernelGGL(adaptive_update_kernel<0>, dim3((unsigned)n_chunks), dim3(256), 0, st(s),
                           params, grads, m, v, (float*)nullptr, seg_of_chunk, l2_coef, norms, lr_t,
                           beta_1, c1m, beta_2, c2m, epsilon, clipnorm);
    return check_launch("adaptive_update_kernel<adam>");
}

extern "C" int m3d_adadelta_keras(float* params, const float* grads, float* accum, float* delta_accum,
                                  int64_t n_chunks, const int32_t* seg_of_chunk, const float* l2_coef,
                                  int32_t n_segments, float lr, float rho, float epsilon,
                                  float clipnorm, float* norms, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    if (n_chunks < 0 || n_segments < 0) return einval("adadelta: negative chunk or segment count");
    if (n_chunks == 0) return M3D_OK;
    if (!params || !grads || !accum || !delta_accum || !seg_of_chunk || !l2_coef ||
        (clipnorm > 0.f && !norms))
        return einval("adadelta: null pointer");
    int rc = clip_norms(params, grads, n_chunks, seg_of_chunk, l2_coef, n_segments, clipnorm, norms, s);
    if (rc) return rc;
    hipLaunchKernelGGL(adaptive_update_kernel<2>, dim3((unsigned)n_chunks), dim3(256), 0, st(s),
                       params, grads, accum, delta_accum, (float*)nullptr, seg_of_chunk, l2_coef, norms,
                       lr, rho, 1.0f - rho, 0.f, 0.f, epsilon, clipnorm);
    return check_launch("adaptive_update_kernel<adadelta>");
}
