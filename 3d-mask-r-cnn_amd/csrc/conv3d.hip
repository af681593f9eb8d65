// Conv3D (Keras Conv3D, channels-last) as fp32-MFMA implicit GEMMs on gfx950.
//
// Replaces the TF builtin Conv3D/BN/ReLU/Add op chain of the reference graph
// (core/models.py:157-273 backbone, 3190-3214 FPN, 512-557 RPN head).
//
// GEMM views (m = output voxel (b,oy,ox,oz), n = output channel,
//             k = (tap, input channel), taps (ky,kx,kz) row-major):
//   fwd       Y[m][n]      = sum_k im2col(X)[m][k] * W[k][n]
//   bwd-data  dX[m'][c]    = sum_(t,n) dZ[m'(t)][n] * W[flip t][c][n]
//   bwd-wgt   dW[k][n]    += sum_m im2col(X)[m][k] * dZ[m][n]
// W is the Keras kernel [kh,kw,kd,Cin,Cout] = [K][Cout] row-major, used
// as-is by all three (no transposed weight copies).
//
// Arithmetic: v_mfma_f32_32x32x2_f32 (exact f32 fma chain, 155 TF/s chip
// peak = the f32 vector rate).  Block = 256 threads = 4 waves; each wave owns
// TMxTN 32x32 accumulator tiles.  K is staged 32 deep through double-buffered
// LDS with register prefetch (global loads of tile t+1 in flight while the
// MFMAs of tile t run; one barrier per k-tile).  Within a 32-deep k-tile the
// MFMA k-step s of lane-half h consumes k = 16h + s for both operands.
// LDS tiles keep the global layout; operand reads are ds_read_b32 with the
// MFMA lane index on the contiguous (or odd-strided) axis: conflict-free.
//
// Fused epilogue: + bias, frozen-BN affine (z*scale+shift), optional z store,
// + residual (same shape or (2,2,1)-upsampled FPN source), ReLU, strided /
// channel-split stores (RPN class|bbox heads write their concatenated outputs
// directly).
#include "common.h"

namespace m3d {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct ConvP {
    const float* a;   // A source (x or dz), channels-last [B,H,W,D,C]
    int B, H, W, D, C;
    int OH, OW, OD;   // M grid
    int kh, kw, kd;
    int sy, sx, sz;
    int py, px, pz;
    int64_t M;
    int K;            // taps * C
    const float* w;
    int N;
    int flip;         // bwd-data: use tap (taps-1-t)
};

struct Epi {
    const float* bias;
    const float* scale;
    const float* shift;
    const float* res;
    int res_mode;
    int relu;
    float* z;
    float* y;
    int64_t ldy;
    float* y2;
    int64_t ldy2;
    int split;
    int YH, YW, YD;
    int ysy, ysx, ysz;
    int accumulate;
    int simple;       // y row == m (same grid, unit store stride)
};

__device__ __forceinline__ float f4get(const float4& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// m < 2^31 is guaranteed by the host checks: 32-bit unsigned division only.
__device__ __forceinline__ void decompose(int64_t m64, int OH, int OW, int OD, int& b, int& oy,
                                          int& ox, int& oz) {
    uint32_t m = (uint32_t)m64;
    uint32_t t = m / (uint32_t)OD;
    oz = (int)(m - t * (uint32_t)OD);
    uint32_t t2 = t / (uint32_t)OW;
    ox = (int)(t - t2 * (uint32_t)OW);
    uint32_t t3 = t2 / (uint32_t)OH;
    oy = (int)(t2 - t3 * (uint32_t)OH);
    b = (int)t3;
}

__device__ __forceinline__ void epi_store(const ConvP& p, const Epi& e, int64_t m, int n, float v) {
    int b = 0, oy = 0, ox = 0, oz = 0;
    if (!e.simple || e.res_mode == 2) decompose(m, p.OH, p.OW, p.OD, b, oy, ox, oz);
    if (e.bias) v += e.bias[n];
    if (e.z) e.z[m * p.N + n] = v;
    if (e.scale) v = v * e.scale[n] + e.shift[n];
    const int64_t yrow = e.simple ? m
                                  : (((int64_t)b * e.YH + (int64_t)oy * e.ysy) * e.YW +
                                     (int64_t)ox * e.ysx) * e.YD + (int64_t)oz * e.ysz;
    if (e.res_mode == 1) {
        v += e.res[yrow * e.ldy + n];
    } else if (e.res_mode == 2) {
        const int64_t rrow = (((int64_t)b * (p.OH >> 1) + (oy >> 1)) * (p.OW >> 1) + (ox >> 1)) * p.OD + oz;
        v += e.res[rrow * p.N + n];
    }
    if (e.relu) v = v > 0.0f ? v : 0.0f;
    if (e.split > 0 && n >= e.split) {
        e.y2[yrow * e.ldy2 + (n - e.split)] = v;
    } else {
        float* dst = e.y + yrow * e.ldy + n;
        if (e.accumulate) v += *dst;
        *dst = v;
    }
}

// -------------------------------------------------------------------------
// fwd / bwd-data implicit GEMM
// -------------------------------------------------------------------------
template <int BM, int BN, int WM, int WN, bool BT, bool AVEC>
__global__ __launch_bounds__(256, 2) void conv_gemm_kernel(ConvP p, Epi e) {
    constexpr int BK = 32;
    constexpr int TM = BM / (WM * 32), TN = BN / (WN * 32);
    static_assert(WM * WN == 4, "4 waves");
    static_assert(TM >= 1 && TN >= 1, "tile");
    // [rows][k] tiles: row stride 36 floats keeps float4 alignment and makes the
    // per-lane 16-float fragment reads (4 x ds_read_b128, rows = lanes) bank-
    // conflict-free (36*i mod 64 dwords spreads 16 rows over all 64 banks).
    constexpr int LDA = BK + 4;
    constexpr int LDB = BT ? (BK + 4) : BN;
    constexpr int A_SZ = BM * LDA;
    constexpr int B_SZ = BT ? BN * LDB : BK * LDB;
    constexpr int AQ = AVEC ? BM / 32 : BM / 8;      // A elements (float4 or float) per thread
    constexpr int BQ = BN / 32;                      // B float4 per thread
    __shared__ __attribute__((aligned(16))) float smem[2 * (A_SZ + B_SZ)];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    // XCD-aware tile order (speed only): the dispatcher deals consecutive
    // workgroups round-robin to the 8 XCDs; remap so each XCD owns a contiguous
    // run of tiles, N-tiles of one M-tile adjacent, so the im2col rows (and
    // their 3x3x3 halo) are re-read from that XCD's L2, not from HBM.
    int64_t m0;
    int n0;
    {
        const int64_t nbx = gridDim.x, nby = gridDim.y, total = nbx * nby;
        const int64_t L = (int64_t)blockIdx.x + nbx * blockIdx.y;
        const int64_t xcd = L % 8, q8 = total / 8, r8 = total % 8;
        const int64_t T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
        m0 = (T / nby) * BM;
        n0 = (int)(T % nby) * BN;
    }
    const int taps_kd = p.kd, taps_kwkd = p.kw * p.kd;
    const int ntaps = p.kh * taps_kwkd;

    // per-thread A rows (vector path): base coordinates
    int a_b[AVEC ? AQ : 1], a_y[AVEC ? AQ : 1], a_x[AVEC ? AQ : 1], a_z[AVEC ? AQ : 1];
    bool a_ok[AVEC ? AQ : 1];
    const int a_col4 = tid & 7;
    if (AVEC) {
#pragma unroll
        for (int q = 0; q < AQ; ++q) {
            const int64_t m = m0 + (tid >> 3) + 32 * q;
            a_ok[q] = m < p.M;
            int b, oy, ox, oz;
            decompose(a_ok[q] ? m : 0, p.OH, p.OW, p.OD, b, oy, ox, oz);
            a_b[q] = b;
            a_y[q] = oy * p.sy - p.py;
            a_x[q] = ox * p.sx - p.px;
            a_z[q] = oz * p.sz - p.pz;
        }
    }

    float4 ra[AVEC ? AQ : 1];
    float rs[AVEC ? 1 : AQ];
    float4 rb[BQ];

    auto load_tile = [&](int kt) {
        const int k0 = kt * BK;
        if (AVEC) {
            const int tap = k0 / p.C;
            const int c0 = k0 - tap * p.C;
            const int ky = tap / taps_kwkd, kx = (tap / taps_kd) % p.kw, kz = tap % taps_kd;
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                const int iy = a_y[q] + ky, ix = a_x[q] + kx, iz = a_z[q] + kz;
                const bool ok = a_ok[q] && iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && iz >= 0 &&
                                iz < p.D;
                if (ok) {
                    const int64_t off = ((((int64_t)a_b[q] * p.H + iy) * p.W + ix) * p.D + iz) * p.C +
                                        c0 + a_col4 * 4;
                    ra[q] = *reinterpret_cast<const float4*>(p.a + off);
                } else {
                    ra[q] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        } else {
            const int col = tid & 31;
            const int k = k0 + col;
            int tap = 0, c = 0, ky = 0, kx = 0, kz = 0;
            if (k < p.K) {
                tap = k / p.C;
                c = k - tap * p.C;
                ky = tap / taps_kwkd; kx = (tap / taps_kd) % p.kw; kz = tap % taps_kd;
            }
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                const int64_t m = m0 + (tid >> 5) + 8 * q;
                float v = 0.f;
                if (k < p.K && m < p.M) {
                    int b, oy, ox, oz;
                    decompose(m, p.OH, p.OW, p.OD, b, oy, ox, oz);
                    const int iy = oy * p.sy - p.py + ky, ix = ox * p.sx - p.px + kx,
                              iz = oz * p.sz - p.pz + kz;
                    if (iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && iz >= 0 && iz < p.D)
                        v = p.a[((((int64_t)b * p.H + iy) * p.W + ix) * p.D + iz) * p.C + c];
                }
                rs[q] = v;
            }
        }
        if (!BT) {
            constexpr int C4 = BN / 4;
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
                const int idx = tid + 256 * q;
                const int kr = idx / C4, c4 = idx % C4;
                const int k = k0 + kr, n = n0 + c4 * 4;
                rb[q] = (k < p.K && n < p.N)
                            ? *reinterpret_cast<const float4*>(p.w + (int64_t)k * p.N + n)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        } else {
            // B(k=(t,c'), n) = w[(t'*N + n)*C + c'], tile rows n, 32 contiguous c'
            const int tap = k0 / p.C;
            const int c0 = k0 - tap * p.C;
            const int wt = p.flip ? (ntaps - 1 - tap) : tap;
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
                const int n = n0 + (tid >> 3) + 32 * q;
                rb[q] = n < p.N ? *reinterpret_cast<const float4*>(
                                      p.w + ((int64_t)wt * p.N + n) * p.C + c0 + a_col4 * 4)
                                : make_float4(0.f, 0.f, 0.f, 0.f);
            }
        }
    };

    auto store_tile = [&](int buf) {
        float* As = smem + buf * (A_SZ + B_SZ);
        float* Bs = As + A_SZ;
        if (AVEC) {
#pragma unroll
            for (int q = 0; q < AQ; ++q)
                *reinterpret_cast<float4*>(As + ((tid >> 3) + 32 * q) * LDA + a_col4 * 4) = ra[q];
        } else {
#pragma unroll
            for (int q = 0; q < AQ; ++q) As[((tid >> 5) + 8 * q) * LDA + (tid & 31)] = rs[q];
        }
        if (!BT) {
            constexpr int C4 = BN / 4;
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
                const int idx = tid + 256 * q;
                *reinterpret_cast<float4*>(Bs + (idx / C4) * LDB + (idx % C4) * 4) = rb[q];
            }
        } else {
#pragma unroll
            for (int q = 0; q < BQ; ++q)
                *reinterpret_cast<float4*>(Bs + ((tid >> 3) + 32 * q) * LDB + a_col4 * 4) = rb[q];
        }
    };

    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int nk = (p.K + BK - 1) / BK;
    const int h = lane >> 5, l32 = lane & 31;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < nk) load_tile(kt + 1);
        const float* As = smem + buf * (A_SZ + B_SZ);
        const float* Bs = As + A_SZ;
        // fragments: lane (l32, h) owns row l32 of each 32-row tile and the 16
        // k values 16h..16h+15 of this k-tile (MFMA step s consumes k = 16h+s)
        float4 af[TM][4];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                af[i][q] = *reinterpret_cast<const float4*>(As + (wm * TM * 32 + i * 32 + l32) * LDA +
                                                            h * 16 + 4 * q);
        float4 bf[BT ? TN : 1][4];
        if (BT) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    bf[j][q] = *reinterpret_cast<const float4*>(Bs + (wn * TN * 32 + j * 32 + l32) * LDB +
                                                                h * 16 + 4 * q);
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int kk = h * 16 + s;
            float b[TN];
#pragma unroll
            for (int j = 0; j < TN; ++j)
                b[j] = BT ? f4get(bf[BT ? j : 0][s >> 2], s & 3)
                          : Bs[kk * LDB + wn * TN * 32 + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(f4get(af[i][s >> 2], s & 3), b[j],
                                                                      acc[i][j], 0, 0, 0);
        }
        if (kt + 1 < nk) store_tile(buf ^ 1);
        __syncthreads();
    }

    // epilogue: D[row][col], col = lane&31 (n), row = (r&3) + 8(r>>2) + 4h (m)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * TN * 32 + j * 32 + l32;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int64_t m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (m < p.M) epi_store(p, e, m, n, acc[i][j][r]);
            }
        }
}

// -------------------------------------------------------------------------
// bwd-weight: dW[k][n] += sum_m im2col(X)[m][k] * dZ[m][n]
// grid (K/BI, N/BJ, splits); each block reduces its m-range, fp32 atomics out.
// -------------------------------------------------------------------------
template <int BI, int BJ, int WI, int WJ, bool AVEC>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(ConvP p, const float* __restrict__ dz,
                                                            float* __restrict__ dw,
                                                            int64_t m_per_split) {
    constexpr int BKM = 32;
    constexpr int TI = BI / (WI * 32), TJ = BJ / (WJ * 32);
    static_assert(WI * WJ == 4, "4 waves");
    constexpr int X_SZ = BKM * BI, G_SZ = BKM * BJ;
    constexpr int XQ = AVEC ? BI / 32 : BI / 8;
    constexpr int GQ = BJ / 32;
    __shared__ __attribute__((aligned(16))) float smem[2 * (X_SZ + G_SZ)];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave / WJ, wj = wave % WJ;
    const int k0 = blockIdx.x * BI;
    const int n0 = blockIdx.y * BJ;
    const int64_t ms = (int64_t)blockIdx.z * m_per_split;
    int64_t me = ms + m_per_split;
    if (me > p.M) me = p.M;
    if (ms >= me) return;
    const int taps_kd = p.kd, taps_kwkd = p.kw * p.kd;

    // fixed column for this thread
    constexpr int XC = AVEC ? BI / 4 : BI;                // columns (float4 or scalar)
    const int xcol = tid % XC;
    const int xrow0 = tid / XC;
    constexpr int XRSTEP = 256 / XC;
    const int kcol = k0 + (AVEC ? xcol * 4 : xcol);
    const bool kok = kcol < p.K;
    int ky = 0, kx = 0, kz = 0, cc = 0;
    if (kok) {
        const int tap = kcol / p.C;
        cc = kcol - tap * p.C;
        ky = tap / taps_kwkd; kx = (tap / taps_kd) % p.kw; kz = tap % taps_kd;
    }
    constexpr int GC = BJ / 4;
    const int gcol = tid % GC, grow0 = tid / GC;
    constexpr int GRSTEP = 256 / GC;

    float4 rx4[AVEC ? XQ : 1];
    float rx1[AVEC ? 1 : XQ];
    float4 rg[GQ];

    // output coordinates of row (mb + xrow0), advanced incrementally (no
    // per-row integer division in the m loop)
    int cb_ = 0, cy_ = 0, cx_ = 0, cz_ = 0;
    decompose(ms + xrow0 < me ? ms + xrow0 : ms, p.OH, p.OW, p.OD, cb_, cy_, cx_, cz_);
    auto advance = [&](int& b, int& y, int& x, int& z, int delta) {
        z += delta;
        while (z >= p.OD) {
            z -= p.OD;
            if (++x == p.OW) {
                x = 0;
                if (++y == p.OH) { y = 0; ++b; }
            }
        }
    };
    auto load_tile = [&](int64_t mb) {
        int rb = cb_, ry = cy_, rx = cx_, rz = cz_;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int64_t m = mb + xrow0 + XRSTEP * q;
            if (q > 0) advance(rb, ry, rx, rz, XRSTEP);
            bool ok = kok && m < me;
            int64_t off = 0;
            if (ok) {
                const int b = rb, oy = ry, ox = rx, oz = rz;
                const int iy = oy * p.sy - p.py + ky, ix = ox * p.sx - p.px + kx,
                          iz = oz * p.sz - p.pz + kz;
                ok = iy >= 0 && iy < p.H && ix >= 0 && ix < p.W && iz >= 0 && iz < p.D;
                off = ((((int64_t)b * p.H + iy) * p.W + ix) * p.D + iz) * p.C + cc;
            }
            if (AVEC) rx4[q] = ok ? *reinterpret_cast<const float4*>(p.a + off) : make_float4(0.f, 0.f, 0.f, 0.f);
            else rx1[q] = ok ? p.a[off] : 0.0f;
        }
        advance(cb_, cy_, cx_, cz_, BKM);
#pragma unroll
        for (int q = 0; q < GQ; ++q) {
            const int64_t m = mb + grow0 + GRSTEP * q;
            const int n = n0 + gcol * 4;
            rg[q] = (m < me && n < p.N) ? *reinterpret_cast<const float4*>(dz + m * p.N + n)
                                        : make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto store_tile = [&](int buf) {
        float* Xs = smem + buf * (X_SZ + G_SZ);
        float* Gs = Xs + X_SZ;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int r = xrow0 + XRSTEP * q;
            if (AVEC) *reinterpret_cast<float4*>(Xs + r * BI + xcol * 4) = rx4[q];
            else Xs[r * BI + xcol] = rx1[q];
        }
#pragma unroll
        for (int q = 0; q < GQ; ++q)
            *reinterpret_cast<float4*>(Gs + (grow0 + GRSTEP * q) * BJ + gcol * 4) = rg[q];
    };

    floatx16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    const int h = lane >> 5, l32 = lane & 31;
    const int nchunks = (int)((me - ms + BKM - 1) / BKM);
    load_tile(ms);
    store_tile(0);
    __syncthreads();
    for (int t = 0; t < nchunks; ++t) {
        const int buf = t & 1;
        if (t + 1 < nchunks) load_tile(ms + (int64_t)(t + 1) * BKM);
        const float* Xs = smem + buf * (X_SZ + G_SZ);
        const float* Gs = Xs + X_SZ;
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int kk = h * 16 + s;
            float a[TI], b[TJ];
#pragma unroll
            for (int i = 0; i < TI; ++i) a[i] = Xs[kk * BI + wi * TI * 32 + i * 32 + l32];
#pragma unroll
            for (int j = 0; j < TJ; ++j) b[j] = Gs[kk * BJ + wj * TJ * 32 + j * 32 + l32];
#pragma unroll
            for (int i = 0; i < TI; ++i)
#pragma unroll
                for (int j = 0; j < TJ; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[i], b[j], acc[i][j], 0, 0, 0);
        }
        if (t + 1 < nchunks) store_tile(buf ^ 1);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int n = n0 + wj * TJ * 32 + j * 32 + l32;
            if (n >= p.N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = k0 + wi * TI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (k < p.K) unsafeAtomicAdd(dw + (int64_t)k * p.N + n, acc[i][j][r]);
            }
        }
}

// ------------------------------------------------------------------ dispatch
template <int BM, int BN, int WM, int WN, bool BT, bool AVEC>
static void launch_gemm(const ConvP& p, const Epi& e, hipStream_t s) {
    dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.N + BN - 1) / BN));
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC>), grid, dim3(256), 0, s, p, e);
}

template <bool BT, bool AVEC>
static void dispatch_gemm(const ConvP& p, const Epi& e, hipStream_t s) {
    if (p.N <= 32) {
        launch_gemm<128, 32, 4, 1, BT, AVEC>(p, e, s);
    } else if (p.N <= 64) {
        launch_gemm<128, 64, 4, 1, BT, AVEC>(p, e, s);
    } else {
        const int64_t blocks128 = ((p.M + 127) / 128) * ((p.N + 127) / 128);
        if (blocks128 < 512) launch_gemm<64, 128, 2, 2, BT, AVEC>(p, e, s);
        else launch_gemm<128, 128, 2, 2, BT, AVEC>(p, e, s);
    }
}

template <int BI, int BJ, int WI, int WJ, bool AVEC>
static void launch_wgrad(const ConvP& p, const float* dz, float* dw, hipStream_t s) {
    const int64_t tiles = (int64_t)((p.K + BI - 1) / BI) * ((p.N + BJ - 1) / BJ);
    int64_t splits = (1024 + tiles - 1) / tiles;                   // aim >= 1024 blocks
    const int64_t max_splits = (p.M + 1023) / 1024;                 // >= 1024 m per block
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    int64_t mper = (p.M + splits - 1) / splits;
    mper = (mper + 31) / 32 * 32;
    splits = (p.M + mper - 1) / mper;
    dim3 grid((unsigned)((p.K + BI - 1) / BI), (unsigned)((p.N + BJ - 1) / BJ), (unsigned)splits);
    hipLaunchKernelGGL((conv_wgrad_kernel<BI, BJ, WI, WJ, AVEC>), grid, dim3(256), 0, s, p, dz, dw,
                       mper);
}

}  // namespace m3d

using namespace m3d;

static int conv_check(int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin, int32_t kh,
                      int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                      int32_t sy, int32_t sx, int32_t sz) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0 || Cin <= 0 || Cout <= 0)
        return einval("conv3d: tensor dimensions must be positive");
    if (kh <= 0 || kw <= 0 || kd <= 0 || sy <= 0 || sx <= 0 || sz <= 0)
        return einval("conv3d: kernel size and strides must be positive");
    if (OH <= 0 || OW <= 0 || OD <= 0) return einval("conv3d: output dimensions must be positive");
    if (Cout % 4) return einval("conv3d: Cout must be a multiple of 4");
    if ((int64_t)kh * kw * kd * Cin > 0x7FFFFFFF) return einval("conv3d: K too large");
    if (B * H * W * D > 0x7FFFFFFF || B * OH * OW * OD > 0x7FFFFFFF)
        return einval("conv3d: more than 2^31 voxels per tensor");
    return M3D_OK;
}

extern "C" int m3d_conv3d_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                              int64_t Cin, const float* w, int32_t kh, int32_t kw, int32_t kd,
                              int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                              int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                              const float* bias, const float* bn_scale, const float* bn_shift,
                              const float* residual, int32_t res_mode, int32_t relu, float* z_out,
                              float* y, int64_t ldy, float* y2, int64_t ldy2, int64_t split_n,
                              m3d_stream_t s) {
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("conv3d: bn_scale and bn_shift must be given together");
    if (res_mode != 0 && residual == nullptr) return einval("conv3d: residual missing");
    if (res_mode == 2 && ((OH & 1) || (OW & 1))) return einval("conv3d: upsampled residual needs even OH/OW");
    if (split_n > 0 && y2 == nullptr) return einval("conv3d: split output needs y2");
    ConvP p{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), w, (int)Cout, 0};
    Epi e{bias, bn_scale, bn_shift, residual, res_mode, relu, z_out, y, ldy > 0 ? ldy : Cout,
          y2, ldy2, (int)split_n, (int)OH, (int)OW, (int)OD, 1, 1, 1, 0, 1};
    if (Cin % 32 == 0) dispatch_gemm<false, true>(p, e, st(s));
    else dispatch_gemm<false, false>(p, e, st(s));
    return check_launch("conv_gemm_kernel(fwd)");
}

extern "C" int m3d_conv3d_bwd_data(const float* dz, const float* w, int64_t B, int64_t H,
                                   int64_t W, int64_t D, int64_t Cin, int32_t kh, int32_t kw,
                                   int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                   int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px,
                                   int32_t pz, float* dx, int32_t accumulate, m3d_stream_t s) {
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (Cout % 32) return einval("conv3d bwd-data: Cout must be a multiple of 32");
    if (Cin % 4) return einval("conv3d bwd-data: Cin must be a multiple of 4");
    const bool unit = kh == 1 && kw == 1 && kd == 1;
    if (!unit && (sy != 1 || sx != 1 || sz != 1))
        return einval("conv3d bwd-data: strided convs supported for 1x1x1 kernels only");
    ConvP p;
    Epi e{};
    e.y = dx;
    e.ldy = Cin;
    e.accumulate = accumulate;
    p.w = w;
    p.N = (int)Cin;
    p.a = dz;
    p.B = (int)B;
    p.C = (int)Cout;
    p.kh = kh; p.kw = kw; p.kd = kd;
    p.K = (int)(kh * kw * kd * Cout);
    p.flip = 1;
    if (unit) {
        // M grid = dz grid; store strided into dx
        p.H = (int)OH; p.W = (int)OW; p.D = (int)OD;
        p.OH = (int)OH; p.OW = (int)OW; p.OD = (int)OD;
        p.sy = p.sx = p.sz = 1;
        p.py = p.px = p.pz = 0;
        e.YH = (int)H; e.YW = (int)W; e.YD = (int)D;
        e.ysy = sy; e.ysx = sx; e.ysz = sz;
        e.simple = (sy == 1 && sx == 1 && sz == 1 && H == OH && W == OW && D == OD);
        if (py || px || pz) return einval("conv3d bwd-data: 1x1x1 conv with padding unsupported");
    } else {
        // M grid = dx grid; A = dz with pad' = k-1-p, flipped taps
        p.H = (int)OH; p.W = (int)OW; p.D = (int)OD;
        p.OH = (int)H; p.OW = (int)W; p.OD = (int)D;
        p.sy = p.sx = p.sz = 1;
        p.py = kh - 1 - py; p.px = kw - 1 - px; p.pz = kd - 1 - pz;
        e.YH = (int)H; e.YW = (int)W; e.YD = (int)D;
        e.ysy = e.ysx = e.ysz = 1;
        e.simple = 1;
    }
    p.M = (int64_t)p.B * p.OH * p.OW * p.OD;
    dispatch_gemm<true, true>(p, e, st(s));
    return check_launch("conv_gemm_kernel(bwd-data)");
}

extern "C" int m3d_conv3d_bwd_weight(const float* x, const float* dz, int64_t B, int64_t H,
                                     int64_t W, int64_t D, int64_t Cin, int32_t kh, int32_t kw,
                                     int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                     int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px,
                                     int32_t pz, float* dw, m3d_stream_t s) {
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    ConvP p{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), nullptr,
            (int)Cout, 0};
    const bool vec = (Cin % 4) == 0;
    if (Cout <= 64) {
        if (vec) launch_wgrad<128, 64, 2, 2, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 64, 2, 2, false>(p, dz, dw, st(s));
    } else {
        if (vec) launch_wgrad<128, 128, 2, 2, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 128, 2, 2, false>(p, dz, dw, st(s));
    }
    return check_launch("conv_wgrad_kernel");
}
