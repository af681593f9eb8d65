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
#include <stdlib.h>

namespace m3d {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef float floatx4 __attribute__((ext_vector_type(4)));

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
    // batched GEMMs (Winograd points): blockIdx.z selects the batch; A, W and Y
    // advance by these element strides (0 for ordinary convs)
    int64_t bsa, bsw, bsy;
    int dly = 1, dlx = 1, dlz = 1;   // dilation (fwd only; mrcnn_mask_conv3b)
    int nbatch = 1;                  // batches (PERSIST: looped inside the grid)
    // depth-slab halo planes beside the slab (the stem and the direct weight
    // gradient, m3d_conv3d_*_halo): the conv runs on the virtual z grid
    // [lower halo (hnlo planes) | slab (hdl) | upper halo], D = its depth; x (a)
    // holds the slab [B,H,W,hdl,C], halo [B,H,W,2*hr,C] the neighbours' planes
    // ([0,hr) from below, [hr,2hr) from above)
    const float* halo = nullptr;
    int hnlo = 0, hdl = 0, hr = 0;
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
    // depth-slab halo (wino_output_kernel<.., HALO>): output z over the
    // halo-extended grid; planes [hlo, hlo + dl) go to y (depth dl), the halo
    // planes to yh [B][H][W][2][N] (plane 0 below, 1 above)
    float* yh;
    int hlo, dl;
    int deconv = 0;   // > 0: 2x2x2 stride-2 transposed conv, n = tap * deconv + o
    // fused BN-ReLU backward of the unit that produced this data gradient's
    // input (m3d_conv3d_bwd_data_bn): the stored value t (after accumulate) is
    // the unit's output gradient; written instead are dz = act'(t) * scale
    // (into y), dpre = act'(t) (into fdres, if set), and per-tile channel sums
    // of dpre, dpre * xhat, dz (rows of fpart, [3][rows][N]) -- the maths of
    // bn_act_bwd_kernel
    int fbn = 0, frelu = 0;
    const float* fy = nullptr;
    const float* fz = nullptr;
    const float* fscale = nullptr;
    const float* fmean = nullptr;
    const float* frstd = nullptr;
    float* fdres = nullptr;
    float* fpart = nullptr;
    int64_t fprows = 0;           // partial rows (stride of the three sum planes)
};



// activation codes (Epi::relu): 0 none, 1 ReLU, 2 sigmoid (mrcnn_mask)
__device__ __forceinline__ float act(int code, float v) {
    if (code == 1) return v > 0.0f ? v : 0.0f;
    if (code == 2) return 1.0f / (1.0f + expf(-v));
    return v;
}

// Raw buffer loads: 32-bit byte offsets, and an out-of-range offset returns 0
// -- used for the implicit zero padding of im2col so the loaders are
// branch-free (no exec-mask divergence around every load).
#define M3D_OOB 0xFFFFFFF0u
// Every caller's base and size are wave-uniform (kernel arguments, blockIdx-
// derived, or a readfirstlane'd wave role); the readfirstlanes make that
// provable to the compiler, which otherwise wraps each buffer op whose
// descriptor it holds in VGPRs (64-bit divisions, per-wave selects) in a
// readfirstlane waterfall loop (cdna_hip_programming.md T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint64_t bytes) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
    const uint32_t nb = __builtin_amdgcn_readfirstlane((uint32_t)(bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : bytes));
    void* const pu = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc(pu, (short)0, (int)nb, 0x00020000);
}
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
    return *reinterpret_cast<float4*>(&v);
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bstore4(__amdgpu_buffer_rsrc_t r, uint32_t off, float a, float b, float c, float d) {
    u32x4 v = {__float_as_uint(a), __float_as_uint(b), __float_as_uint(c), __float_as_uint(d)};
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
}

__device__ __forceinline__ float f4get(const float4& v, int i) {
    return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// ---- exact 3-way bf16 split of fp32 operands (X3 GEMM mode) ---------------
// x = hi + mid + lo with hi = bf16(x), mid = bf16(x - hi), lo = bf16(x - hi - mid):
// both subtractions are exact (Sterbenz), and 3 x 8 significant bits cover the
// 24-bit f32 significand, so the split is exact for normal x.  A product a*b
// is sum_{p+q<=2} a_p b_q (6 bf16 MFMAs, each product exact in the f32
// accumulator); the dropped terms are below 2^-24 |a b| -- the rounding error
// of the f32 FMA itself.  v_mfma_f32_32x32x16_bf16 retires 16x the FLOPs per
// cycle of v_mfma_f32_32x32x2_f32, so 6 of them are 2.7x the f32 MFMA rate.
typedef short bf16x8 __attribute__((ext_vector_type(8)));
__device__ __forceinline__ uint32_t bf16_bits(float x) {
    return (uint32_t)__builtin_bit_cast(unsigned short, (__bf16)x);
}
__device__ __forceinline__ void split3(float x, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = bf16_bits(x);
    const float r = x - __uint_as_float(h << 16);
    m = bf16_bits(r);
    l = bf16_bits(r - __uint_as_float(m << 16));
}
// float4 (4 consecutive k) -> three 4 x bf16 packets (element j at bits 16j).
// Two elements per conversion (v_cvt_pk_bf16_f32 with two sources) and per
// subtraction (v_pk_add_f32): 20 VALU per float4 instead of 41 for four
// scalar split3 -- the same bits (both subtractions exact).
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(f32x2_t v) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ f32x2_t unpk_bf16(uint32_t p) {
    return f32x2_t{__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
}
__device__ __forceinline__ void split3x2(f32x2_t x, uint32_t& h, uint32_t& m, uint32_t& l) {
    h = pk_bf16(x);
    const f32x2_t r = x - unpk_bf16(h);
    m = pk_bf16(r);
    l = pk_bf16(r - unpk_bf16(m));
}
__device__ __forceinline__ void split3x4(const float4& v, uint2* o) {
    uint32_t h0, m0, l0, h1, m1, l1;
    split3x2(f32x2_t{v.x, v.y}, h0, m0, l0);
    split3x2(f32x2_t{v.z, v.w}, h1, m1, l1);
    o[0] = make_uint2(h0, h1);
    o[1] = make_uint2(m0, m1);
    o[2] = make_uint2(l0, l1);
}
// One 16-deep k step of an fp32 product sum on the split: acc += sum_k a_k b_k
// as the six bf16 MFMAs, small terms first: (lo,hi) (mid,mid) (hi,lo) (mid,hi)
// (hi,mid) (hi,hi), one accumulator chain.  (Round 5 measured the alternative
// -- each k step's six into a fresh accumulator, one VALU add into acc -- on
// the MI355X: the 128^3 gradient median rose 2.28e-6 -> 3.29e-6 and the step
// slowed; the MFMA's accumulation into C beats an fp32 rounding per step.)
__device__ __forceinline__ void x3_mac(floatx16& acc, const bf16x8& ah, const bf16x8& am, const bf16x8& al,
                                       const bf16x8& bh, const bf16x8& bm, const bf16x8& bl) {
    floatx16 c = acc;
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}
// x3_mac of two accumulator tiles sharing the A fragment, their two six-MFMA
// chains interleaved: each accumulator sees its products in x3_mac's order
// (bit-identical results), but consecutive MFMAs are independent, so an MFMA
// does not wait for its predecessor's result (weight-gradient GEMM -3 %).
__device__ __forceinline__ void x3_mac_pair(floatx16& acc0, floatx16& acc1, const bf16x8& ah, const bf16x8& am,
                                            const bf16x8& al, const bf16x8& b0h, const bf16x8& b0m,
                                            const bf16x8& b0l, const bf16x8& b1h, const bf16x8& b1m,
                                            const bf16x8& b1l) {
    floatx16 c0 = acc0, c1 = acc1;
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, b1h, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b0m, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b1m, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b0l, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b1l, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b0h, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, b1h, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b0m, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b1m, c1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b0h, c0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, b1h, c1, 0, 0, 0);
}
// x3_mac over a wave's TM x TN accumulator tiles with fragments af[i][plane],
// bf[j][plane], tile pairs interleaved (x3_mac_pair)
template <int TM, int TN>
__device__ __forceinline__ void x3_mac_tiles(floatx16 (&acc)[TM][TN], const bf16x8 (&af)[TM][3],
                                             const bf16x8 (&bf)[TN][3]) {
    if constexpr (TN % 2 == 0) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; j += 2)
                x3_mac_pair(acc[i][j], acc[i][j + 1], af[i][0], af[i][1], af[i][2], bf[j][0], bf[j][1], bf[j][2],
                            bf[j + 1][0], bf[j + 1][1], bf[j + 1][2]);
    } else {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
                x3_mac(acc[i][j], af[i][0], af[i][1], af[i][2], bf[j][0], bf[j][1], bf[j][2]);
    }
}
// byte offset of (row, k) in an X3 LDS plane: 32 k x bf16 = 64-B rows, 16-B
// chunks XOR-swizzled by (row >> 2) & 3 so a 16-lane ds_read_b128 phase over
// 16 consecutive rows of one chunk hits 16 distinct 4-bank groups.
__device__ __forceinline__ int x3_off(int row, int k) {
    return row * 64 + ((((k >> 3) ^ (row >> 2)) & 3) << 4) + (k & 7) * 2;
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

// row of the output tensor that GEMM row m / column n lands in (strided,
// (2,2,1)-upsampled or 2x2x2-deconvolved stores); n is reduced to the channel.
__device__ __forceinline__ int64_t out_row(const ConvP& p, const Epi& e, int b, int oy, int ox, int oz,
                                           int& n) {
    if (e.deconv) {
        const int t = n / e.deconv;
        n -= t * e.deconv;
        return (((int64_t)b * e.YH + 2 * oy + (t >> 2)) * e.YW + 2 * ox + ((t >> 1) & 1)) * e.YD + 2 * oz +
               (t & 1);
    }
    return (((int64_t)b * e.YH + (int64_t)oy * e.ysy) * e.YW + (int64_t)ox * e.ysx) * e.YD +
           (int64_t)oz * e.ysz;
}

__device__ __forceinline__ void epi_store(const ConvP& p, const Epi& e, int64_t m, int n, float v) {
    int b = 0, oy = 0, ox = 0, oz = 0;
    if (!e.simple || e.res_mode == 2) decompose(m, p.OH, p.OW, p.OD, b, oy, ox, oz);
    const int64_t zrow = m * p.N + n;
    const int64_t yrow = e.simple ? m : out_row(p, e, b, oy, ox, oz, n);
    if (e.bias) v += e.bias[n];
    if (e.z) e.z[zrow] = v;
    if (e.scale) v = v * e.scale[n] + e.shift[n];
    if (e.res_mode == 1) {
        v += e.res[yrow * e.ldy + n];
    } else if (e.res_mode == 2) {
        const int64_t rrow = (((int64_t)b * (p.OH >> 1) + (oy >> 1)) * (p.OW >> 1) + (ox >> 1)) * p.OD + oz;
        v += e.res[rrow * p.N + n];
    }
    v = act(e.relu, v);
    if (e.res_mode == 3) v += e.res[yrow * e.ldy + n];      // Add() after the activation
    if (e.split > 0 && n >= e.split) {
        e.y2[yrow * e.ldy2 + (n - e.split)] = v;
    } else {
        float* dst = e.y + yrow * e.ldy + n;
        if (e.accumulate) v += *dst;
        *dst = v;
    }
}

// Four consecutive output channels n..n+3 of row m (same op order as epi_store,
// element-wise): 16-byte loads / stores when the row strides allow it.
__device__ __forceinline__ float4 ld4(const float* q) { return *reinterpret_cast<const float4*>(q); }
__device__ __forceinline__ void st4(float* q, const float4& v) { *reinterpret_cast<float4*>(q) = v; }

// The fused BN-act backward of four channels n..n+3 of row m (simple rows):
// bn_act_bwd_kernel's per-element maths, sums accumulated in s[3][4].  The
// caller loads y4 / z4 (and the channel's scale / mean / rstd in bn[3]) ahead
// of the batch's stores: a load issued after a store to a possibly aliasing
// address waits for it.
__device__ __forceinline__ void epi_bnbwd4(const Epi& e, int64_t m, int n, float4 t, float4 y4, float4 z4,
                                           const float4 (&bn)[3], float (&s)[3][4]) {
    const int64_t off = m * e.ldy + n;
    float g[4] = {t.x, t.y, t.z, t.w};
    if (e.frelu) {
        if (!(y4.x > 0.f)) g[0] = 0.f;
        if (!(y4.y > 0.f)) g[1] = 0.f;
        if (!(y4.z > 0.f)) g[2] = 0.f;
        if (!(y4.w > 0.f)) g[3] = 0.f;
    }
    const float sc[4] = {bn[0].x, bn[0].y, bn[0].z, bn[0].w}, mu[4] = {bn[1].x, bn[1].y, bn[1].z, bn[1].w};
    const float rs[4] = {bn[2].x, bn[2].y, bn[2].z, bn[2].w}, zz[4] = {z4.x, z4.y, z4.z, z4.w};
    float d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        d[q] = g[q] * sc[q];
        s[0][q] += g[q];
        s[1][q] += g[q] * ((zz[q] - mu[q]) * rs[q]);
        s[2][q] += d[q];
    }
    st4(e.y + off, make_float4(d[0], d[1], d[2], d[3]));
    if (e.fdres) st4(e.fdres + off, make_float4(g[0], g[1], g[2], g[3]));
}

__device__ __forceinline__ void epi_store4(const ConvP& p, const Epi& e, int64_t m, int n, float4 v) {
    if (e.split > 0 || (e.ldy & 3)) {
        epi_store(p, e, m, n, v.x);
        epi_store(p, e, m, n + 1, v.y);
        epi_store(p, e, m, n + 2, v.z);
        epi_store(p, e, m, n + 3, v.w);
        return;
    }
    int b = 0, oy = 0, ox = 0, oz = 0;
    if (!e.simple || e.res_mode == 2) decompose(m, p.OH, p.OW, p.OD, b, oy, ox, oz);
    const int64_t zrow = m * p.N + n;
    const int64_t yrow = e.simple ? m : out_row(p, e, b, oy, ox, oz, n);   // (n -> channel)
    if (e.bias) {
        const float4 bb = ld4(e.bias + n);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
    }
    if (e.z) st4(e.z + zrow, v);
    if (e.scale) {
        const float4 sc = ld4(e.scale + n), sh = ld4(e.shift + n);
        v.x = v.x * sc.x + sh.x; v.y = v.y * sc.y + sh.y;
        v.z = v.z * sc.z + sh.z; v.w = v.w * sc.w + sh.w;
    }
    if (e.res_mode == 1 || e.res_mode == 2) {
        const float4 r = e.res_mode == 1
                             ? ld4(e.res + yrow * e.ldy + n)
                             : ld4(e.res + ((((int64_t)b * (p.OH >> 1) + (oy >> 1)) * (p.OW >> 1) +
                                             (ox >> 1)) * p.OD + oz) * p.N + n);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    if (e.relu) {
        v.x = act(e.relu, v.x); v.y = act(e.relu, v.y); v.z = act(e.relu, v.z); v.w = act(e.relu, v.w);
    }
    if (e.res_mode == 3) {
        const float4 r = ld4(e.res + yrow * e.ldy + n);
        v.x += r.x; v.y += r.y; v.z += r.z; v.w += r.w;
    }
    float* dst = e.y + yrow * e.ldy + n;
    if (e.accumulate) {
        const float4 o = ld4(dst);
        v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
    }
    st4(dst, v);
}

// epi_store4 of a simple (y row == m) store whose same-shape residual
// (res_mode 1, no accumulate) or accumulated destination (res_mode 0) was loaded beforehand
// into `pre` -- the epilogue issues all of a thread's loads before its first
// store (the res / y pointers may alias, so the compiler cannot hoist a load
// over an earlier store: one HBM round trip per float4 otherwise).
__device__ __forceinline__ void epi_store4_pre(const ConvP& p, const Epi& e, int64_t m, int n, float4 v,
                                               const float4& pre) {
    const int64_t zrow = m * p.N + n;
    if (e.bias) {
        const float4 bb = ld4(e.bias + n);
        v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w;
    }
    if (e.z) st4(e.z + zrow, v);
    if (e.scale) {
        const float4 sc = ld4(e.scale + n), sh = ld4(e.shift + n);
        v.x = v.x * sc.x + sh.x; v.y = v.y * sc.y + sh.y;
        v.z = v.z * sc.z + sh.z; v.w = v.w * sc.w + sh.w;
    }
    if (e.res_mode == 1) {
        v.x += pre.x; v.y += pre.y; v.z += pre.z; v.w += pre.w;
    }
    if (e.relu) {
        v.x = act(e.relu, v.x); v.y = act(e.relu, v.y); v.z = act(e.relu, v.z); v.w = act(e.relu, v.w);
    }
    float* dst = e.y + m * e.ldy + n;
    if (e.accumulate) {      // (res_mode 0 here: pre holds the old destination)
        v.x += pre.x; v.y += pre.y; v.z += pre.z; v.w += pre.w;
    }
    st4(dst, v);
}

// -------------------------------------------------------------------------
// fwd / bwd-data implicit GEMM
// -------------------------------------------------------------------------
// FBN: the data gradient with the fused BN-ReLU backward of the unit it feeds
// (its own instantiation at 2 blocks/CU: the epilogue's extra rows and sums
// spill at 3, and must not touch the register budget of the other forms)
template <int BM, int BN, int WM, int WN, bool BT, bool AVEC, int BK, int NBUF, bool PERSIST = false,
          bool X3 = false, bool FBN = false>
__global__ __launch_bounds__(256, BK == 64 ? 1 : (NBUF == 1 && !FBN ? 3 : 2)) void conv_gemm_kernel(ConvP p,
                                                                                                  Epi e) {
    static_assert(BK == 32 || BK == 64, "BK");
    static_assert(!X3 || (BK == 32 && NBUF == 1 && AVEC && (BT || BN >= 64)), "X3 mode");
    static_assert(AVEC || BK == 32, "scalar A loader is BK=32");
    static_assert(!FBN || !PERSIST, "fused BN backward: one tile per block");
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
    constexpr int KC4 = BK / 4;                      // float4 columns of a k-tile row
    constexpr int RPP = 256 / KC4;                   // tile rows loaded per pass
    constexpr int AQ = AVEC ? BM / RPP : BM / 8;     // A elements (float4 or float) per thread
    constexpr int BQ = BT ? BN / RPP : BK * BN / 1024;   // B float4 per thread
    // NBUF 2: double-buffered LDS (one barrier per k-tile); NBUF 1: one LDS
    // stage (two barriers per k-tile) so 3 workgroups fit a CU.  Both keep the
    // next k-tile's global loads in flight in registers during the MFMAs.
    static_assert(NBUF == 1 || NBUF == 2, "NBUF");
    // X3: three bf16 planes per operand, [row][32 k] (64-B rows, swizzled),
    // B rows = n for both B layouts (the !BT loader transposes while splitting)
    constexpr int STAGE = X3 ? 3 * (BM + BN) * BK / 2 : A_SZ + B_SZ;   // floats
    __shared__ __attribute__((aligned(16))) float smem[NBUF * STAGE];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / WN, wn = wave % WN;
    // XCD-aware tile order (speed only): the dispatcher deals consecutive
    // workgroups round-robin to the 8 XCDs; remap so each XCD owns a contiguous
    // run of tiles, N-tiles of one M-tile adjacent, so the im2col rows (and
    // their 3x3x3 halo) are re-read from that XCD's L2, not from HBM.
    // PERSIST: a grid of ~one wave of workgroups loops over all tiles (all
    // batches), issuing the next tile's first k-tile loads before the current
    // tile's epilogue, so short-K GEMMs (the Winograd point GEMMs, K = Cin)
    // do not pay a cold prologue per tile.  gridDim.x is a multiple of 8, so a
    // workgroup stays on its XCD and walks that XCD's contiguous tile range.
    static_assert(!PERSIST || AVEC, "persistent mode uses the vector A loader");
    const int64_t nbx = (p.M + BM - 1) / BM, nby = (p.N + BN - 1) / BN;
    const int64_t per_batch = nbx * nby;
    const int64_t total = PERSIST ? per_batch * (int64_t)p.nbatch : (int64_t)gridDim.x * gridDim.y;
    int64_t L = PERSIST ? (int64_t)blockIdx.x : (int64_t)blockIdx.x + (int64_t)gridDim.x * blockIdx.y;
    const int64_t Lstep = PERSIST ? (int64_t)gridDim.x : total;
    if (L >= total) return;
    const float* const a_base = p.a;
    const float* const w_base = p.w;
    float* const y_base = e.y;
    int64_t m0 = 0;
    int n0 = 0;
    auto map_tile = [&](int64_t Lt) {
        const int64_t xcd = Lt % 8, q8 = total / 8, r8 = total % 8;
        const int64_t T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Lt / 8;
        const int64_t bz = PERSIST ? T / per_batch : (int64_t)blockIdx.z;
        const int64_t Tt = PERSIST ? T - bz * per_batch : T;
        m0 = (Tt / nby) * BM;
        n0 = (int)(Tt % nby) * BN;
        p.a = a_base + bz * p.bsa;
        p.w = w_base + bz * p.bsw;
        e.y = y_base + bz * p.bsy;
    };
    map_tile(L);
    const int taps_kd = p.kd, taps_kwkd = p.kw * p.kd;
    const int ntaps = p.kh * taps_kwkd;

    // per-thread A rows (vector path): base coordinates and 32-bit element
    // offsets (tensor bytes < 4 GiB is checked on the host)
    int a_y[AVEC ? AQ : 1], a_x[AVEC ? AQ : 1], a_z[AVEC ? AQ : 1], a_off[AVEC ? AQ : 1];
    bool a_ok[AVEC ? AQ : 1];
    const int a_col4 = tid % KC4;
    const int rowW = p.D * p.C, rowH = p.W * rowW;
    __amdgpu_buffer_rsrc_t rsA, rsB;
    auto setup_rows = [&]() {
        if (AVEC) {
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                const int64_t m = m0 + tid / KC4 + RPP * q;
                a_ok[q] = m < p.M;
                int b, oy, ox, oz;
                decompose(a_ok[q] ? m : 0, p.OH, p.OW, p.OD, b, oy, ox, oz);
                a_y[q] = oy * p.sy - p.py;
                a_x[q] = ox * p.sx - p.px;
                a_z[q] = oz * p.sz - p.pz;
                a_off[q] = ((b * p.H + a_y[q]) * p.W + a_x[q]) * rowW + a_z[q] * p.C + a_col4 * 4;
            }
        }
        rsA = make_rsrc(p.a, (uint64_t)p.B * p.H * p.W * p.D * p.C * 4);
        // BT rows are (tap, n) of p.C channels; a split-K slice (p.K < taps * p.C) reads a
        // channel window of every row, so the range is the whole weight
        rsB = make_rsrc(p.w, BT ? (uint64_t)ntaps * p.N * p.C * 4 : (uint64_t)p.K * p.N * 4);
    };
    setup_rows();

    float4 ra[AVEC ? AQ : 1];
    float rs[AVEC ? 1 : AQ];
    float4 rb[BQ];

    auto load_tile = [&](int kt) {
        const int k0 = kt * BK;
        if (AVEC) {
            const int tap = k0 / p.C;
            const int c0 = k0 - tap * p.C;
            const int ky = tap / taps_kwkd * p.dly, kx = (tap / taps_kd) % p.kw * p.dlx,
                      kz = tap % taps_kd * p.dlz;
            const int toff = ky * rowH + kx * rowW + kz * p.C + c0;
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                const bool ok = a_ok[q] && (unsigned)(a_y[q] + ky) < (unsigned)p.H &&
                                (unsigned)(a_x[q] + kx) < (unsigned)p.W &&
                                (unsigned)(a_z[q] + kz) < (unsigned)p.D;
                ra[q] = bload4(rsA, ok ? (uint32_t)(a_off[q] + toff) * 4u : M3D_OOB);
            }
        } else {
            const int col = tid & 31;
            const int k = k0 + col;
            int tap = 0, c = 0, ky = 0, kx = 0, kz = 0;
            if (k < p.K) {
                tap = k / p.C;
                c = k - tap * p.C;
                ky = tap / taps_kwkd * p.dly; kx = (tap / taps_kd) % p.kw * p.dlx; kz = tap % taps_kd * p.dlz;
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
                // X3: thread owns k rows BQ*(tid/C4) .. +BQ-1 of one n quad
                const int kr = X3 ? BQ * (tid / C4) + q : idx / C4, c4 = X3 ? tid % C4 : idx % C4;
                const int k = k0 + kr, n = n0 + c4 * 4;
                rb[q] = bload4(rsB, (k < p.K && n < p.N) ? (uint32_t)(k * p.N + n) * 4u : M3D_OOB);
            }
        } else {
            // B(k=(t,c'), n) = w[(t'*N + n)*C + c'], tile rows n, 32 contiguous c'
            const int tap = k0 / p.C;
            const int c0 = k0 - tap * p.C;
            const int wt = p.flip ? (ntaps - 1 - tap) : tap;
#pragma unroll
            for (int q = 0; q < BQ; ++q) {
                const int n = n0 + tid / KC4 + RPP * q;
                rb[q] = bload4(rsB, n < p.N ? (uint32_t)((wt * p.N + n) * p.C + c0 + a_col4 * 4) * 4u
                                            : M3D_OOB);
            }
        }
    };

    auto store_tile = [&](int buf) {
        if constexpr (X3) {
            char* Ab = reinterpret_cast<char*>(smem);
            char* Bb = Ab + 3 * BM * BK * 2;
#pragma unroll
            for (int q = 0; q < AQ; ++q) {
                uint2 o[3];
                split3x4(ra[q], o);
                const int off = x3_off(tid / KC4 + RPP * q, a_col4 * 4);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl)
                    *reinterpret_cast<uint2*>(Ab + pl * (BM * BK * 2) + off) = o[pl];
            }
            if constexpr (BT) {
#pragma unroll
                for (int q = 0; q < BQ; ++q) {
                    uint2 o[3];
                    split3x4(rb[q], o);
                    const int off = x3_off(tid / KC4 + RPP * q, a_col4 * 4);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        *reinterpret_cast<uint2*>(Bb + pl * (BN * BK * 2) + off) = o[pl];
                }
            } else {
                // rb[q] = B[k0 + BQ*g + q][n .. n+3]: per n, BQ consecutive k
                constexpr int C4 = BN / 4;
                const int g = tid / C4, n4 = (tid % C4) * 4;
                uint32_t hb[BQ][4], mb[BQ][4], lb[BQ][4];
#pragma unroll
                for (int q = 0; q < BQ; ++q) {
                    split3(rb[q].x, hb[q][0], mb[q][0], lb[q][0]);
                    split3(rb[q].y, hb[q][1], mb[q][1], lb[q][1]);
                    split3(rb[q].z, hb[q][2], mb[q][2], lb[q][2]);
                    split3(rb[q].w, hb[q][3], mb[q][3], lb[q][3]);
                }
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const int off = x3_off(n4 + c, BQ * g);
                    if constexpr (BQ == 4) {
                        *reinterpret_cast<uint2*>(Bb + off) =
                            make_uint2(hb[0][c] | (hb[1][c] << 16), hb[2][c] | (hb[3][c] << 16));
                        *reinterpret_cast<uint2*>(Bb + BN * BK * 2 + off) =
                            make_uint2(mb[0][c] | (mb[1][c] << 16), mb[2][c] | (mb[3][c] << 16));
                        *reinterpret_cast<uint2*>(Bb + 2 * BN * BK * 2 + off) =
                            make_uint2(lb[0][c] | (lb[1][c] << 16), lb[2][c] | (lb[3][c] << 16));
                    } else {
                        static_assert(BQ == 2, "X3 B tile");
                        *reinterpret_cast<uint32_t*>(Bb + off) = hb[0][c] | (hb[1][c] << 16);
                        *reinterpret_cast<uint32_t*>(Bb + BN * BK * 2 + off) = mb[0][c] | (mb[1][c] << 16);
                        *reinterpret_cast<uint32_t*>(Bb + 2 * BN * BK * 2 + off) = lb[0][c] | (lb[1][c] << 16);
                    }
                }
            }
            return;
        }
        float* As = smem + buf * (A_SZ + B_SZ);
        float* Bs = As + A_SZ;
        if (AVEC) {
#pragma unroll
            for (int q = 0; q < AQ; ++q)
                *reinterpret_cast<float4*>(As + (tid / KC4 + RPP * q) * LDA + a_col4 * 4) = ra[q];
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
                *reinterpret_cast<float4*>(Bs + (tid / KC4 + RPP * q) * LDB + a_col4 * 4) = rb[q];
        }
    };

    const int nk = (p.K + BK - 1) / BK;
    const int h = lane >> 5, l32 = lane & 31;
    load_tile(0);
    store_tile(0);
    __syncthreads();
    while (true) {
    floatx16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;

    for (int kt = 0; kt < nk; ++kt) {
        const int buf = NBUF == 2 ? (kt & 1) : 0;
        if (kt + 1 < nk) load_tile(kt + 1);
        if constexpr (X3) {
            const char* Ab = reinterpret_cast<const char*>(smem);
            const char* Bb = Ab + 3 * BM * BK * 2;
            // (fresh-accumulator form: one k step at a time -- unrolled, the two
            // steps' fragments and partials exceed the register budget)
#pragma unroll 2
            for (int s16 = 0; s16 < BK / 16; ++s16) {
                // lane (l32, h): row l32, k = 16 s16 + 8h .. +7 (one 16-B chunk)
                bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int off = x3_off(wm * TM * 32 + i * 32 + l32, 16 * s16 + 8 * h);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        af[i][pl] = *reinterpret_cast<const bf16x8*>(Ab + pl * (BM * BK * 2) + off);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int off = x3_off(wn * TN * 32 + j * 32 + l32, 16 * s16 + 8 * h);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl)
                        bfr[j][pl] = *reinterpret_cast<const bf16x8*>(Bb + pl * (BN * BK * 2) + off);
                }
                x3_mac_tiles<TM, TN>(acc, af, bfr);
            }
        } else {
        const float* As = smem + buf * (A_SZ + B_SZ);
        const float* Bs = As + A_SZ;
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
        // fragments: lane (l32, h) owns row l32 of each 32-row tile and the 16
        // k values 32ks+16h .. +15 of this k-tile (MFMA step s consumes k = 32ks+16h+s)
        float4 af[TM][4];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                af[i][q] = *reinterpret_cast<const float4*>(As + (wm * TM * 32 + i * 32 + l32) * LDA +
                                                            ks * 32 + h * 16 + 4 * q);
        float4 bf[BT ? TN : 1][4];
        if (BT) {
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    bf[j][q] = *reinterpret_cast<const float4*>(Bs + (wn * TN * 32 + j * 32 + l32) * LDB +
                                                                ks * 32 + h * 16 + 4 * q);
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int kk = ks * 32 + h * 16 + s;
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
        }
        }
        if (NBUF == 2) {
            if (kt + 1 < nk) store_tile(buf ^ 1);
            __syncthreads();
        } else {
            __syncthreads();
            if (kt + 1 < nk) {
                store_tile(0);
                __syncthreads();
            }
        }
    }

    // epilogue: D[row][col], col = lane&31 (n), row = (r&3) + 8(r>>2) + 4h (m).
    // The tile is staged through LDS (row stride BN+8: the two lane halves
    // write rows 4 apart = 32 banks apart, conflict-free) and leaves as
    // row-contiguous float4s: 16-byte stores and one epilogue evaluation per
    // 4 channels instead of per element.  (The k-loop ended on a barrier.)
    // PERSIST: once the accumulators are staged in LDS (acc dead), map the
    // next tile and put its first k-tile loads in flight behind this tile's
    // global epilogue stores.
    const int64_t m0c = m0;
    const int n0c = n0;
    const int64_t Ln = L + Lstep;
    const bool more = PERSIST && Ln < total;
    constexpr int LDT = BN + 8;
    constexpr int HALVES = (BM * LDT <= NBUF * STAGE) ? 1 : 2;   // staged in row halves
    constexpr int HR = BM / HALVES;
    static_assert(HR * LDT <= NBUF * STAGE, "epilogue tile must fit the k-loop LDS");
    static_assert(HALVES == 1 || (TM * 32) % HR == 0 || HR % (TM * 32) == 0, "wave rows vs halves");
    float* Ts = smem;
    constexpr int C4T = BN / 4;
    constexpr int QN = (HR * C4T + 255) / 256;
    // residual / accumulated-destination rows loaded before the staging (block-uniform)
    const bool pf = !PERSIST && e.simple && e.split <= 0 && !(e.ldy & 3) &&
                    ((e.res_mode == 1 && !e.accumulate) || (e.res_mode == 0 && e.accumulate));
    float fs[3][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};   // fused BN sums
    // fused BN: a thread's channel quad is the same in every batch (256 % C4T == 0)
    static_assert(256 % C4T == 0, "fixed channel quad per thread");
    float4 fbn4[3] = {make_float4(1.f, 1.f, 1.f, 1.f), make_float4(0.f, 0.f, 0.f, 0.f),
                      make_float4(1.f, 1.f, 1.f, 1.f)};
    if (FBN) {
        const int n = n0c + (tid % C4T) * 4;
        if (n < p.N) {
            if (e.fscale) fbn4[0] = ld4(e.fscale + n);
            if (e.fz) { fbn4[1] = ld4(e.fmean + n); fbn4[2] = ld4(e.frstd + n); }
        }
    }
    for (int hf = 0; hf < HALVES; ++hf) {
        if (hf) __syncthreads();                 // previous half fully read
        if ((wm * TM * 32) / HR == hf) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int j = 0; j < TN; ++j)
#pragma unroll
                    for (int r = 0; r < 16; ++r)
                        Ts[(wm * TM * 32 - hf * HR + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LDT +
                           wn * TN * 32 + j * 32 + l32] = acc[i][j][r];
        }
        __syncthreads();
        float* y_next = e.y;
        if (PERSIST && more && hf == HALVES - 1) {
            float* const yc = e.y;
            map_tile(Ln);                        // sets p.a/p.w/e.y, m0/n0 of the next tile
            y_next = e.y;
            e.y = yc;
            setup_rows();
            load_tile(0);
        }
        // PB float4 per thread per batch: with pf, the batch's residual /
        // destination loads are all issued before its first store
        constexpr int PB = QN < 4 ? QN : 4;
        static_assert(QN % PB == 0, "epilogue batches");
#pragma unroll
        for (int q0 = 0; q0 < QN; q0 += PB) {
            float4 pre[PB];
            float4 fy4[PB], fz4[PB];
            if (FBN) {                           // the batch's y / z rows before its first store
#pragma unroll
                for (int u = 0; u < PB; ++u) {
                    const int idx = tid + 256 * (q0 + u);
                    const int row = idx / C4T, c4 = idx % C4T;
                    const int64_t m = m0c + hf * HR + row;
                    const int n = n0c + c4 * 4;
                    const bool in = idx < HR * C4T && m < p.M && n < p.N;
                    fy4[u] = in && e.frelu ? ld4(e.fy + m * e.ldy + n) : make_float4(1.f, 1.f, 1.f, 1.f);
                    fz4[u] = in && e.fz ? ld4(e.fz + m * e.ldy + n) : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            if (pf) {
                const float* src = e.res_mode == 1 ? e.res : e.y;
#pragma unroll
                for (int u = 0; u < PB; ++u) {
                    const int idx = tid + 256 * (q0 + u);
                    const int row = idx / C4T, c4 = idx % C4T;
                    const int64_t m = m0c + hf * HR + row;
                    const int n = n0c + c4 * 4;
                    pre[u] = (idx < HR * C4T && m < p.M && n < p.N) ? ld4(src + m * e.ldy + n)
                                                                    : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
#pragma unroll
            for (int u = 0; u < PB; ++u) {
                const int idx = tid + 256 * (q0 + u);
                const int row = idx / C4T, c4 = idx % C4T;
                const int64_t m = m0c + hf * HR + row;
                const int n = n0c + c4 * 4;
                if ((HR * C4T % 256 == 0 || idx < HR * C4T) && m < p.M && n < p.N) {
                    const float4 v = *reinterpret_cast<const float4*>(Ts + row * LDT + c4 * 4);
                    if (PERSIST) {  // plain C store (host-checked: simple epilogue, nothing fused)
                        st4(e.y + m * e.ldy + n, v);
                    } else if (FBN) {     // (host-checked: simple rows, no bias / BN / residual / act)
                        float4 t = v;
                        if (e.accumulate) {
                            const float4 o = pf ? pre[u] : ld4(e.y + m * e.ldy + n);
                            t.x += o.x; t.y += o.y; t.z += o.z; t.w += o.w;
                        }
                        epi_bnbwd4(e, m, n, t, fy4[u], fz4[u], fbn4, fs);
                    } else if (pf) {
                        epi_store4_pre(p, e, m, n, v, pre[u]);
                    } else {
                        epi_store4(p, e, m, n, v);
                    }
                }
            }
        }
        e.y = y_next;
    }
    if constexpr (FBN) {
        if (e.fpart) {
            // channel sums of the tile: threads t, t + C4T, ... hold channel quad t % C4T
            __syncthreads();                     // staged tile fully read: Ts reused
            float* red = Ts;                     // [256][12]
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int q = 0; q < 4; ++q) red[tid * 12 + a * 4 + q] = fs[a][q];
            __syncthreads();
            if (tid < C4T) {
                float r[12];
#pragma unroll
                for (int k = 0; k < 12; ++k) r[k] = red[tid * 12 + k];
                for (int o = tid + C4T; o < 256; o += C4T)
#pragma unroll
                    for (int k = 0; k < 12; ++k) r[k] += red[o * 12 + k];
                const int n = n0c + tid * 4;
                const int64_t row = m0c / BM;
                if (n < p.N)
#pragma unroll
                    for (int a = 0; a < 3; ++a)
                        st4(e.fpart + ((int64_t)a * e.fprows + row) * p.N + n,
                            make_float4(r[a * 4], r[a * 4 + 1], r[a * 4 + 2], r[a * 4 + 3]));
            }
        }
    }
    if (!more) break;
    L = Ln;
    __syncthreads();                             // staged tile fully read
    store_tile(0);
    __syncthreads();
    }
}

// -------------------------------------------------------------------------
// Weight-gradient epilogue target.  Default: fp32 atomics into C (the m-splits
// of a tile arrive in any order, so the last bits vary run to run).
// Deterministic mode (m3d_set_deterministic): each split stores its tile into
// part[split][batch][K][N] of the registered scratch and wg_reduce_kernel adds
// the splits to C in split order; with a single split (the scratch too small
// for two), the one writer of each element adds to C without an atomic.
// -------------------------------------------------------------------------
struct WgOut {
    float* part;
    int64_t pstride;      // floats per split (nbatch * K * N)
    int plain;
};

__device__ __forceinline__ void wg_put(const WgOut& o, float* C, float* P, int64_t idx, float v) {
    if (P) P[idx] = v;
    else if (o.plain) C[idx] += v;
    else unsafeAtomicAdd(C + idx, v);
}

// C[b*bsc + r] += sum_{s = 0..splits-1} part[s][b][r]  (r < K*N), summed in s order
__global__ __launch_bounds__(256) void wg_reduce_kernel(const float* __restrict__ part, int splits,
                                                        int64_t pstride, int64_t kn, int64_t bsc,
                                                        float* __restrict__ C) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= pstride) return;
    float s = part[i];
    for (int q = 1; q < splits; ++q) s += part[q * pstride + i];
    const int64_t b = i / kn, r = i - b * kn;
    C[b * bsc + r] += s;
}

// deterministic-mode target for `splits` m-splits of an nbatch x K x N gradient
// (splits may be lowered to what the scratch holds)
static WgOut wg_out(int64_t& splits, int64_t nbatch, int64_t K, int64_t N) {
    WgOut o{nullptr, 0, 0};
    const DetState d = det();
    if (!d.on) return o;
    const int64_t per = nbatch * K * N;
    const int64_t fit = (int64_t)(d.bytes / sizeof(float)) / per;
    if (splits <= 1 || fit < 2) {
        splits = 1;
        o.plain = 1;
        return o;
    }
    if (splits > fit) splits = fit;
    o.part = static_cast<float*>(d.scratch);
    o.pstride = per;
    return o;
}

static void wg_finish(const WgOut& o, int64_t splits, int64_t nbatch, int64_t K, int64_t N, int64_t bsc,
                      float* C, hipStream_t s) {
    if (!o.part) return;
    hipLaunchKernelGGL(wg_reduce_kernel, dim3(grid_for(o.pstride, 256)), dim3(256), 0, s, o.part, (int)splits,
                       o.pstride, K * N, nbatch > 1 ? bsc : K * N, C);
}

// -------------------------------------------------------------------------
// bwd-weight: dW[k][n] += sum_m im2col(X)[m][k] * dZ[m][n]
// grid (K/BI, N/BJ, splits); each block reduces its m-range, fp32 atomics out
// (or the deterministic-mode target, WgOut).
// -------------------------------------------------------------------------
template <int BI, int BJ, int WI, int WJ, bool AVEC, bool HALO = false>
__global__ __launch_bounds__(256, 2) void conv_wgrad_kernel(ConvP p, const float* __restrict__ dz,
                                                            float* __restrict__ dw,
                                                            int64_t m_per_split, WgOut wo) {
    constexpr int BKM = 32;
    constexpr int TI = BI / (WI * 32), TJ = BJ / (WJ * 32);
    static_assert(WI * WJ == 4, "4 waves");
    constexpr int X_SZ = BKM * BI, G_SZ = BKM * BJ;
    constexpr int XQ = AVEC ? BI / 32 : BI / 8;
    constexpr int GQ = BJ / 32;
    __shared__ __attribute__((aligned(16))) float smem[2 * (X_SZ + G_SZ)];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave / WJ, wj = wave % WJ;
    // XCD-aware order: the dispatcher deals consecutive workgroups round-robin
    // to the 8 XCDs; remap so each XCD runs a contiguous range, i.e. the (K,N)
    // tiles of one m-range share their A / dZ rows through one L2 (without it
    // every tile of an m-range sat on a different XCD and re-read the rows
    // from HBM: 2.7x the algorithmic bytes)
    const int64_t gxy = (int64_t)gridDim.x * gridDim.y;
    const int64_t total = gxy * gridDim.z;
    const int64_t Lb = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    const int64_t xcd = Lb % 8, q8 = total / 8, r8 = total % 8;
    const int64_t Lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Lb / 8;
    const int bz_ = (int)(Lt / gxy), rem = (int)(Lt % gxy);
    const int k0 = (rem % gridDim.x) * BI;
    const int n0 = (rem / gridDim.x) * BJ;
    const int64_t nsplit = (p.M + m_per_split - 1) / m_per_split;
    const int64_t batch = bz_ / nsplit;
    float* const wp = wo.part ? wo.part + (bz_ % nsplit) * wo.pstride + batch * (int64_t)p.K * p.N : nullptr;
    if (batch) {
        p.a += batch * p.bsa;
        dz += batch * p.bsw;
        dw += batch * p.bsy;
    }
    const int64_t ms = (int64_t)(bz_ % nsplit) * m_per_split;
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
        if (z >= p.OD) {                 // rare when OD >= 32: carry by division
            x += z / p.OD;
            z %= p.OD;
            if (x >= p.OW) {
                y += x / p.OW;
                x %= p.OW;
                if (y >= p.OH) {
                    b += y / p.OH;
                    y %= p.OH;
                }
            }
        }
    };
    const int dx_ = HALO ? p.hdl : p.D;               // depth of the tensor behind p.a
    const __amdgpu_buffer_rsrc_t rsX =
        make_rsrc(p.a, (uint64_t)p.B * p.H * p.W * dx_ * p.C * 4);
    const __amdgpu_buffer_rsrc_t rsG = make_rsrc(dz, (uint64_t)p.M * p.N * 4);
    const int rowWx = dx_ * p.C, rowHx = p.W * rowWx;
    // halo planes: a second descriptor; each element is loaded from both with
    // one offset out of range (0) and the lane picks its source (no per-lane
    // descriptor select)
    const __amdgpu_buffer_rsrc_t rsH =
        make_rsrc(HALO ? p.halo : p.a, HALO ? (uint64_t)p.B * p.H * p.W * 2 * p.hr * p.C * 4 : 0);
    const int rowWh = 2 * p.hr * p.C, rowHh = p.W * rowWh;
    auto load_tile = [&](int64_t mb) {
        int rb = cb_, ry = cy_, rx = cx_, rz = cz_;
#pragma unroll
        for (int q = 0; q < XQ; ++q) {
            const int64_t m = mb + xrow0 + XRSTEP * q;
            if (q > 0) advance(rb, ry, rx, rz, XRSTEP);
            const int iy = ry * p.sy - p.py + ky, ix = rx * p.sx - p.px + kx,
                      iz = rz * p.sz - p.pz + kz;
            const bool ok = kok && m < me && (unsigned)iy < (unsigned)p.H &&
                            (unsigned)ix < (unsigned)p.W && (unsigned)iz < (unsigned)p.D;
            if constexpr (HALO) {
                const int zl = iz - p.hnlo;
                const bool inx = ok && (unsigned)zl < (unsigned)p.hdl;
                const bool inh = ok && !inx;
                const int pl = zl < 0 ? zl + p.hr : p.hr + zl - p.hdl;
                const uint32_t ox = inx ? (uint32_t)((rb * p.H + iy) * rowHx + ix * rowWx + zl * p.C + cc) * 4u
                                        : M3D_OOB;
                const uint32_t oh = inh ? (uint32_t)((rb * p.H + iy) * rowHh + ix * rowWh + pl * p.C + cc) * 4u
                                        : M3D_OOB;
                if (AVEC) {
                    const float4 vx = bload4(rsX, ox), vh = bload4(rsH, oh);
                    rx4[q] = inh ? vh : vx;
                } else {
                    const float vx = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsX, (int)ox, 0, 0));
                    const float vh = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsH, (int)oh, 0, 0));
                    rx1[q] = inh ? vh : vx;
                }
            } else {
                const uint32_t off = ok ? (uint32_t)((rb * p.H + iy) * rowHx + ix * rowWx + iz * p.C + cc) * 4u
                                        : M3D_OOB;
                if (AVEC) rx4[q] = bload4(rsX, off);
                else rx1[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsX, (int)off, 0, 0));
            }
        }
        advance(cb_, cy_, cx_, cz_, BKM);
#pragma unroll
        for (int q = 0; q < GQ; ++q) {
            const int64_t m = mb + grow0 + GRSTEP * q;
            const int n = n0 + gcol * 4;
            rg[q] = bload4(rsG, (m < me && n < p.N) ? (uint32_t)(m * p.N + n) * 4u : M3D_OOB);
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
                if (k < p.K) wg_put(wo, dw, wp, (int64_t)k * p.N + n, acc[i][j][r]);
            }
        }
}

// ------------------------------------------------------------------ dispatch
// CUs of the calling thread's current device, asked per call (the runtime
// answers from its device table): nothing is cached across calls or devices
static int num_cus() {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    return n;
}

// M3D_GEMM_X3 (bit mask, default 31): fp32 GEMMs on the exact 3-way bf16 split
// (6 bf16 MFMAs per product, see split3) instead of v_mfma_f32_32x32x2_f32.
// bit 0: Winograd fwd / bwd-data point GEMMs on operands pre-split by the
// transforms (x3_gemm_kernel; measured 39.9 -> 37.9 ms/step at 128^3, GEMM
// error vs fp64 below the f32 MFMA's: scripts/x3_accuracy.py); bit 1:
// implicit-GEMM convs splitting in the LDS store (neutral to -0.3 ms/step
// through round 3, on since round 4: -0.25 ms with the fused BN backward); bit 2: the
// Winograd weight-gradient GEMMs (x3_wgrad_kernel; 38.2 -> 37.0 ms/step);
// bit 3: the weight gradients of 1x1x1 stride-1 convs on the same kernel;
// bit 4: the Winograd input transform writes U as fp32 (4 B per point
// instead of 3 x 2 B) and the point GEMM (x3_gemm256_af_kernel, or
// x3_gemm_kernel<AF32>) splits it on its way into LDS: a third less HBM
// traffic for U, 34.2 -> 32.9 ms/step at 128^3 (default on).
static int x3_mask() {
    static constexpr int v = M3D_TUNE_GEMM_X3;
    return v;
}
static int gemm_x3_env() { return x3_mask() & 1; }
static int conv_x3_env() { return (x3_mask() >> 1) & 1; }

template <int BM, int BN, int WM, int WN, bool BT, bool AVEC, int BK>
static void launch_gemm(const ConvP& p, const Epi& e, hipStream_t s, int nbatch) {
    dim3 grid((unsigned)((p.M + BM - 1) / BM), (unsigned)((p.N + BN - 1) / BN), (unsigned)nbatch);
    if constexpr (BT && BK == 32) {
        if (e.fbn) {                       // the fused BN-ReLU backward's own instantiation
            if constexpr (AVEC) {
                if (conv_x3_env()) {       // the same GEMM form as the unfused data gradient
                    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1, false, true, true>), grid,
                                       dim3(256), 0, s, p, e);
                    return;
                }
            }
            hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1, false, false, true>), grid,
                               dim3(256), 0, s, p, e);
            return;
        }
    }
    if constexpr (BK == 32 && AVEC) {      // (the scalar-A loader spills at 3 blocks/CU)
        // one LDS stage at 3 blocks/CU (3-5 % faster than two stages at 2); the
        // batched plain GEMMs (Winograd points) as a persistent tile loop
        const int64_t tiles = (int64_t)grid.x * grid.y * nbatch;
        const int64_t resident = (int64_t)num_cus() * 3;
        const bool plain = e.simple && !e.bias && !e.scale && !e.res_mode && !e.relu && !e.z && !e.split &&
                           !e.accumulate && !e.deconv && !e.fbn && (e.ldy & 3) == 0;
        const bool persist = nbatch > 1 && plain && tiles > 2 * resident;
        ConvP pp = p;
        pp.nbatch = nbatch;
        const unsigned g = (unsigned)(resident / 8 * 8);
        if constexpr (BT || BN >= 64) {
            if (conv_x3_env()) {
                if (persist)
                    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1, true, true>), dim3(g),
                                       dim3(256), 0, s, pp, e);
                else
                    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1, false, true>), grid,
                                       dim3(256), 0, s, p, e);
                return;
            }
        }
        if (persist)
            hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1, true>), dim3(g), dim3(256), 0, s,
                               pp, e);
        else
            hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 1>), grid, dim3(256), 0, s, p, e);
        return;
    }
    hipLaunchKernelGGL((conv_gemm_kernel<BM, BN, WM, WN, BT, AVEC, BK, 2>), grid, dim3(256), 0, s, p, e);
}

template <bool BT, bool AVEC>
static void dispatch_gemm(const ConvP& p, const Epi& e, hipStream_t s, int nbatch = 1) {
    // 32-deep k-tiles (64-deep at 1 block/CU measured 25-30 % slower)
    if (p.N <= 32) {
        launch_gemm<128, 32, 4, 1, BT, AVEC, 32>(p, e, s, nbatch);
    } else if (p.N <= 64) {
        launch_gemm<128, 64, 4, 1, BT, AVEC, 32>(p, e, s, nbatch);
    } else {
        const int64_t blocks128 = ((p.M + 127) / 128) * ((p.N + 127) / 128) * nbatch;
        if (blocks128 < 512) launch_gemm<64, 128, 2, 2, BT, AVEC, 32>(p, e, s, nbatch);
        else launch_gemm<128, 128, 2, 2, BT, AVEC, 32>(p, e, s, nbatch);
    }
}

// M3D_WGRAD_MINM: minimum output rows reduced per workgroup (default 512: measured
// 45.6 ms/step vs 46.4 at 256, 47.0 at 1024, 47.5 at 128)
static int wgrad_minm_env() {
    static constexpr int v = M3D_TUNE_WGRAD_MINM;
    return v;
}

template <int BI, int BJ, int WI, int WJ, bool AVEC, bool HALO = false>
static void launch_wgrad(const ConvP& p, const float* dz, float* dw, hipStream_t s, int nbatch = 1) {
    const int64_t tiles = (int64_t)((p.K + BI - 1) / BI) * ((p.N + BJ - 1) / BJ) * nbatch;
    int64_t splits = (1024 + tiles - 1) / tiles;                   // aim >= 1024 blocks
    int64_t minm = wgrad_minm_env() > 32 ? wgrad_minm_env() : 32;
    const int64_t max_splits = (p.M + minm - 1) / minm;             // >= minm m per block
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    const WgOut wo = wg_out(splits, nbatch, p.K, p.N);
    int64_t mper = (p.M + splits - 1) / splits;
    mper = (mper + 31) / 32 * 32;
    splits = (p.M + mper - 1) / mper;
    dim3 grid((unsigned)((p.K + BI - 1) / BI), (unsigned)((p.N + BJ - 1) / BJ),
              (unsigned)(splits * nbatch));
    hipLaunchKernelGGL((conv_wgrad_kernel<BI, BJ, WI, WJ, AVEC, HALO>), grid, dim3(256), 0, s, p, dz, dw,
                       mper, wo);
    wg_finish(wo, splits, nbatch, p.K, p.N, p.bsy, dw, s);
}


// ---- weight-gradient GEMM on the exact bf16 split (plain batched rows) ----
// C[b][k][n] += sum_m A[b][m][k] B[b][m][n] (the Winograd weight gradient:
// A = transformed input, B = transformed output gradient), split3 of both
// operands in the LDS store.  The reduction index m is the slow axis of both
// operands, so each loader thread takes 8 consecutive m rows of one float4
// column and writes, per column, the 8 m values as one 16-byte k-chunk of the
// [row = k or n][32 m] planes (same swizzled image as x3_gemm_kernel).
// Threads 0-127 load A, 128-255 load B.  grid (K/128, N/128, splits * batch)
// with the XCD-contiguous order of conv_wgrad_kernel; fp32 atomics out.
template <int OCC>
__global__ __launch_bounds__(256, OCC) void x3_wgrad_kernel(const float* __restrict__ A,
                                                            const float* __restrict__ Bm,
                                                            float* __restrict__ C, int64_t M, int K, int N,
                                                            int64_t m_per_split, int64_t bsa, int64_t bsb,
                                                            int64_t bsc, WgOut wo) {
    constexpr int BI = 128, BJ = 128, TI = 2, TJ = 2, BKM = 32;
    constexpr int PL = 128 * BKM * 2;                    // bytes per plane (128 rows x 64 B)
    __shared__ __attribute__((aligned(16))) char smem[6 * PL];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wi = wave >> 1, wj = wave & 1, h = lane >> 5, l32 = lane & 31;
    const int64_t gxy = (int64_t)gridDim.x * gridDim.y;
    const int64_t total = gxy * gridDim.z;
    const int64_t Lb = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    const int64_t xcd = Lb % 8, q8 = total / 8, r8 = total % 8;
    const int64_t Lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Lb / 8;
    const int bz = (int)(Lt / gxy), rem = (int)(Lt % gxy);
    const int k0 = (rem % gridDim.x) * BI;
    const int n0 = (rem / gridDim.x) * BJ;
    const int64_t nsplit = (M + m_per_split - 1) / m_per_split;
    const int64_t batch = bz / nsplit;
    float* const wp = wo.part ? wo.part + (bz % nsplit) * wo.pstride + batch * (int64_t)K * N : nullptr;
    A += batch * bsa;
    Bm += batch * bsb;
    C += batch * bsc;
    const int64_t ms = (int64_t)(bz % nsplit) * m_per_split;
    const int64_t me = ms + m_per_split < M ? ms + m_per_split : M;
    if (ms >= me) return;
    // loader role: operand, float4 column, 8-row group
    // wave-uniform role (readfirstlane): a lane-divergent select of the buffer
    // resource wraps every load in a readfirstlane waterfall loop
    const bool isB = __builtin_amdgcn_readfirstlane(tid) >= 128;
    const int lt = tid & 127, c4 = lt & 31, grp = lt >> 5;
    const int ld = isB ? N : K;
    const int col = (isB ? n0 : k0) + c4 * 4;
    const bool colok = col < ld;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(isB ? (const void*)Bm : (const void*)A, (uint64_t)M * ld * 4);
    char* const Pb = smem + (isB ? 3 * PL : 0);
    float4 v[8];
    auto load = [&](int64_t mb) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int64_t m = mb + grp * 8 + r;
            v[r] = bload4(rs, (colok && m < me) ? (uint32_t)(m * ld + col) * 4u : M3D_OOB);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint32_t hh[8], mm[8], ll[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) split3(f4get(v[r], c), hh[r], mm[r], ll[r]);
            const int off = x3_off(c4 * 4 + c, grp * 8);
            *reinterpret_cast<uint4*>(Pb + off) =
                make_uint4(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16));
            *reinterpret_cast<uint4*>(Pb + PL + off) =
                make_uint4(mm[0] | (mm[1] << 16), mm[2] | (mm[3] << 16), mm[4] | (mm[5] << 16), mm[6] | (mm[7] << 16));
            *reinterpret_cast<uint4*>(Pb + 2 * PL + off) =
                make_uint4(ll[0] | (ll[1] << 16), ll[2] | (ll[3] << 16), ll[4] | (ll[5] << 16), ll[6] | (ll[7] << 16));
        }
    };
    floatx16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    const char* const As = smem;
    const char* const Bs = smem + 3 * PL;
    const int nchunks = (int)((me - ms + BKM - 1) / BKM);
    load(ms);
    store();
    __syncthreads();
    for (int t = 0; t < nchunks; ++t) {
        if (t + 1 < nchunks) load(ms + (int64_t)(t + 1) * BKM);
#pragma unroll 2
        for (int s16 = 0; s16 < 2; ++s16) {
            bf16x8 af[TI][3], bfr[TJ][3];
#pragma unroll
            for (int i = 0; i < TI; ++i) {
                const int off = x3_off(wi * TI * 32 + i * 32 + l32, 16 * s16 + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * PL + off);
            }
#pragma unroll
            for (int j = 0; j < TJ; ++j) {
                const int off = x3_off(wj * TJ * 32 + j * 32 + l32, 16 * s16 + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * PL + off);
            }
            x3_mac_tiles<TI, TJ>(acc, af, bfr);
        }
        __syncthreads();
        if (t + 1 < nchunks) {
            store();
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int n = n0 + wj * TJ * 32 + j * 32 + l32;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = k0 + wi * TI * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (k < K) wg_put(wo, C, wp, (int64_t)k * N + n, acc[i][j][r]);
            }
        }
}

// ---- the same product on 64x64 tiles (K or N <= 64: the res2 gradients) -----
// x3_wgrad_kernel's 128x128 tile at K = N = 64 runs four times the MFMAs it
// needs (three of its four waves multiply zeros), at K = 64 twice.  Here a
// workgroup owns one 64x64 output tile and the four waves split the m chunk
// instead of the tile: a chunk is
// 64 rows of m, staged as two 32-m sub-images per plane (the x3_off image of
// x3_wgrad_kernel, 64 rows each), and wave w multiplies m rows 16w..16w+15 into
// its own 64x64 accumulator (2 x 2 MFMA blocks).  The four partial tiles are
// summed through LDS in wave order at the end: one output per element and
// workgroup (fp32 atomics, or the deterministic partials, as x3_wgrad_kernel).
// grid: tiles * splits * batch workgroups (x), XCD-contiguous order with the
// tiles of one (batch, split) adjacent, so they share its m rows in one L2.
template <int OCC>
__global__ __launch_bounds__(256, OCC) void x3_wgrad64_kernel(const float* __restrict__ A,
                                                              const float* __restrict__ Bm,
                                                              float* __restrict__ C, int64_t M, int K, int N,
                                                              int64_t m_per_split, int64_t bsa, int64_t bsb,
                                                              int64_t bsc, WgOut wo) {
    constexpr int TI = 2, TJ = 2, BKM = 64;
    constexpr int SUB = 64 * 64;                         // one 32-m sub-image: 64 rows x 64 B
    constexpr int PL = 2 * SUB;                          // one plane of a 64-m chunk
    constexpr int RED = 4 * 64 * 64 * 4;                 // the four waves' partial tiles
    constexpr int SMEM = RED > 6 * PL ? RED : 6 * PL;
    __shared__ __attribute__((aligned(16))) char smem[SMEM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5, l32 = lane & 31;
    const int64_t total = gridDim.x;
    const int64_t Lb = blockIdx.x;
    const int64_t xcd = Lb % 8, q8 = total / 8, r8 = total % 8;
    const int64_t Lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Lb / 8;
    const int tk = (K + 63) / 64, tiles = tk * ((N + 63) / 64);
    const int tile = (int)(Lt % tiles);
    const int k0 = (tile % tk) * 64, n0 = (tile / tk) * 64;
    const int64_t bz = Lt / tiles;
    const int64_t nsplit = (M + m_per_split - 1) / m_per_split;
    const int64_t batch = bz / nsplit;
    float* const wp = wo.part ? wo.part + (bz % nsplit) * wo.pstride + batch * (int64_t)K * N : nullptr;
    A += batch * bsa;
    Bm += batch * bsb;
    C += batch * bsc;
    const int64_t ms = (bz % nsplit) * m_per_split;
    const int64_t me = ms + m_per_split < M ? ms + m_per_split : M;
    if (ms >= me) return;                                // (block-uniform)
    // loader role (wave-uniform): operand, float4 column (16 = 64 columns), 8-row group (8 = 64 rows)
    const bool isB = __builtin_amdgcn_readfirstlane(tid) >= 128;
    const int lt = tid & 127, c4 = lt & 15, grp = lt >> 4;
    const int ld = isB ? N : K;
    const int col = (isB ? n0 : k0) + c4 * 4;
    const bool colok = col < ld;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(isB ? (const void*)Bm : (const void*)A, (uint64_t)M * ld * 4);
    char* const Pb = smem + (isB ? 3 * PL : 0);
    const int soff = (grp >> 2) * SUB;
    const int lrow = c4 * 4;                             // the column's row in the tile image
    float4 v[8];
    auto load = [&](int64_t mb) {
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const int64_t m = mb + grp * 8 + r;
            v[r] = bload4(rs, (colok && m < me) ? (uint32_t)(m * ld + col) * 4u : M3D_OOB);
        }
    };
    auto store = [&]() {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            uint32_t hh[8], mm[8], ll[8];
#pragma unroll
            for (int r = 0; r < 8; ++r) split3(f4get(v[r], c), hh[r], mm[r], ll[r]);
            const int off = soff + x3_off(lrow + c, (grp & 3) * 8);
            *reinterpret_cast<uint4*>(Pb + off) =
                make_uint4(hh[0] | (hh[1] << 16), hh[2] | (hh[3] << 16), hh[4] | (hh[5] << 16), hh[6] | (hh[7] << 16));
            *reinterpret_cast<uint4*>(Pb + PL + off) =
                make_uint4(mm[0] | (mm[1] << 16), mm[2] | (mm[3] << 16), mm[4] | (mm[5] << 16), mm[6] | (mm[7] << 16));
            *reinterpret_cast<uint4*>(Pb + 2 * PL + off) =
                make_uint4(ll[0] | (ll[1] << 16), ll[2] | (ll[3] << 16), ll[4] | (ll[5] << 16), ll[6] | (ll[7] << 16));
        }
    };
    floatx16 acc[TI][TJ];
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    // this wave's 16 m rows of a chunk: sub-image wave / 2, k 16 (wave % 2) + 8h
    const char* const As = smem + (wave >> 1) * SUB;
    const char* const Bs = As + 3 * PL;
    const int kq = 16 * (wave & 1) + 8 * h;
    const int nchunks = (int)((me - ms + BKM - 1) / BKM);
    load(ms);
    store();
    __syncthreads();
    for (int t = 0; t < nchunks; ++t) {
        if (t + 1 < nchunks) load(ms + (int64_t)(t + 1) * BKM);
        bf16x8 af[TI][3], bfr[TJ][3];
#pragma unroll
        for (int i = 0; i < TI; ++i) {
            const int off = x3_off(i * 32 + l32, kq);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * PL + off);
        }
#pragma unroll
        for (int j = 0; j < TJ; ++j) {
            const int off = x3_off(j * 32 + l32, kq);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * PL + off);
        }
        x3_mac_tiles<TI, TJ>(acc, af, bfr);
        __syncthreads();
        if (t + 1 < nchunks) {
            store();
            __syncthreads();
        }
    }
    // (the loop's last barrier ended every read of the operand images)
    float* const R = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int i = 0; i < TI; ++i)
#pragma unroll
        for (int j = 0; j < TJ; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r)
                R[(wave * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * 64 + j * 32 + l32] = acc[i][j][r];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int idx = tid + 256 * q, k = k0 + (idx >> 6), n = n0 + (idx & 63);
        const float s = ((R[idx] + R[4096 + idx]) + R[8192 + idx]) + R[12288 + idx];
        if (k < K && n < N) wg_put(wo, C, wp, (int64_t)k * N + n, s);
    }
}

// ---- weight-gradient GEMM, 256x256 tiles, transposed LDS reads -------------
// Same product as x3_wgrad_kernel (C[b][k][n] += sum_m A[b][m][k] B[b][m][n],
// fp32 operands with the reduction index m as their rows, exact bf16 split).
// 512 threads = 8 waves (2 x 4; 128 x 64 outputs = 4 x 2 32x32 MFMA blocks per
// wave), one workgroup per CU.  A k-step is 16 rows of m: every thread loads
// two float4 of each operand (each wave one row-contiguous 1 KB access),
// splits them and writes each plane's four bf16 with one ds_write_b64 into a
// row-major [16 m][256 col] image (no register transpose).  The MFMA operand
// wants 8 consecutive m of one column per lane: two ds_read_b64_tr_b16 (4 rows
// x 16 columns per 16-lane group, gfx950's transposing LDS read) deliver it.
// Rows are padded to 576 B so the transposed reads (4 rows x 64 contiguous
// bytes per 32-lane half) and the row writes are bank-conflict-free.  Two LDS
// stages (2 x 54 KB) and two register sets: the loads of step t+2 are issued
// before the MFMAs of step t, the operands of step t+1 (loaded during step
// t-1) are split and written into the other stage behind them; one barrier
// per step.  fp32 atomics out (the m range is split over workgroups).
typedef short v4s __attribute__((ext_vector_type(4)));
constexpr int W2_BK = 16;
constexpr int W2_PITCH = 512 + 64;              // row pitch: 256 bf16 + 64 B pad
constexpr int W2_PL = W2_BK * W2_PITCH;         // one plane: 16 rows (9 KB)
constexpr int W2_STAGE = 6 * W2_PL;             // 3 planes of A + 3 of B = 54 KB

// The 64-B pad puts rows r..r+3 on four different 64-B bank groups, so a
// transposed read (4 rows x 64 contiguous bytes per 32-lane half) is
// conflict-free, and every fragment offset is a constant from one base.
__device__ __forceinline__ int w2_off(int row, int col) { return row * W2_PITCH + col * 2; }
__device__ __forceinline__ bf16x8 w2_frag(const char* plane, int o1, int o2) {
    typedef __attribute__((address_space(3))) v4s lds_v4s;
    const v4s r1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + o1));
    const v4s r2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(plane + o2));
    return __builtin_shufflevector(r1, r2, 0, 1, 2, 3, 4, 5, 6, 7);
}

// DBG (timing probes, selected by M3D_X3W_DBG): 1 no global loads, 2 no MFMAs,
// 3 neither split nor LDS writes (MFMAs on a stale stage), 4 loads issued and
// waited for at once, their data unused, 5 loads only (no split, no MFMA)
// One workgroup's pass over rows [ms, me) of one 256x256 output tile (k0, n0)
// of one batch item (A, Bm, C already offset to it), then its tile out.
template <int DBG>
__device__ __forceinline__ void x3w_segment(char* __restrict__ smem, const float* __restrict__ A,
                                            const float* __restrict__ Bm, float* __restrict__ C, int64_t M,
                                            int K, int N, int64_t ms, int64_t me, int k0, int n0,
                                            const WgOut& wo, float* wp, int64_t rot_seed) {
    if (ms >= me) return;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wk = wave >> 2, wn = wave & 3, h = lane >> 5, l32 = lane & 31;
    // loader: rows lr and lr + 8 of the step, columns lc..lc+3 of both operands
    const int lr = tid >> 6, lc = (tid & 63) * 4;
    const bool aok = k0 + lc < K, bok = n0 + lc < N;
    const uint32_t mrows = (uint32_t)(me - ms);
    // wave-uniform descriptors (a per-lane base would wrap every load in a
    // readfirstlane waterfall loop); rows relative to ms, 32-bit offsets
    const __amdgpu_buffer_rsrc_t rsa = make_rsrc(A + ms * K + k0, (uint64_t)(M - ms) * K * 4);
    const __amdgpu_buffer_rsrc_t rsb = make_rsrc(Bm + ms * N + n0, (uint64_t)(M - ms) * N * 4);
    const uint32_t oc = (uint32_t)lc * 4u;
    const uint32_t rowa = (uint32_t)K * 4u, rowb = (uint32_t)N * 4u;
    const int nk = (int)((me - ms + W2_BK - 1) / W2_BK);
    // Every workgroup walks its m range from a different step (rotation by
    // its tile index; the N-tiles sharing an A tile, same index, stay in step
    // for L2): the 256 concurrent streams start 8-16 MB apart, and in lockstep
    // they would hit the same HBM channels (2.2 TB/s measured without it).
    const int rot = (int)((rot_seed * 17) % nk);
    // steps past the last one load zeros (out-of-range offset): no branch in the loop
    auto load = [&](int kt, float4 (&va)[2], float4 (&vb)[2]) {
        const int ph = kt + rot >= nk ? kt + rot - nk : kt + rot;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const uint32_t m = (uint32_t)ph * W2_BK + lr + 8 * u;
            const bool in = kt < nk && m < mrows;
            if (DBG == 1) {
                va[u] = make_float4(m, u, kt, 1.0f);
                vb[u] = make_float4(u, m, 2.0f, kt);
            } else if (DBG == 4) {     // real loads, results sunk at once (no use)
                float4 ta = bload4(rsa, (in && aok) ? oc + m * rowa : M3D_OOB);
                float4 tb = bload4(rsb, (in && bok) ? oc + m * rowb : M3D_OOB);
                asm volatile("" ::"v"(ta.x), "v"(tb.x));
                va[u] = make_float4(m, u, kt, 1.0f);
                vb[u] = make_float4(u, m, 2.0f, kt);
            } else {
                va[u] = bload4(rsa, (in && aok) ? oc + m * rowa : M3D_OOB);
                vb[u] = bload4(rsb, (in && bok) ? oc + m * rowb : M3D_OOB);
            }
        }
    };
    auto split_store = [&](int buf, const float4 (&va)[2], const float4 (&vb)[2]) {
        if (DBG == 3 || DBG == 5) {
            asm volatile("" ::"v"(va[0].x), "v"(va[1].x), "v"(vb[0].x), "v"(vb[1].x));
            return;
        }
        char* S = smem + buf * W2_STAGE;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int off = w2_off(lr + 8 * u, lc);
            uint2 pa[3], pb[3];
            split3x4(va[u], pa);
            split3x4(vb[u], pb);
#pragma unroll
            for (int q = 0; q < 3; ++q) {
                *reinterpret_cast<uint2*>(S + q * W2_PL + off) = pa[q];
                *reinterpret_cast<uint2*>(S + (3 + q) * W2_PL + off) = pb[q];
            }
        }
    };
    // transposed-read offsets: lane 4q+p of 16-lane group g reads row 8(g>>1)+q
    // (and +4), columns base + 16(g&1) + 4p .. +3
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int trow = 8 * (g >> 1) + q, tcol = 16 * (g & 1) + 4 * p;
    const int abase = w2_off(trow, wk * 128 + tcol), bbase = w2_off(trow, wn * 64 + tcol);
    floatx16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    auto mfma_step = [&](int kt) {
        const char* S = smem + (kt & 1) * W2_STAGE;
        bf16x8 bfr[2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                bfr[j][pl] = w2_frag(S + (3 + pl) * W2_PL + j * 64, bbase, bbase + 4 * W2_PITCH);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            bf16x8 af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) af[pl] = w2_frag(S + pl * W2_PL + i * 64, abase, abase + 4 * W2_PITCH);
            if (DBG == 2 || DBG == 5) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j][0] += (float)(af[0][0] ^ af[1][1] ^ af[2][2] ^ bfr[j][0][3] ^ bfr[j][1][4] ^ bfr[j][2][5]);
                continue;
            }
            x3_mac_pair(acc[i][0], acc[i][1], af[0], af[1], af[2], bfr[0][0], bfr[0][1], bfr[0][2],
                                  bfr[1][0], bfr[1][1], bfr[1][2]);
        }
    };
    // two named register sets (static indexing): X carries step kt+1 (loaded
    // during step kt-1), Y receives step kt+2; the roles swap every step
    float4 xa[2], xb[2], ya[2], yb[2];
    load(0, xa, xb);
    split_store(0, xa, xb);
    load(1, xa, xb);
    __syncthreads();
    // sched_barrier(0) pins each step's loads ahead of its MFMAs (hipcc would
    // sink them to the end of the step, leaving one step of latency cover)
    for (int kt = 0; kt < nk; kt += 2) {
        load(kt + 2, ya, yb);
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(kt);
        split_store((kt + 1) & 1, xa, xb);   // the other stage: last read in step kt-1
        __syncthreads();
        load(kt + 3, xa, xb);                // zeros past the end (no branch)
        __builtin_amdgcn_sched_barrier(0);
        mfma_step(kt + 1);                   // past nk: a stage of zeros, no effect
        split_store(kt & 1, ya, yb);
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int n = n0 + wn * 64 + j * 32 + l32;
            if (n >= N) continue;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int k = k0 + wk * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                if (k < K) wg_put(wo, C, wp, (int64_t)k * N + n, acc[i][j][r]);
            }
        }
}

// Stream-K decomposition (non-deterministic mode): the launch's units (batch
// item, output tile, 16-row step) are cut into gridDim.x equal contiguous
// ranges, one per workgroup, so a launch whose tiles x splits leave a partial
// last round of one-per-CU workgroups (e.g. 288 tiles on 256 CUs: 1.125 rounds
// ran as 2) runs as one balanced round; a tile whose steps span two ranges is
// added into C by both (fp32 atomics, as the m splits).
struct X3wSK {
    int64_t units = 0;           // nbatch * tk * tn * nk
    int nk = 0, tk = 0, tn = 0;  // steps per tile, k / n tiles
};

template <int DBG, bool SK = false>
__global__ __launch_bounds__(512, 1) void x3_wgrad_tr_kernel(const float* __restrict__ A,
                                                             const float* __restrict__ Bm,
                                                             float* __restrict__ C, int64_t M, int K,
                                                             int N, int64_t m_per_split, int64_t bsa,
                                                             int64_t bsb, int64_t bsc, WgOut wo, X3wSK sk) {
    __shared__ __attribute__((aligned(16))) char smem[2 * W2_STAGE];
    if constexpr (SK) {
        // XCD-contiguous: the workgroups of one XCD take consecutive unit ranges.
        // The tn column tiles of one (batch, k tile) share their A rows, so they
        // run in lockstep: workgroups form groups of tn adjacent ones, a group
        // walks one range of (batch, k tile, step) units and member j takes
        // column tile j of each.  (Ranges over whole tiles drifted the partner
        // tiles' steps apart -- 288 steps per workgroup against 256 per tile --
        // and every A row was fetched from HBM twice: PMC 2.55 vs 1.89 GB.)
        const int64_t G = gridDim.x, L = blockIdx.x;
        const int64_t xcd = L % 8, q8 = G / 8, r8 = G % 8;
        const int64_t g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
        const int64_t Gg = G / sk.tn, grp = g / sk.tn;
        const int nj = (int)(g - grp * sk.tn);
        const int64_t ug = sk.units / sk.tn;              // (batch, k tile, step) units
        int64_t u = grp * ug / Gg;
        const int64_t ue = (grp + 1) * ug / Gg;
        while (u < ue) {
            const int64_t t = u / sk.nk;                  // batch * tk + k tile
            const int64_t s0 = u - t * sk.nk;
            const int64_t s1 = s0 + (ue - u) < sk.nk ? s0 + (ue - u) : sk.nk;
            const int64_t batch = t / sk.tk;
            const int kt = (int)(t - batch * sk.tk);
            const int64_t me = s1 * W2_BK < M ? s1 * W2_BK : M;
            x3w_segment<DBG>(smem, A + batch * bsa, Bm + batch * bsb, C + batch * bsc, M, K, N, s0 * W2_BK, me,
                             kt * 256, nj * 256, wo, nullptr, 0);
            u += s1 - s0;
        }
        return;
    }
    const int64_t gxy = (int64_t)gridDim.x * gridDim.y;
    const int64_t total = gxy * gridDim.z;
    const int64_t Lb = blockIdx.x + (int64_t)gridDim.x * (blockIdx.y + (int64_t)gridDim.y * blockIdx.z);
    const int64_t xcd = Lb % 8, q8 = total / 8, r8 = total % 8;
    const int64_t Lt = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + Lb / 8;
    const int bz = (int)(Lt / gxy), rem = (int)(Lt % gxy);
    const int k0 = (rem % gridDim.x) * 256;
    const int n0 = (rem / gridDim.x) * 256;
    const int64_t nsplit = (M + m_per_split - 1) / m_per_split;
    const int64_t batch = bz / nsplit;
    float* const wp = wo.part ? wo.part + (bz % nsplit) * wo.pstride + batch * (int64_t)K * N : nullptr;
    const int64_t ms = (int64_t)(bz % nsplit) * m_per_split;
    const int64_t me = ms + m_per_split < M ? ms + m_per_split : M;
    x3w_segment<DBG>(smem, A + batch * bsa, Bm + batch * bsb, C + batch * bsc, M, K, N, ms, me, k0, n0, wo, wp, bz);
}

// M3D_X3W_TR (default 1): the 256x256 transposed-read weight-gradient kernel
// for GEMMs with K, N >= 192; 0 keeps the 128x128 x3_wgrad_kernel everywhere.
static int wgrad_tr_env() {
    static constexpr int v = M3D_TUNE_X3W_TR;
    return v;
}

static void launch_wgrad_tr(const float* A, const float* Bm, float* C, int64_t M, int K, int N, int nbatch,
                            int64_t bsa, int64_t bsb, int64_t bsc, hipStream_t s) {
    const int64_t tiles = (int64_t)((K + 255) / 256) * ((N + 255) / 256) * nbatch;
    const int64_t cus = num_cus();
    static constexpr int64_t minm = M3D_TUNE_X3W_TR_MINM;
    if (M3D_TUNE_X3W_SK && !det().on && M >= (int64_t)M3D_TUNE_X3W_SK_MIN_STEPS * W2_BK) {
        // stream-K (X3wSK): one balanced round of workgroups, each >= minm rows
        // (only for tiles of >= 32 steps: with short tiles the minm floor would
        // give one workgroup a run of tiles, each with its own atomic epilogue)
        X3wSK sk{};
        sk.nk = (int)((M + W2_BK - 1) / W2_BK);
        sk.tk = (K + 255) / 256;
        sk.tn = (N + 255) / 256;
        sk.units = tiles * sk.nk;
        const int64_t min_steps = (minm + W2_BK - 1) / W2_BK;
        int64_t G = (sk.units + min_steps - 1) / min_steps;
        if (G > cus) G = cus;
        G = G / sk.tn * sk.tn;                        // whole groups of the tn column tiles
        if (G < sk.tn) G = sk.tn;
        hipLaunchKernelGGL((x3_wgrad_tr_kernel<0, true>), dim3((unsigned)G), dim3(512), 0, s, A, Bm, C, M, K, N,
                           (int64_t)0, bsa, bsb, bsc, WgOut{nullptr, 0, 0}, sk);
        return;
    }
    int64_t splits = (cus + tiles - 1) / tiles;
    // M3D_X3W_TR_MINM: fewest m rows per workgroup.  Every split adds a 256x256
    // fp32 atomic epilogue: the small-m 1x1x1 gradients of res4 / res5 (m = 8192
    // / 2048 at 128^3, 4 output tiles) split 64 ways at the old floor of 64 rows,
    // and their 16.7 M atomics per launch slowed the data-gradient stream beside
    // them.  256: 128^3 step 28.73 -> 27.8 ms (scripts/gpu_wgrad1b.sh, wg1c/d A/B:
    // 256 / 384 / 512 equal within noise, 1024 28.2-28.5 ms); alone 73 -> 64 us.
    const int64_t max_splits = (M + minm - 1) / minm;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    const WgOut wo = wg_out(splits, nbatch, K, N);
    int64_t mper = (M + splits - 1) / splits;
    mper = (mper + W2_BK - 1) / W2_BK * W2_BK;
    splits = (M + mper - 1) / mper;
    dim3 grid((unsigned)((K + 255) / 256), (unsigned)((N + 255) / 256), (unsigned)(splits * nbatch));
    hipLaunchKernelGGL(x3_wgrad_tr_kernel<0>, grid, dim3(512), 0, s, A, Bm, C, M, K, N, mper, bsa, bsb, bsc, wo,
                       X3wSK{});
    wg_finish(wo, splits, nbatch, K, N, bsc, C, s);
}

// M3D_GEMM_X3 bit 2: the batched Winograd weight-gradient GEMMs on x3_wgrad_kernel
static int wgrad_x3_env() { return (x3_mask() >> 2) & 1; }

// C[b] += A[b]^T B[b]: A [M][K], B [M][N], C [K][N], batch strides bsa/bsb/bsc
static void launch_wgrad_x3(const float* A, const float* Bm, float* C, int64_t M, int K, int N, int nbatch,
                            int64_t bsa, int64_t bsb, int64_t bsc, hipStream_t s) {
    if (wgrad_tr_env() && K >= 192 && N >= 192) {
        launch_wgrad_tr(A, Bm, C, M, K, N, nbatch, bsa, bsb, bsc, s);
        return;
    }
    if (K <= 64 || N <= 64) {          // x3_wgrad64_kernel: 64x64 tiles, the m chunk over the waves
        const int64_t tiles = (int64_t)((K + 63) / 64) * ((N + 63) / 64);
        int64_t splits = (1024 + tiles * nbatch - 1) / (tiles * nbatch);
        const int64_t minm = wgrad_minm_env() > 64 ? wgrad_minm_env() : 64;
        const int64_t max_splits = (M + minm - 1) / minm;
        if (splits > max_splits) splits = max_splits;
        if (splits < 1) splits = 1;
        const WgOut wo = wg_out(splits, nbatch, K, N);
        int64_t mper = (M + splits - 1) / splits;
        mper = (mper + 63) / 64 * 64;
        splits = (M + mper - 1) / mper;
        hipLaunchKernelGGL((x3_wgrad64_kernel<2>), dim3((unsigned)(tiles * splits * nbatch)), dim3(256), 0, s, A, Bm, C, M,
                           K, N, mper, bsa, bsb, bsc, wo);
        wg_finish(wo, splits, nbatch, K, N, bsc, C, s);
        return;
    }
    const int64_t tiles = (int64_t)((K + 127) / 128) * ((N + 127) / 128) * nbatch;
    int64_t splits = (1024 + tiles - 1) / tiles;
    const int64_t minm = wgrad_minm_env() > 32 ? wgrad_minm_env() : 32;
    const int64_t max_splits = (M + minm - 1) / minm;
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    const WgOut wo = wg_out(splits, nbatch, K, N);
    int64_t mper = (M + splits - 1) / splits;
    mper = (mper + 31) / 32 * 32;
    splits = (M + mper - 1) / mper;
    dim3 grid((unsigned)((K + 127) / 128), (unsigned)((N + 127) / 128), (unsigned)(splits * nbatch));
    // 2 blocks/CU (3 at 164 VGPRs: faster alone, step unchanged)
    hipLaunchKernelGGL((x3_wgrad_kernel<2>), grid, dim3(256), 0, s, A, Bm, C, M, K, N, mper, bsa, bsb, bsc, wo);
    wg_finish(wo, splits, nbatch, K, N, bsc, C, s);
}

// =========================================================================
// Winograd F(NYx2xNZ, 3x3x3) for stride-1 'same' 3x3x3 convs: F(NY,3) along y
// (NY = M3D_TUNE_WINO_NY: 4 by default since round 4, 2), F(2,3) along x,
// F(NZ,3) along z (NZ = 2, or 4 by default).  The F(2,3) formulas below are
// written for y and x; with NY = 4 the y axis takes the F(4,3) ones (ZT<4>).
//   fwd:   Y   = A^T [ (G W G^T) . (B^T X B) ] A        (per 2x2xNZ output tile)
//   dgrad: dX  = same with W'[t][n][c] = W[flip t][c][n]
//   wgrad: dW  = G^T [ sum_tiles (B^T X B) . (A dZ A^T) ] G
// 1-D F(2,3), points 0, 1, -1, inf:
//   B^T d = [d0-d2, d1+d2, d2-d1, d1-d3]      G g = [g0, (g0+g1+g2)/2, (g0-g1+g2)/2, g2]
//   A^T m = [m0+m1+m2, m1-m2-m3]              A e = [e0, e0+e1, e0-e1, -e1]
//   G^T v = [v0+(v1+v2)/2, (v1-v2)/2, (v1+v2)/2+v3]
// 1-D F(4,3) along z, points 0, 1, -1, 1/2, -1/2, inf (exact rationals;
// the half-integer points keep the fp32 error at the F(2,3)/direct level --
// measured 4.3e-6 vs 4.6e-6 relative for a 256-channel direct fp32 conv, where
// the integer points +-2 give 1.3x that and F(4,3) on all three axes 15x):
//   B^T d = [d0/4 - 5/4 d2 + d4, -(d1+d2)/4 + d3 + d4, (d1-d2)/4 - d3 + d4,
//            -d1/2 - d2 + d3/2 + d4, d1/2 - d2 - d3/2 + d4, d1/4 - 5/4 d3 + d5]
//   G g   = [4 g0, 2/3 (g0+g1+g2), 2/3 (g0-g1+g2), -8/3 g0 - 4/3 g1 - 2/3 g2,
//            -8/3 g0 + 4/3 g1 - 2/3 g2, g2]
//   A^T m = [m0+m1+m2+m3+m4, m1-m2+(m3-m4)/2, m1+m2+(m3+m4)/4, m1-m2+(m3-m4)/8+m5]
// The 16*(NZ+2) point-wise products (64 or 96) become independent GEMMs (one
// per point xi) run by the same MFMA kernels in batched mode: 27*2*2*NZ /
// (16*(NZ+2)) = 3.375x (NZ=2) or 4.5x (NZ=4) fewer FLOPs than the direct
// implicit GEMM, and the transformed operands are 8x / 6x the tensors they
// come from.  Transformed operands live in a caller workspace, xi-major:
// U[P][T][C], V[P][K][N], M[P][T][N].
// =========================================================================
// Tile grid over the OUTPUT (depth D); the transformed input is read from a
// tensor of depth Din at z = NZ*tz - pz + k ('same': Din = D, pz = 1; a depth
// slab extended by z-halo planes: Din = D + halos, pz = 1 - lower halo).
struct WinoGeom {
    int B, H, W, D, Din, pz, TY, TX, TZ;
    int64_t T;
    // depth-slab halo (wino_input_kernel<.., HALO>): planes z = -1 and z = Din
    // of the slab read from halo [B][H][W][2][C] (plane 0 / 1) when present
    const float* halo;
    int hlo, hhi;
    // z-tile subset of an input-transform launch (depth-slab overlap of the halo
    // exchange): 0 all tiles, 1 interior only (tz in [1, TZ-1): no halo plane in
    // the window), 2 the first / last z tile only
    int tz_mode;
    // XCD-aware block order of the transform kernels (M3D_WINO_XCD=1): the
    // round-robin XCD dispatch gets contiguous tile ranges per XCD, so the
    // windows that overlap neighbouring tiles' stay in one L2
    int xcd;
};

__device__ __forceinline__ int64_t wino_block(const WinoGeom& g) {
    const unsigned nb = gridDim.x, b = blockIdx.x;
    if (g.xcd && (nb & 7u) == 0) return (int64_t)(b & 7u) * (nb >> 3) + (b >> 3);
    return b;
}

__device__ __forceinline__ void bt4(float& a0, float& a1, float& a2, float& a3) {
    const float t0 = a0 - a2, t1 = a1 + a2, t2 = a2 - a1, t3 = a1 - a3;
    a0 = t0; a1 = t1; a2 = t2; a3 = t3;
}
__device__ __forceinline__ void g3(float g0, float g1, float g2, float* o) {
    o[0] = g0;
    o[1] = (g0 + g1 + g2) * 0.5f;
    o[2] = (g0 - g1 + g2) * 0.5f;
    o[3] = g2;
}
__device__ __forceinline__ void at4(float m0, float m1, float m2, float m3, float& o0, float& o1) {
    o0 = m0 + m1 + m2;
    o1 = m1 - m2 - m3;
}
__device__ __forceinline__ void a4(float e0, float e1, float* o) {
    o[0] = e0; o[1] = e0 + e1; o[2] = e0 - e1; o[3] = -e1;
}
__device__ __forceinline__ void gt4(float v0, float v1, float v2, float v3, float* o) {
    o[0] = v0 + (v1 + v2) * 0.5f;
    o[1] = (v1 - v2) * 0.5f;
    o[2] = (v1 + v2) * 0.5f + v3;
}

// The transformed operands (U, DY: 6-8x the tensor they come from) are
// written once and read once by the point GEMMs, and M is read once by the
// output transform: non-temporal, so the streams do not evict the input tile
// rows that neighbouring tiles re-read (each input element belongs to up to
// 2x2x2 overlapping 4x4xP windows).
__device__ __forceinline__ void wino_st(float* p, float v) {
    __builtin_nontemporal_store(v, p);
}
__device__ __forceinline__ float wino_ld(const float* p) {
    return __builtin_nontemporal_load(p);
}

// z-axis transforms of F(NZ,3): P = NZ + 2 points
template <int NZ> struct ZT;
template <> struct ZT<2> {
    static constexpr int P = 4;
    __device__ static void bt(float* d) { bt4(d[0], d[1], d[2], d[3]); }
    __device__ static void g(const float* w, float* o) { g3(w[0], w[1], w[2], o); }
    __device__ static void at(const float* m, float* o) { at4(m[0], m[1], m[2], m[3], o[0], o[1]); }
    __device__ static void a(const float* e, float* o) { a4(e[0], e[1], o); }
    __device__ static void gt(const float* v, float* o) { gt4(v[0], v[1], v[2], v[3], o); }
};
template <> struct ZT<4> {
    static constexpr int P = 6;
    __device__ static void bt(float* d) {
        const float d0 = d[0], d1 = d[1], d2 = d[2], d3 = d[3], d4 = d[4], d5 = d[5];
        d[0] = d0 * 0.25f - d2 * 1.25f + d4;
        d[1] = -(d1 + d2) * 0.25f + d3 + d4;
        d[2] = (d1 - d2) * 0.25f - d3 + d4;
        d[3] = -d1 * 0.5f - d2 + d3 * 0.5f + d4;
        d[4] = d1 * 0.5f - d2 - d3 * 0.5f + d4;
        d[5] = d1 * 0.25f - d3 * 1.25f + d5;
    }
    __device__ static void g(const float* w, float* o) {
        const float c23 = 2.0f / 3.0f;
        o[0] = 4.0f * w[0];
        o[1] = c23 * (w[0] + w[1] + w[2]);
        o[2] = c23 * (w[0] - w[1] + w[2]);
        o[3] = -(8.0f / 3.0f) * w[0] - (4.0f / 3.0f) * w[1] - c23 * w[2];
        o[4] = -(8.0f / 3.0f) * w[0] + (4.0f / 3.0f) * w[1] - c23 * w[2];
        o[5] = w[2];
    }
    __device__ static void at(const float* m, float* o) {
        const float s12 = m[1] + m[2], d12 = m[1] - m[2], s34 = m[3] + m[4], d34 = m[3] - m[4];
        o[0] = m[0] + s12 + s34;
        o[1] = d12 + d34 * 0.5f;
        o[2] = s12 + s34 * 0.25f;
        o[3] = d12 + d34 * 0.125f + m[5];
    }
    // A = (A^T)^T: e [4] -> 6
    __device__ static void a(const float* e, float* o) {
        o[0] = e[0];
        o[1] = e[0] + e[1] + e[2] + e[3];
        o[2] = e[0] - e[1] + e[2] - e[3];
        o[3] = e[0] + e[1] * 0.5f + e[2] * 0.25f + e[3] * 0.125f;
        o[4] = e[0] - e[1] * 0.5f + e[2] * 0.25f - e[3] * 0.125f;
        o[5] = e[3];
    }
    // G^T: v [6] -> 3
    __device__ static void gt(const float* v, float* o) {
        const float c23 = 2.0f / 3.0f;
        o[0] = 4.0f * v[0] + c23 * (v[1] + v[2]) - (8.0f / 3.0f) * (v[3] + v[4]);
        o[1] = c23 * (v[1] - v[2]) - (4.0f / 3.0f) * (v[3] - v[4]);
        o[2] = c23 * (v[1] + v[2]) - c23 * (v[3] + v[4]) + v[5];
    }
};

// y-axis transforms: F(WNY,3) -- 2: F(2,3) as on x; 4: F(4,3) as on z (a 4x2xNZ
// output tile: 4.5 instead of 6 points per output for NZ = 4, at a larger
// rounding amplification; M3D_TUNE_WINO_NY)
constexpr int WNY = M3D_TUNE_WINO_NY;
using YT = ZT<WNY>;
constexpr int PY = YT::P;

__device__ __forceinline__ void tile_coords(int64_t t, const WinoGeom& g, int& b, int& ty, int& tx,
                                            int& tz) {
    tz = (int)(t % g.TZ);
    int64_t r = t / g.TZ;
    tx = (int)(r % g.TX);
    r /= g.TX;
    ty = (int)(r % g.TY);
    b = (int)(r / g.TY);
}

// U[xi][t][c] = (B^T (x) B^T (x) Bz^T) d, d = the 4x4xP input tile at
// (2ty-1, 2tx-1, NZ*tz-pz); xi = (a*4 + b)*P + k.
// X3O: U is written as the three bf16 planes of split3 (uint16 [3][points][T][C])
// for x3_gemm_kernel -- the split is done once here, not per GEMM k-tile.
template <int NZ, bool X3O = false, bool HALO = false, int NYT = WNY>
__global__ __launch_bounds__(256) void wino_input_kernel(const float* __restrict__ x, WinoGeom g,
                                                         int C, float* __restrict__ U) {
    constexpr int P = ZT<NZ>::P, PYt = ZT<NYT>::P;
    const int64_t i = wino_block(g) * blockDim.x + threadIdx.x;
    if (i >= g.T * C) return;
    const int c = (int)(i % C);
    const int64_t t = i / C;
    int b, ty, tx, tz;
    tile_coords(t, g, b, ty, tx, tz);
    if (g.tz_mode) {
        const bool edge = tz == 0 || tz == g.TZ - 1;
        if ((g.tz_mode == 1) == edge) return;
    }
    float d[PYt][4][P];
    // branch-free window loads: raw buffer loads whose out-of-range offset
    // returns 0 (the zero padding), so all 16*P loads issue back to back
    // (conditional global loads compiled to a branch + wait per element)
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(x, (uint64_t)g.B * g.H * g.W * g.Din * C * 4);
    __amdgpu_buffer_rsrc_t rh;
    if constexpr (HALO) rh = make_rsrc(g.halo, (uint64_t)g.B * g.H * g.W * 2 * C * 4);
#pragma unroll
    for (int a = 0; a < PYt; ++a) {
        const int y = NYT * ty - 1 + a;
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
            const int xx = 2 * tx - 1 + bb;
            const bool ok = (unsigned)y < (unsigned)g.H && (unsigned)xx < (unsigned)g.W;
            const uint32_t row = (uint32_t)((((b * g.H + y) * g.W + xx) * g.Din) * C + c);
#pragma unroll
            for (int k = 0; k < P; ++k) {
                const int z = NZ * tz - g.pz + k;
                const bool in = ok && (unsigned)z < (unsigned)g.Din;
                d[a][bb][k] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(rs, in ? (row + (uint32_t)z * C) * 4u : M3D_OOB, 0, 0));
                if constexpr (HALO) {
                    // only the first / last window planes can reach a neighbour's plane
                    if (k == 0 || k == P - 1) {
                        const int q = z < 0 ? 0 : 1;
                        const bool hz = ok && ((z == -1 && g.hlo) || (z == g.Din && g.hhi));
                        const uint32_t hoff = (uint32_t)((((b * g.H + y) * g.W + xx) * 2 + q) * C + c) * 4u;
                        const float hv = __builtin_bit_cast(
                            float, __builtin_amdgcn_raw_buffer_load_b32(rh, hz ? hoff : M3D_OOB, 0, 0));
                        d[a][bb][k] = hz ? hv : d[a][bb][k];
                    }
                }
            }
        }
    }
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) ZT<NZ>::bt(d[a][bb]);
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int k = 0; k < P; ++k) bt4(d[a][0][k], d[a][1][k], d[a][2][k], d[a][3][k]);
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float col[PYt];
#pragma unroll
            for (int a = 0; a < PYt; ++a) col[a] = d[a][bb][k];
            ZT<NYT>::bt(col);
#pragma unroll
            for (int a = 0; a < PYt; ++a) d[a][bb][k] = col[a];
        }
    const int64_t stride = g.T * C;
    if constexpr (X3O) {
        unsigned short* o = reinterpret_cast<unsigned short*>(U) + t * C + c;
        const int64_t pstride = (int64_t)PYt * 4 * P * stride;
#pragma unroll
        for (int a = 0; a < PYt; ++a)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                for (int k = 0; k < P; ++k) {
                    uint32_t hh, mm, ll;
                    split3(d[a][bb][k], hh, mm, ll);
                    unsigned short* q = o + (int64_t)((a * 4 + bb) * P + k) * stride;
                    __builtin_nontemporal_store((unsigned short)hh, q);
                    __builtin_nontemporal_store((unsigned short)mm, q + pstride);
                    __builtin_nontemporal_store((unsigned short)ll, q + 2 * pstride);
                }
        return;
    }
    float* o = U + t * C + c;
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int k = 0; k < P; ++k) wino_st(o + (int64_t)((a * 4 + bb) * P + k) * stride, d[a][bb][k]);
}

// V[xi][k'][n'] = (G (x) G (x) Gz) w.  fwd: k'=cin, n'=cout; bwd (transpose_flip):
// k'=cout, n'=cin, w taken at the flipped tap.
// wt[t][n][c] = w[t][c][n] for the 27 taps (32x32 tiles through LDS)
__global__ __launch_bounds__(256) void x3_wt_kernel(const float* __restrict__ w, int C, int N,
                                                    float* __restrict__ wt) {
    __shared__ float tile[32][33];
    const int t = blockIdx.z, c0 = blockIdx.y * 32, n0 = blockIdx.x * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int64_t base = (int64_t)t * C * N;
#pragma unroll
    for (int r = ty; r < 32; r += 8)
        if (c0 + r < C && n0 + tx < N) tile[r][tx] = w[base + (int64_t)(c0 + r) * N + n0 + tx];
    __syncthreads();
#pragma unroll
    for (int r = ty; r < 32; r += 8)
        if (n0 + r < N && c0 + tx < C) wt[base + (int64_t)(n0 + r) * C + c0 + tx] = tile[tx][r];
}

// X3O: V is written as split3 planes, transposed: uint16 [3][points][n'][k'].
template <int NZ, bool X3O = false, int NYT = WNY>
__global__ __launch_bounds__(256) void wino_weight_kernel(const float* __restrict__ w, int Cin,
                                                          int Cout, int transpose_flip,
                                                          float* __restrict__ V) {
    constexpr int P = ZT<NZ>::P, PYt = ZT<NYT>::P;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t KN = (int64_t)Cin * Cout;
    if (i >= KN) return;
    int cin, cout, kp, np_, Np;
    // thread order: the output's contiguous axis fastest (X3O writes [n'][k'])
    const bool cout_fast = X3O ? transpose_flip != 0 : !transpose_flip;
    if (cout_fast) { cout = (int)(i % Cout); cin = (int)(i / Cout); }
    else { cin = (int)(i % Cin); cout = (int)(i / Cin); }
    if (!transpose_flip) { kp = cin; np_ = cout; Np = Cout; }
    else { kp = cout; np_ = cin; Np = Cin; }
    float gw[3][3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int t = transpose_flip ? ((2 - a) * 3 + (2 - b)) * 3 + (2 - k) : (a * 3 + b) * 3 + k;
                // X3O forward: w arrives transposed ([27][Cout][Cin], x3_wt_kernel) so
                // the cin-fastest lanes read it coalesced
                gw[a][b][k] = (X3O && !transpose_flip) ? w[(int64_t)t * KN + (int64_t)cout * Cin + cin]
                                                       : w[(int64_t)t * KN + (int64_t)cin * Cout + cout];
            }
    float t1[3][3][P];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) ZT<NZ>::g(gw[a][b], t1[a][b]);
    float t2[3][4][P];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float o[4];
            g3(t1[a][0][k], t1[a][1][k], t1[a][2][k], o);
#pragma unroll
            for (int b = 0; b < 4; ++b) t2[a][b][k] = o[b];
        }
    if constexpr (X3O) {
        unsigned short* out = reinterpret_cast<unsigned short*>(V) + (int64_t)np_ * (KN / Np) + kp;
        const int64_t pstride = (int64_t)PYt * 4 * P * KN;
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int k = 0; k < P; ++k) {
                float o[PYt];
                const float gy[3] = {t2[0][b][k], t2[1][b][k], t2[2][b][k]};
                ZT<NYT>::g(gy, o);
#pragma unroll
                for (int a = 0; a < PYt; ++a) {
                    uint32_t hh, mm, ll;
                    split3(o[a], hh, mm, ll);
                    unsigned short* q = out + (int64_t)((a * 4 + b) * P + k) * KN;
                    q[0] = (unsigned short)hh;
                    q[pstride] = (unsigned short)mm;
                    q[2 * pstride] = (unsigned short)ll;
                }
            }
        return;
    }
    float* out = V + (int64_t)kp * Np + np_;
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float o[PYt];
            const float gy[3] = {t2[0][b][k], t2[1][b][k], t2[2][b][k]};
            ZT<NYT>::g(gy, o);
#pragma unroll
            for (int a = 0; a < PYt; ++a) out[(int64_t)((a * 4 + b) * P + k) * KN] = o[a];
        }
}

// Y tile (2x2xNZ) = (A^T (x) A^T (x) Az^T) M[.][t][n], then the conv epilogue.
template <int NZ, bool HALO, int NYT>
__device__ __forceinline__ void wino_output_body(const float* __restrict__ Mt, const WinoGeom& g,
                                                 int N, const Epi& e);
template <int NZ, int NYT = WNY>
__global__ __launch_bounds__(256) void wino_output_kernel(const float* __restrict__ Mt, WinoGeom g,
                                                          int N, Epi e) {
    wino_output_body<NZ, false, NYT>(Mt, g, N, e);
}
// depth-slab data gradient: interior planes into e.y, halo planes into e.yh
template <int NZ, int NYT = WNY>
__global__ __launch_bounds__(256) void wino_output_halo_kernel(const float* __restrict__ Mt, WinoGeom g,
                                                               int N, Epi e) {
    wino_output_body<NZ, true, NYT>(Mt, g, N, e);
}

template <int NZ, bool HALO, int NYT>
__device__ __forceinline__ void wino_output_body(const float* __restrict__ Mt, const WinoGeom& g,
                                                 int N, const Epi& e) {
    constexpr int P = ZT<NZ>::P, PYt = ZT<NYT>::P;
    const int64_t i = wino_block(g) * blockDim.x + threadIdx.x;
    if (i >= g.T * N) return;
    const int n = (int)(i % N);
    const int64_t t = i / N;
    int b, ty, tx, tz;
    tile_coords(t, g, b, ty, tx, tz);
    const int64_t stride = g.T * N;
    const float* src = Mt + t * N + n;
    float m[PYt][4][P];
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb)
#pragma unroll
            for (int k = 0; k < P; ++k) m[a][bb][k] = wino_ld(src + (int64_t)((a * 4 + bb) * P + k) * stride);
    float r1[PYt][4][NZ];
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) ZT<NZ>::at(m[a][bb], r1[a][bb]);
    float r2[PYt][2][NZ];
#pragma unroll
    for (int a = 0; a < PYt; ++a)
#pragma unroll
        for (int k = 0; k < NZ; ++k)
            at4(r1[a][0][k], r1[a][1][k], r1[a][2][k], r1[a][3][k], r2[a][0][k], r2[a][1][k]);
    float o[NYT][2][NZ];
#pragma unroll
    for (int bb = 0; bb < 2; ++bb)
#pragma unroll
        for (int k = 0; k < NZ; ++k) {
            float col[PYt], oy[NYT];
#pragma unroll
            for (int a = 0; a < PYt; ++a) col[a] = r2[a][bb][k];
            ZT<NYT>::at(col, oy);
#pragma unroll
            for (int a = 0; a < NYT; ++a) o[a][bb][k] = oy[a];
        }
    const float bias = e.bias ? e.bias[n] : 0.0f;
    const float sc = e.scale ? e.scale[n] : 1.0f, sh = e.scale ? e.shift[n] : 0.0f;
#pragma unroll
    for (int a = 0; a < NYT; ++a) {
        const int y = NYT * ty + a;
        if (y >= g.H) continue;
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) {
            const int xx = 2 * tx + bb;
            if (xx >= g.W) continue;
#pragma unroll
            for (int k = 0; k < NZ; ++k) {
                const int z = NZ * tz + k;
                if (z >= g.D) continue;
                const int64_t col = ((int64_t)b * g.H + y) * g.W + xx;
                if constexpr (HALO) {
                    const int zi = z - e.hlo;
                    if (zi < 0 || zi >= e.dl) {          // a neighbour's plane: its gradient, fresh
                        e.yh[(col * 2 + (zi < 0 ? 0 : 1)) * N + n] = o[a][bb][k];
                        continue;
                    }
                    float* dst = e.y + (col * e.dl + zi) * e.ldy + n;
                    const float v = o[a][bb][k];
                    *dst = e.accumulate ? v + *dst : v;
                    continue;
                }
                const int64_t row = col * g.D + z;
                float v = o[a][bb][k];
                if (e.bias) v += bias;
                if (e.z) e.z[row * N + n] = v;
                if (e.scale) v = v * sc + sh;
                if (e.res_mode == 1) v += e.res[row * e.ldy + n];
                if (e.relu) v = v > 0.0f ? v : 0.0f;
                float* dst = e.y + row * e.ldy + n;
                if (e.accumulate) v += *dst;
                *dst = v;
            }
        }
    }
}

// The data-gradient output transform with the fused BN-ReLU backward of the
// unit whose output dx is (m3d_conv3d_bwd_data_wino_bn): per element of dx
// (after accumulate) bn_act_bwd_kernel's maths -- dz into dx, dpre into fdres
// -- and per-block channel sums, one partial row per 256 (tile, channel)
// pairs: N < 256 (256 % N == 0): the block's 256 / N tiles, row = block;
// N % 256 == 0: one tile's 256 channels, row = tile.
template <int NZ, int NYT = WNY>
__global__ __launch_bounds__(256) void wino_output_bn_kernel(const float* __restrict__ Mt, WinoGeom g, int N,
                                                             Epi e) {
    constexpr int P = ZT<NZ>::P, PYt = ZT<NYT>::P;
    const int tid = threadIdx.x;
    const int64_t i = (int64_t)blockIdx.x * 256 + tid;
    const bool valid = i < g.T * N;
    const int n = (int)(i % N);
    const int64_t t = i / N;
    float sp = 0.f, sx = 0.f, sz = 0.f;
    if (valid) {
        int b, ty, tx, tz;
        tile_coords(t, g, b, ty, tx, tz);
        const int64_t stride = g.T * N;
        const float* src = Mt + t * N + n;
        float m[PYt][4][P];
#pragma unroll
        for (int a = 0; a < PYt; ++a)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb)
#pragma unroll
                for (int k = 0; k < P; ++k) m[a][bb][k] = wino_ld(src + (int64_t)((a * 4 + bb) * P + k) * stride);
        float r1[PYt][4][NZ];
#pragma unroll
        for (int a = 0; a < PYt; ++a)
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) ZT<NZ>::at(m[a][bb], r1[a][bb]);
        float r2[PYt][2][NZ];
#pragma unroll
        for (int a = 0; a < PYt; ++a)
#pragma unroll
            for (int k = 0; k < NZ; ++k)
                at4(r1[a][0][k], r1[a][1][k], r1[a][2][k], r1[a][3][k], r2[a][0][k], r2[a][1][k]);
        float o[NYT][2][NZ];
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int k = 0; k < NZ; ++k) {
                float col[PYt], oy[NYT];
#pragma unroll
                for (int a = 0; a < PYt; ++a) col[a] = r2[a][bb][k];
                ZT<NYT>::at(col, oy);
#pragma unroll
                for (int a = 0; a < NYT; ++a) o[a][bb][k] = oy[a];
            }
        const float sc = e.fscale ? e.fscale[n] : 1.0f;
        const float mu = e.fz ? e.fmean[n] : 0.0f, rs = e.fz ? e.frstd[n] : 1.0f;
        // per output row pair a: its loads (old dx, y, z) before its stores -- a load
        // issued after a store to a possibly aliasing address waits for it -- in two
        // halves, so only 2 x 2 x NZ x 3 loaded values are live beside o
        const int64_t ostr = (int64_t)g.D * e.ldy;             // output x step
        const int64_t obase = ((((int64_t)b * g.H + NYT * ty) * g.W + 2 * tx) * g.D + NZ * tz) * e.ldy + n;
#pragma unroll
        for (int a = 0; a < NYT; ++a) {
            float ov[2][NZ], yv[2][NZ], zv[2][NZ];
            bool in[2][NZ];
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int k = 0; k < NZ; ++k) {
                    in[bb][k] = NYT * ty + a < g.H && 2 * tx + bb < g.W && NZ * tz + k < g.D;
                    const int64_t off = obase + (a * (int64_t)g.W + bb) * ostr + k * e.ldy;
                    ov[bb][k] = in[bb][k] && e.accumulate ? e.y[off] : 0.0f;
                    yv[bb][k] = in[bb][k] && e.frelu ? e.fy[off] : 1.0f;
                    zv[bb][k] = in[bb][k] && e.fz ? e.fz[off] : 0.0f;
                }
#pragma unroll
            for (int bb = 0; bb < 2; ++bb)
#pragma unroll
                for (int k = 0; k < NZ; ++k) {
                    if (!in[bb][k]) continue;
                    const int64_t off = obase + (a * (int64_t)g.W + bb) * ostr + k * e.ldy;
                    float gv = o[a][bb][k];
                    if (e.accumulate) gv += ov[bb][k];
                    if (e.frelu && !(yv[bb][k] > 0.f)) gv = 0.f;
                    const float d = gv * sc;
                    sp += gv;
                    sx += gv * ((zv[bb][k] - mu) * rs);
                    sz += d;
                    e.y[off] = d;
                    if (e.fdres) e.fdres[off] = gv;
                }
        }
    }
    if (!e.fpart) return;                        // (block-uniform)
    if (N % 256 == 0) {
        if (valid) {
            e.fpart[(0 * e.fprows + t) * N + n] = sp;
            e.fpart[(1 * e.fprows + t) * N + n] = sx;
            e.fpart[(2 * e.fprows + t) * N + n] = sz;
        }
        return;
    }
    __shared__ float red[3][256];
    red[0][tid] = sp;
    red[1][tid] = sx;
    red[2][tid] = sz;
    __syncthreads();
    if (tid < N) {
        float a0 = 0.f, a1 = 0.f, a2 = 0.f;
        for (int q = tid; q < 256; q += N) {
            a0 += red[0][q];
            a1 += red[1][q];
            a2 += red[2][q];
        }
        const int64_t row = blockIdx.x;
        e.fpart[(0 * e.fprows + row) * N + tid] = a0;
        e.fpart[(1 * e.fprows + row) * N + tid] = a1;
        e.fpart[(2 * e.fprows + row) * N + tid] = a2;
    }
}

// DY[xi][t][n] = (A (x) A (x) Az) e, e = the 2x2xNZ output-gradient tile (0 outside).
template <int NZ>
__global__ __launch_bounds__(256) void wino_grad_kernel(const float* __restrict__ dz, WinoGeom g,
                                                        int N, float* __restrict__ DY) {
    constexpr int P = ZT<NZ>::P;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.T * N) return;
    const int n = (int)(i % N);
    const int64_t t = i / N;
    int b, ty, tx, tz;
    tile_coords(t, g, b, ty, tx, tz);
    float ev[WNY][2][NZ];
#pragma unroll
    for (int a = 0; a < WNY; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb)
#pragma unroll
            for (int k = 0; k < NZ; ++k) {
                const int y = WNY * ty + a, xx = 2 * tx + bb, z = NZ * tz + k;
                ev[a][bb][k] = (y < g.H && xx < g.W && z < g.D)
                                   ? dz[((((int64_t)b * g.H + y) * g.W + xx) * g.D + z) * N + n]
                                   : 0.0f;
            }
    float t1[WNY][2][P];
#pragma unroll
    for (int a = 0; a < WNY; ++a)
#pragma unroll
        for (int bb = 0; bb < 2; ++bb) ZT<NZ>::a(ev[a][bb], t1[a][bb]);
    float t2[WNY][4][P];
#pragma unroll
    for (int a = 0; a < WNY; ++a)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float o[4];
            a4(t1[a][0][k], t1[a][1][k], o);
#pragma unroll
            for (int bb = 0; bb < 4; ++bb) t2[a][bb][k] = o[bb];
        }
    const int64_t stride = g.T * N;
    float* out = DY + t * N + n;
#pragma unroll
    for (int bb = 0; bb < 4; ++bb)
#pragma unroll
        for (int k = 0; k < P; ++k) {
            float ey[WNY], o[PY];
#pragma unroll
            for (int a = 0; a < WNY; ++a) ey[a] = t2[a][bb][k];
            YT::a(ey, o);
#pragma unroll
            for (int a = 0; a < PY; ++a) wino_st(out + (int64_t)((a * 4 + bb) * P + k) * stride, o[a]);
        }
}

// dW[t][c][n] += (G^T (x) G^T (x) Gz^T) dWh[.][c][n]
template <int NZ>
__global__ __launch_bounds__(256) void wino_wgrad_out_kernel(const float* __restrict__ dWh, int C,
                                                             int N, float* __restrict__ dw) {
    constexpr int P = ZT<NZ>::P;
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t CN = (int64_t)C * N;
    if (i >= CN) return;
    float v[PY][4][P];
#pragma unroll
    for (int a = 0; a < PY; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
            for (int k = 0; k < P; ++k) v[a][b][k] = dWh[(int64_t)((a * 4 + b) * P + k) * CN + i];
    float t1[PY][4][3];
#pragma unroll
    for (int a = 0; a < PY; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) ZT<NZ>::gt(v[a][b], t1[a][b]);
    float t2[PY][3][3];
#pragma unroll
    for (int a = 0; a < PY; ++a)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float o[3];
            gt4(t1[a][0][k], t1[a][1][k], t1[a][2][k], t1[a][3][k], o);
#pragma unroll
            for (int b = 0; b < 3; ++b) t2[a][b][k] = o[b];
        }
#pragma unroll
    for (int b = 0; b < 3; ++b)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            float vy[PY], o[3];
#pragma unroll
            for (int a = 0; a < PY; ++a) vy[a] = t2[a][b][k];
            YT::gt(vy, o);
#pragma unroll
            for (int a = 0; a < 3; ++a) dw[(int64_t)((a * 3 + b) * 3 + k) * CN + i] += o[a];
        }
}

// ---- batched fp32 GEMM on pre-split operands (Winograd point GEMMs) ------
// C[b][m][n] = sum_k A[b][m][k] B[b][n][k]; A and B are the three bf16 planes
// of split3 (uint16 [3][batch][rows][K], k contiguous, written by the X3O
// transforms), C fp32 [batch][M][N].  128x128 tiles, 32-deep k-tiles staged
// through one swizzled LDS stage (x3_off) with the next k-tile's 16-byte
// chunks in flight in registers; 6 bf16 MFMAs per product (see split3).
// PERSIST: a resident grid loops over all tiles of all batches (XCD-
// contiguous order, as conv_gemm_kernel).
// conv epilogue applied by x3_gemm256_af_kernel to its tile (a 1x1x1 conv's
// GEMM, nbatch 1, rows = voxels, ld = N): epi_store4's operations per element
// in its order -- + bias, z store, * scale + shift, + same-shape residual,
// activation -- so the fused form is bit-identical to the GEMM + epilogue pass
struct X3Epi {
    const float* bias = nullptr;
    const float* scale = nullptr;
    const float* shift = nullptr;
    const float* res = nullptr;   // [M][N] (res_mode 1) or nullptr
    float* z = nullptr;           // pre-BN output or nullptr
    int act = 0;                  // act() code
    int on = 0;                    // 0: plain C store, 1: the forward conv epilogue above, 2: the fused
                               // BN-ReLU backward below (a 1x1x1 conv's data gradient)
    // on == 2: epi_bnbwd4's maths per element of the data gradient g (accumulate 0):
    // g masked by y > 0 (frelu), dz = g * fscale into C, g into fdres, and the channel
    // sums (g, g * (fz - fmean) * frstd, dz) of each 128-row half tile into fpart row
    // 2 * (m0 / 256) + (wave row)
    const float* fy = nullptr;
    const float* fz = nullptr;
    const float* fscale = nullptr;
    const float* fmean = nullptr;
    const float* frstd = nullptr;
    float* fdres = nullptr;
    float* fpart = nullptr;
    int64_t fprows = 0;
    int frelu = 0;
    int facc = 0;                 // on == 2: the gradient is accumulator + C (C holds the parked gradient)
};

struct X3G {
    // default member initialisers: a descriptor declared without an initialiser
    // is still all-zero (round 5: an uninitialised ep.on ran the fused epilogue
    // on garbage and faulted; tests/test_sanitizers.py checks the declarations)
    const unsigned short* a = nullptr;
    const float* af = nullptr;    // AF32: A as fp32 [batch][M][K], split in the LDS store
    const unsigned short* b = nullptr;
    float* c = nullptr;
    int64_t M = 0;
    int K = 0, N = 0, nbatch = 0;
    int64_t psa = 0, psb = 0;     // plane strides (elements)
    int64_t bsa = 0, bsb = 0, bsc = 0;   // batch strides (elements)
    X3Epi ep = {};                // x3_gemm256_af_kernel only (zero: the plain C store)
};

// byte offset of (row, chunk) in a 16-deep X3 plane: 32-B rows of two 16-B
// chunks, the chunk flipped for rows 8..15 of each 16-row group, so a 16-lane
// ds_read_b128 phase over 16 consecutive rows covers the 64 banks once
__device__ __forceinline__ int x3_off16(int row, int kc) {
    return row * 32 + (((kc ^ (row >> 3)) & 1) << 4);
}

// BK 16: two LDS stages (one barrier per k-tile), 3 blocks/CU; BK 32: one
// stage (two barriers per k-tile), 2 blocks/CU.
template <int BK>
__device__ __forceinline__ int x3_soff(int row, int kc) {
    if constexpr (BK == 16) return x3_off16(row, kc);
    else return x3_off(row, kc * 8);
}

// BNT 64: 128x64 tiles for N = 64 (the res2 64-channel Winograd layers; a
// 128-column tile would multiply 64 columns of zeros), each wave 64 x 32.
template <int BK, bool PERSIST, int OCC = (BK == 16 ? 3 : 2), bool AF32 = false, int BNT = 128>
__global__ __launch_bounds__(256, OCC) void x3_gemm_kernel(X3G g) {
    static_assert(BK == 16 || BK == 32, "BK");
    static_assert(BNT == 128 || BNT == 64, "BNT");
    constexpr int BM = 128, BN = BNT, TM = 2, TN = BNT / 64;
    constexpr int NBUF = BK == 16 ? 2 : 1;
    constexpr int KCH = BK / 8, CPT = BM * KCH / 256;   // 16-B chunks per row / per thread and plane
    constexpr int CPTB = BN * KCH / 256;                // the same for B (BN rows)
    constexpr int PLA = BM * BK * 2, PLB = BN * BK * 2;   // bytes per plane
    constexpr int STAGE = 3 * (PLA + PLB);
    constexpr int LDT = BN + 8, HR = 64;                  // epilogue staging (2 row halves)
    static_assert(HR * LDT * 4 <= NBUF * STAGE, "staging fits");
    __shared__ __attribute__((aligned(16))) char smem[NBUF * STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, h = lane >> 5, l32 = lane & 31;
    const int64_t nbx = (g.M + BM - 1) / BM, nby = (g.N + BN - 1) / BN;
    const int64_t per_batch = nbx * nby, total = per_batch * g.nbatch;
    int64_t L = PERSIST ? (int64_t)blockIdx.x : (int64_t)blockIdx.x + (int64_t)gridDim.x * blockIdx.y;
    const int64_t Lstep = PERSIST ? (int64_t)gridDim.x : total;
    const int nk = g.K / BK;
    float* const Ts = reinterpret_cast<float*>(smem);
    int soff[CPT];
    uint32_t lrow[CPT];
#pragma unroll
    for (int u = 0; u < CPT; ++u) {
        const int c = tid + 256 * u;
        soff[u] = x3_soff<BK>(c / KCH, c % KCH);
    }
    for (; L < total; L += Lstep) {
        const int64_t xcd = L % 8, q8 = total / 8, r8 = total % 8;
        const int64_t T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
        const int64_t bz = T / per_batch, Tt = T - bz * per_batch;
        const int64_t m0 = (Tt / nby) * BM;
        const int n0 = (int)(Tt % nby) * BN;
        __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) {
            if constexpr (AF32) {
                if (pl == 0) ra[0] = make_rsrc(g.af + bz * g.bsa + m0 * g.K, (uint64_t)(g.M - m0) * g.K * 4);
            } else {
                ra[pl] = make_rsrc(g.a + pl * g.psa + bz * g.bsa + m0 * g.K, (uint64_t)(g.M - m0) * g.K * 2);
            }
            rb[pl] = make_rsrc(g.b + pl * g.psb + bz * g.bsb + (int64_t)n0 * g.K, (uint64_t)(g.N - n0) * g.K * 2);
        }
#pragma unroll
        for (int u = 0; u < CPT; ++u) {
            const int c = tid + 256 * u;
            lrow[u] = (uint32_t)((c / KCH) * g.K + (c % KCH) * 8) * 2u;
        }
        uint4 va[AF32 ? 1 : 3][CPT], vb[3][CPTB];
        float4 fa[AF32 ? CPT : 1][2];   // AF32: the 8 fp32 k of each A chunk
        auto load = [&](int kt) {
#pragma unroll
            for (int q = 0; q < 3; ++q)
#pragma unroll
                for (int u = 0; u < CPT; ++u) {
                    const int off = (int)(lrow[u] + (uint32_t)kt * (BK * 2));
                    if constexpr (AF32) {
                        if (q == 0) {   // element offset of the chunk = byte offset of its bf16 image / 2
                            fa[u][0] = bload4(ra[0], (uint32_t)off * 2u);
                            fa[u][1] = bload4(ra[0], (uint32_t)off * 2u + 16u);
                        }
                    } else {
                        va[q][u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(ra[q], off, 0, 0));
                    }
                    if (u < CPTB)
                        vb[q][u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rb[q], off, 0, 0));
                }
        };
        auto store = [&](int buf) {
            char* As = smem + buf * STAGE;
            char* Bs = As + 3 * PLA;
#pragma unroll
            for (int u = 0; u < CPT; ++u) {
                if constexpr (AF32) {
                    uint2 lo4[3], hi4[3];
                    split3x4(fa[u][0], lo4);
                    split3x4(fa[u][1], hi4);
#pragma unroll
                    for (int q = 0; q < 3; ++q)
                        *reinterpret_cast<uint4*>(As + q * PLA + soff[u]) =
                            make_uint4(lo4[q].x, lo4[q].y, hi4[q].x, hi4[q].y);
                } else {
#pragma unroll
                    for (int q = 0; q < 3; ++q) *reinterpret_cast<uint4*>(As + q * PLA + soff[u]) = va[q][u];
                }
                if (u < CPTB) {
#pragma unroll
                    for (int q = 0; q < 3; ++q) *reinterpret_cast<uint4*>(Bs + q * PLB + soff[u]) = vb[q][u];
                }
            }
        };
        floatx16 acc[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int j = 0; j < TN; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
        load(0);
        store(0);
        __syncthreads();
        for (int kt = 0; kt < nk; ++kt) {
            if (kt + 1 < nk) load(kt + 1);
            const char* As = smem + (NBUF == 2 ? (kt & 1) : 0) * STAGE;
            const char* Bs = As + 3 * PLA;
#pragma unroll BK / 16
            for (int s16 = 0; s16 < BK / 16; ++s16) {
                // lane (l32, h): row l32 of its 32-row blocks, k = 16 s16 + 8h .. +7
                bf16x8 af[TM][3], bfr[TN][3];
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    const int off = x3_soff<BK>(wm * TM * 32 + i * 32 + l32, 2 * s16 + h);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) af[i][pl] = *reinterpret_cast<const bf16x8*>(As + pl * PLA + off);
                }
#pragma unroll
                for (int j = 0; j < TN; ++j) {
                    const int off = x3_soff<BK>(wn * TN * 32 + j * 32 + l32, 2 * s16 + h);
#pragma unroll
                    for (int pl = 0; pl < 3; ++pl) bfr[j][pl] = *reinterpret_cast<const bf16x8*>(Bs + pl * PLB + off);
                }
                // small terms first: (lo,hi) (mid,mid) (hi,lo) (mid,hi) (hi,mid) (hi,hi)
                x3_mac_tiles<TM, TN>(acc, af, bfr);
            }
            if constexpr (NBUF == 2) {
                // the other stage was last read in iteration kt-1, before its closing barrier
                if (kt + 1 < nk) store((kt + 1) & 1);
                __syncthreads();
            } else {
                __syncthreads();
                if (kt + 1 < nk) {
                    store(0);
                    __syncthreads();
                }
            }
        }
        // epilogue: two 64-row halves staged through LDS, float4 row stores
        float* const cb = g.c + bz * g.bsc;
        for (int hf = 0; hf < 2; ++hf) {
            if (hf) __syncthreads();
            if (wm == hf) {
#pragma unroll
                for (int i = 0; i < TM; ++i)
#pragma unroll
                    for (int j = 0; j < TN; ++j)
#pragma unroll
                        for (int r = 0; r < 16; ++r)
                            Ts[(i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h) * LDT + wn * TN * 32 + j * 32 + l32] =
                                acc[i][j][r];
            }
            __syncthreads();
#pragma unroll
            for (int q = 0; q < HR * (BN / 4) / 256; ++q) {
                const int idx = tid + 256 * q;
                const int row = idx / (BN / 4), c4 = idx % (BN / 4);
                const int64_t m = m0 + hf * HR + row;
                const int n = n0 + c4 * 4;
                if (m < g.M && n < g.N)
                    st4(cb + m * g.N + n, *reinterpret_cast<const float4*>(Ts + row * LDT + c4 * 4));
            }
        }
        __syncthreads();
    }
}

// ---- the same batched GEMM, 256x256 tiles, LDS-DMA staged -------------------
// C[b][m][n] = sum_k A[b][m][k] B[b][n][k] on the pre-split planes (as
// x3_gemm_kernel).  512 threads = 8 waves (2 x 4; 128 x 64 outputs = 4 x 2
// 32x32 blocks per wave), one workgroup per CU.  A stage is 16 k of all six
// planes (3 of A, 3 of B; 256 rows x 32 B = 8 KB each, 48 KB): every wave
// moves 32 rows of each plane with one buffer_load_dwordx4 ... lds (1 KB,
// written lane-linearly), so the conflict-free x3_off16 swizzle of the image
// (chunk flipped for rows 8..15 of each 16) goes on the SOURCE address.  Three
// LDS stages: the loads of step t+2 are issued right after the barrier that
// ends step t-1's reads of that stage, and stay in flight across the next
// barrier -- a counted vmcnt(6) retires exactly step t's DMA before the
// barrier that precedes its reads (raw s_barrier: __syncthreads() would emit a
// vmcnt(0) and drain the prefetch).  No VGPR staging, no VALU in the loop.
constexpr int G2_BK = 16;
constexpr int G2_PL = 256 * G2_BK * 2;   // one plane of one operand: 8 KB
constexpr int G2_STAGE = 6 * G2_PL;      // 48 KB
constexpr int G2_NST = 3;

__device__ __forceinline__ void g2_dma(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff,
                                             0, 0, 0);
}

// DBG (timing probes, M3D_X3_256_DBG): 1 no epilogue stores, 2 no MFMAs,
// 3 no DMA (MFMAs on stale stages), 4 neither MFMAs nor stores (DMA only)
template <int DBG>
__global__ __launch_bounds__(512, 1) void x3_gemm256_kernel(X3G g) {
    __shared__ __attribute__((aligned(16))) char smem[G2_NST * G2_STAGE];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3, h = lane >> 5, l32 = lane & 31;
    const int64_t nbx = (g.M + 255) / 256, nby = g.N / 256;
    const int64_t per_batch = nbx * nby, total = per_batch * g.nbatch;
    const int64_t L = (int64_t)blockIdx.x + (int64_t)gridDim.x * blockIdx.y;
    if (L >= total) return;
    const int64_t xcd = L % 8, q8 = total / 8, r8 = total % 8;
    const int64_t T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
    const int64_t bz = T / per_batch, Tt = T - bz * per_batch;
    const int64_t m0 = (Tt / nby) * 256;
    const int64_t n0 = (Tt % nby) * 256;
    // descriptors start at the tile's first row: rows past M read zeros
    __amdgpu_buffer_rsrc_t rs[6];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl) {
        rs[pl] = make_rsrc(g.a + pl * g.psa + bz * g.bsa + m0 * g.K, (uint64_t)(g.M - m0) * g.K * 2);
        rs[3 + pl] = make_rsrc(g.b + pl * g.psb + bz * g.bsb + n0 * g.K, (uint64_t)256 * g.K * 2);
    }
    // loader lane: row 32 wave + lane/2 of every plane, LDS slot lane&1 holds
    // k-chunk (slot ^ row bit 3) -- the x3_off16 image
    const int lrow = 32 * wave + (lane >> 1);
    const uint32_t lsrc = (uint32_t)lrow * (uint32_t)g.K * 2u + (uint32_t)(((lane & 1) ^ ((lrow >> 3) & 1)) << 4);
    const int nk = g.K / G2_BK;
    auto issue = [&](int kt) {
        char* S = smem + (kt % G2_NST) * G2_STAGE + wave * 1024;
        const uint32_t off = lsrc + (uint32_t)kt * (G2_BK * 2);
        if (DBG == 3) return;
#pragma unroll
        for (int pl = 0; pl < 6; ++pl) g2_dma(rs[pl], S + pl * G2_PL, off);
    };
    floatx16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    issue(0);
    if (nk > 1) issue(1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        // stage kt+2 reuses the stage of step kt-1, whose reads all waves
        // finished before the barrier above
        if (kt + 2 < nk) issue(kt + 2);
        const char* S = smem + (kt % G2_NST) * G2_STAGE;
        bf16x8 bfr[2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int off = x3_off16(wn * 64 + j * 32 + l32, h);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                bfr[j][pl] = *reinterpret_cast<const bf16x8*>(S + (3 + pl) * G2_PL + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int off = x3_off16(wm * 128 + i * 32 + l32, h);
            bf16x8 af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) af[pl] = *reinterpret_cast<const bf16x8*>(S + pl * G2_PL + off);
            // small terms first: (lo,hi) (mid,mid) (hi,lo) (mid,hi) (hi,mid) (hi,hi)
            if (DBG == 2 || DBG == 4) {
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j][0] += (float)(af[0][0] ^ af[1][1] ^ af[2][2] ^ bfr[j][0][3] ^ bfr[j][1][4] ^ bfr[j][2][5]);
                continue;
            }
            x3_mac_pair(acc[i][0], acc[i][1], af[0], af[1], af[2], bfr[0][0], bfr[0][1], bfr[0][2],
                                    bfr[1][0], bfr[1][1], bfr[1][2]);
        }
    }
    if (DBG == 1 || DBG == 4) {   // keep the accumulators live, store nothing
        float t = 0.0f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) t += acc[i][j][r];
        if (t == 1.2345f) g.c[0] = t;
        return;
    }
    // epilogue straight from the accumulators: per store instruction two
    // 128-B row segments; rows past M dropped by the descriptor's range
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(g.c + bz * g.bsc + m0 * g.N, (uint64_t)(g.M - m0) * g.N * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = (int)n0 + wn * 64 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                // (a named copy: hipcc 7.2 miscompiles __builtin_bit_cast of a
                // vector-element lvalue into a read of element 0)
                const float v = acc[i][j][r];
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                      (int)(((uint32_t)row * (uint32_t)g.N + (uint32_t)col) * 4u),
                                                      0, 0);
            }
        }
}

// ---- x3_gemm256 with A in fp32 (4 B per point instead of three bf16 planes) --
// The Winograd input transform is the step's largest HBM writer (6 B per point
// of U, 12 GB per 128^3 step); with U in fp32 it writes and the GEMM reads a
// third less.  A is loaded into registers two steps ahead (thread t: row t/2,
// the 8 k of chunk t&1: two float4), split3 in registers and written into the
// same swizzled x3_off16 image with one ds_write_b128 per plane (each 8-lane
// write group covers 32 banks once); B (the weight planes) still moves by
// LDS-DMA.  Per step and wave: A-load(kt+2) (2 ops) then B-DMA(kt+2) (3 ops),
// always issued (out-of-range steps read zeros into unused stages), so the
// counted waits are static: vmcnt(5) retires B-DMA(kt) at the top of step kt,
// vmcnt(8) the A rows of step kt+1 before they are split into stage kt+1.
// Every stage is its own __shared__ array and the k loop is unrolled by 6
// (stage = kt % 3, register set = kt % 2, both static), so the compiler can see
// that the DMA in flight and the ds_reads / ds_writes of other stages do not
// alias and inserts no vmcnt(0) drain of the prefetch.  Same split, same MFMA
// order: bit-identical to x3_gemm256_kernel.
template <int N_> struct IC { static constexpr int v = N_; };
// EPI (compile-time, one instantiation per epilogue so each gets its own
// register allocation): 0 the plain C store, 1 the forward conv epilogue,
// 2 the fused BN-ReLU backward (X3Epi.on)
template <int EPI>
#ifndef M3D_X3AF_STAMP
#define M3D_X3AF_STAMP 0   // timing probe (debug builds): per-workgroup clock stamps into C row m0
#endif
__global__ __launch_bounds__(512, 1) void x3_gemm256_af_kernel(X3G g) {
#if M3D_X3AF_STAMP
    __shared__ __attribute__((aligned(16))) char sAll[18 * G2_PL + 256];
    uint32_t* const stampbuf = reinterpret_cast<uint32_t*>(sAll + 18 * G2_PL);
    char* const sA0 = sAll;
    char* const sA1 = sAll + 3 * G2_PL;
    char* const sA2 = sAll + 6 * G2_PL;
    char* const sB0 = sAll + 9 * G2_PL;
    char* const sB1 = sAll + 12 * G2_PL;
    char* const sB2 = sAll + 15 * G2_PL;
    const uint32_t st_t0 = (uint32_t)__builtin_amdgcn_s_memtime();
    const uint32_t st_r0 = (uint32_t)__builtin_amdgcn_s_memrealtime();
#else
    __shared__ __attribute__((aligned(16))) char sA0[3 * G2_PL], sA1[3 * G2_PL], sA2[3 * G2_PL];
    __shared__ __attribute__((aligned(16))) char sB0[3 * G2_PL], sB1[3 * G2_PL], sB2[3 * G2_PL];
#endif
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 2, wn = wave & 3, h = lane >> 5, l32 = lane & 31;
    const int64_t nbx = (g.M + 255) / 256, nby = g.N / 256;
    const int64_t per_batch = nbx * nby, total = per_batch * g.nbatch;
    const int64_t L = (int64_t)blockIdx.x + (int64_t)gridDim.x * blockIdx.y;
    if (L >= total) return;
    const int64_t xcd = L % 8, q8 = total / 8, r8 = total % 8;
    const int64_t T = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
    const int64_t bz = T / per_batch, Tt = T - bz * per_batch;
    const int64_t m0 = (Tt / nby) * 256;
    const int64_t n0 = (Tt % nby) * 256;
    const int nk = g.K / G2_BK;
    // A: fp32 rows from the tile's first row (rows past M and steps past nk read zeros)
    const __amdgpu_buffer_rsrc_t ra = make_rsrc(g.af + bz * g.bsa + m0 * g.K, (uint64_t)(g.M - m0) * g.K * 4);
    const int arow = tid >> 1, ach = tid & 1;
    const uint32_t aoff0 = ((uint32_t)arow * (uint32_t)g.K + (uint32_t)ach * 8u) * 4u;
    const int awr = x3_off16(arow, ach);
    __amdgpu_buffer_rsrc_t rb[3];
#pragma unroll
    for (int pl = 0; pl < 3; ++pl)
        rb[pl] = make_rsrc(g.b + pl * g.psb + bz * g.bsb + n0 * g.K, (uint64_t)256 * g.K * 2);
    const int lrow = 32 * wave + (lane >> 1);
    const uint32_t lsrc = (uint32_t)lrow * (uint32_t)g.K * 2u + (uint32_t)(((lane & 1) ^ ((lrow >> 3) & 1)) << 4);
    auto stA = [&](auto st) -> char* {
        if constexpr (decltype(st)::v == 0) return sA0;
        else if constexpr (decltype(st)::v == 1) return sA1;
        else return sA2;
    };
    auto stB = [&](auto st) -> char* {
        if constexpr (decltype(st)::v == 0) return sB0;
        else if constexpr (decltype(st)::v == 1) return sB1;
        else return sB2;
    };
    using AReg = float4;
    auto load_a = [&](int kt, float4 (&v)[2]) {
        const bool in = kt < nk;
        const uint32_t o = aoff0 + (uint32_t)kt * (G2_BK * 4);
        v[0] = bload4(ra, in ? o : M3D_OOB);
        v[1] = bload4(ra, in ? o + 16u : M3D_OOB);
    };
    auto dma_b = [&](auto st, int kt) {
        char* S = stB(st) + wave * 1024;
        const uint32_t off = kt < nk ? lsrc + (uint32_t)kt * (G2_BK * 2) : M3D_OOB;
#pragma unroll
        for (int pl = 0; pl < 3; ++pl) g2_dma(rb[pl], S + pl * G2_PL, off);
    };
    auto split_a = [&](auto st, const AReg (&v)[2]) {
        char* S = stA(st) + awr;
        uint2 lo4[3], hi4[3];
        split3x4(make_float4(v[0][0], v[0][1], v[0][2], v[0][3]), lo4);
        split3x4(make_float4(v[1][0], v[1][1], v[1][2], v[1][3]), hi4);
#pragma unroll
        for (int q = 0; q < 3; ++q)
            *reinterpret_cast<uint4*>(S + q * G2_PL) = make_uint4(lo4[q].x, lo4[q].y, hi4[q].x, hi4[q].y);
    };
    floatx16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.0f;
    // A three steps ahead (three register sets): per step A(kt+3) then B(kt+2)
    // are issued, so A(kt+1) (issued at step kt-2, before B(kt)) is retired by
    // the top-of-step wait for B(kt) and no wait sits inside the step
    AReg xa[2], ya[2], za[2];
    load_a(0, xa);
    load_a(1, ya);
    dma_b(IC<0>{}, 0);
    load_a(2, za);
    dma_b(IC<1>{}, 1);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");  // A(0)
    split_a(IC<0>{}, xa);
#if M3D_X3AF_STAMP
    const uint32_t st_t1 = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
    // step kt on stage st = kt % 3: cur holds A(kt+1) (loaded at step kt-1), nxt
    // receives A(kt+2) (its A(kt) was split at step kt-1)
    auto step = [&](auto st, int kt, AReg (&cur)[2], AReg (&nxt)[2]) {
        constexpr int s0 = decltype(st)::v;
        asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)" ::: "memory");   // B(kt); own A(kt) writes
        __builtin_amdgcn_s_barrier();
#if M3D_X3AF_STAMP
        if (tid == 0 && kt < 56) stampbuf[kt] = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
        load_a(kt + 3, nxt);
        dma_b(IC<(s0 + 2) % 3>{}, kt + 2);       // stage last read at step kt-1
        split_a(IC<(s0 + 1) % 3>{}, cur);        // stage last read at step kt-2
        const char* SA = stA(st);
        const char* SB = stB(st);
        bf16x8 bfr[2][3];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int off = x3_off16(wn * 64 + j * 32 + l32, h);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                bfr[j][pl] = *reinterpret_cast<const bf16x8*>(SB + pl * G2_PL + off);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int off = x3_off16(wm * 128 + i * 32 + l32, h);
            bf16x8 af[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) af[pl] = *reinterpret_cast<const bf16x8*>(SA + pl * G2_PL + off);
            x3_mac_pair(acc[i][0], acc[i][1], af[0], af[1], af[2], bfr[0][0], bfr[0][1], bfr[0][2],
                                    bfr[1][0], bfr[1][1], bfr[1][2]);
        }
    };
    // stage kt % 3 and register set kt % 2 static: six steps per trip
    // step kt: cur = set (kt+1) % 3 holds A(kt+1), nxt = set kt % 3 (A(kt) split at step kt-1)
    for (int kt = 0;;) {
        step(IC<0>{}, kt, ya, xa); if (++kt >= nk) break;
        step(IC<1>{}, kt, za, ya); if (++kt >= nk) break;
        step(IC<2>{}, kt, xa, za); if (++kt >= nk) break;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // the trailing (zero) loads
#if M3D_X3AF_STAMP
    const uint32_t st_t2 = (uint32_t)__builtin_amdgcn_s_memtime();
#endif
    const __amdgpu_buffer_rsrc_t rc = make_rsrc(g.c + bz * g.bsc + m0 * g.N, (uint64_t)(g.M - m0) * g.N * 4);
    if constexpr (EPI == 2) {
        // fused BN-ReLU backward (X3Epi on == 2), staged per wave through LDS:
        // each wave writes one 32-row block of its 128 x 64 accumulator tile into
        // a private LDS slot (no barrier: only the wave reads it back), reads it
        // row-major as float4 and applies the BN backward with float4 y / z loads
        // and float4 dz / dres stores.  The accumulators die block by block, so
        // the epilogue needs few registers (the per-element form held the tile,
        // 32 loads and their lane offsets at once and spilled ~140 registers).
        // Rows past M load zeros (masked, summed as 0) and their stores are
        // dropped; an absent y / z / dres has an empty descriptor.
        const X3Epi& E = g.ep;
        const uint64_t rbytes = (uint64_t)(g.M - m0) * g.N * 4;
        const __amdgpu_buffer_rsrc_t ry = make_rsrc(E.fy ? E.fy + m0 * g.N : g.c, E.frelu ? rbytes : 0);
        const __amdgpu_buffer_rsrc_t rzz = make_rsrc(E.fz ? E.fz + m0 * g.N : g.c, E.fz ? rbytes : 0);
        const __amdgpu_buffer_rsrc_t rd = make_rsrc(E.fdres ? E.fdres + m0 * g.N : g.c, E.fdres ? rbytes : 0);
        const bool relu = __builtin_amdgcn_readfirstlane(E.frelu) != 0;
        const bool accum = __builtin_amdgcn_readfirstlane(E.facc) != 0;
        const __amdgpu_buffer_rsrc_t rca = make_rsrc(g.c + m0 * g.N, accum ? rbytes : 0);
        constexpr int WLD = 68;                           // staging row pitch (floats)
        __syncthreads();                                  // every wave's last stage reads are done
        char* const slot0 = (wave % 6 == 0) ? sA0 : (wave % 6 == 1) ? sA1 : (wave % 6 == 2) ? sA2
                          : (wave % 6 == 3) ? sB0 : (wave % 6 == 4) ? sB1 : sB2;
        float* const Tw = reinterpret_cast<float*>(slot0 + (wave / 6) * (32 * WLD * 4));
        const int c4 = lane & 15, rq = lane >> 4;
        const int col = (int)n0 + wn * 64 + c4 * 4;
        float sc[4], mu[4], rs[4], sp[4], sx[4], sz[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sc[e] = E.fscale ? E.fscale[col + e] : 1.0f;
            mu[e] = E.fz ? E.fmean[col + e] : 0.0f;
            rs[e] = E.fz ? E.frstd[col + e] : 1.0f;
            sp[e] = sx[e] = sz[e] = 0.0f;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r)
                    Tw[((r & 3) + 8 * (r >> 2) + 4 * h) * WLD + j * 32 + l32] = acc[i][j][r];
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int lr = rq + 4 * q;
                const float4 a = *reinterpret_cast<const float4*>(Tw + lr * WLD + c4 * 4);
                const uint32_t off = ((uint32_t)(wm * 128 + i * 32 + lr) * (uint32_t)g.N + (uint32_t)col) * 4u;
                const float4 y4 = bload4(ry, off), z4 = bload4(rzz, off), c4v = bload4(rca, off);
                float gv[4], d[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    // the implicit GEMM's accumulate (C += conv^T dz): one fp32 add, then the mask
                    const float t = accum ? f4get(a, e) + f4get(c4v, e) : f4get(a, e);
                    gv[e] = (relu && !(f4get(y4, e) > 0.f)) ? 0.f : t;
                    d[e] = gv[e] * sc[e];
                    sp[e] += gv[e];
                    sx[e] += gv[e] * ((f4get(z4, e) - mu[e]) * rs[e]);
                    sz[e] += d[e];
                }
                bstore4(rc, off, d[0], d[1], d[2], d[3]);
                bstore4(rd, off, gv[0], gv[1], gv[2], gv[3]);
                // the running sums pinned here: left free, the scheduler deferred
                // the 96 serial adds of a block behind all its loads and kept every
                // row's gv / d live until then (spills)
#pragma unroll
                for (int e = 0; e < 4; ++e) asm volatile("" : "+v"(sp[e]), "+v"(sx[e]), "+v"(sz[e]));
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // block i read back before block i+1 is staged
        }
        if (!E.fpart) return;
        // column sums of each 128-row half tile (wave row wm): the four lane groups
        // (rows rq + 4q) combined, one partial row per half tile (no block barrier)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            sp[e] += __shfl_xor(sp[e], 16); sx[e] += __shfl_xor(sx[e], 16); sz[e] += __shfl_xor(sz[e], 16);
            sp[e] += __shfl_xor(sp[e], 32); sx[e] += __shfl_xor(sx[e], 32); sz[e] += __shfl_xor(sz[e], 32);
        }
        if (rq == 0) {
            const int64_t prow = (m0 / 256) * 2 + wm;
            float* const f0 = E.fpart + ((int64_t)0 * E.fprows + prow) * g.N + col;
            float* const f1 = E.fpart + ((int64_t)1 * E.fprows + prow) * g.N + col;
            float* const f2 = E.fpart + ((int64_t)2 * E.fprows + prow) * g.N + col;
            *reinterpret_cast<float4*>(f0) = make_float4(sp[0], sp[1], sp[2], sp[3]);
            *reinterpret_cast<float4*>(f1) = make_float4(sx[0], sx[1], sx[2], sx[3]);
            *reinterpret_cast<float4*>(f2) = make_float4(sz[0], sz[1], sz[2], sz[3]);
        }
        return;
    }
    if constexpr (EPI == 1) {
        // the fused conv epilogue (X3Epi): per accumulator tile its 16 residual
        // values are loaded before its first store; rows past M read zeros and
        // their stores are dropped (the descriptors' range)
        const X3Epi& E = g.ep;
        const uint64_t rbytes = (uint64_t)(g.M - m0) * g.N * 4;
        const __amdgpu_buffer_rsrc_t rr = make_rsrc(E.res ? E.res + m0 * g.N : g.c, E.res ? rbytes : 0);
        const __amdgpu_buffer_rsrc_t rz = make_rsrc(E.z ? E.z + m0 * g.N : g.c, E.z ? rbytes : 0);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = (int)n0 + wn * 64 + j * 32 + l32;
            const float bias = E.bias ? E.bias[col] : 0.0f;
            const float sc = E.scale ? E.scale[col] : 1.0f, sh = E.scale ? E.shift[col] : 0.0f;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float rv[16];
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    rv[r] = E.res ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                        rr, (int)(((uint32_t)row * (uint32_t)g.N + (uint32_t)col) * 4u), 0, 0))
                                  : 0.0f;
                }
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int row = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                    const int off = (int)(((uint32_t)row * (uint32_t)g.N + (uint32_t)col) * 4u);
                    float v = acc[i][j][r];
                    if (E.bias) v += bias;
                    if (E.z) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rz, off, 0, 0);
                    if (E.scale) v = v * sc + sh;
                    if (E.res) v += rv[r];
                    if (E.act) v = act(E.act, v);
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc, off, 0, 0);
                }
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int col = (int)n0 + wn * 64 + j * 32 + l32;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
                const float v = acc[i][j][r];
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rc,
                                                      (int)(((uint32_t)row * (uint32_t)g.N + (uint32_t)col) * 4u),
                                                      0, 0);
            }
        }
#if M3D_X3AF_STAMP
    // wave 0 wrote C row m0, columns n0..n0+31 above: its own later stores win
    const uint32_t st_t3 = (uint32_t)__builtin_amdgcn_s_memtime();
    const uint32_t st_r3 = (uint32_t)__builtin_amdgcn_s_memrealtime();
    if (wave == 0) {
        uint32_t v = 0;
        if (lane == 0) v = st_t0;
        else if (lane == 1) v = st_t1;
        else if (lane == 2) v = st_t2;
        else if (lane == 3) v = st_t3;
        else if (lane == 4) v = st_r0;
        else if (lane == 5) v = st_r3;
        else if (lane == 6) v = (uint32_t)nk;
        else if (lane == 7) v = (uint32_t)__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_ID (XCC/SE/CU ids)
        else if (lane >= 8 && lane - 8 < nk && lane - 8 < 56) v = stampbuf[lane - 8];
        __builtin_amdgcn_raw_buffer_store_b32(v, rc, (int)(((uint32_t)n0 + (uint32_t)lane) * 4u), 0, 0);
    }
#endif
}


// M3D_WINO_NZ = 2 selects the F(2x2x2) tiles (A/B testing; default 4: F(2x2x4))
static int wino_nz() {
    static constexpr int v = M3D_TUNE_WINO_NZ;
    return v;
}
// The weight gradient runs on the forward's F(2x2x4) tiles (round 3; was
// F(2x2x2)): the forward keeps its fp32 transformed input U and the weight
// gradient reads it (no second input transform), with 96 instead of 64 point
// GEMMs over half the tiles -- 25 % fewer MFMA FLOPs.  Its tile-summed products
// pass through G^T, whose F(4,3) rows amplify the fp32 summation error:
// measured 3.3e-6 / 2.8e-6 vs F(2x2x2)'s 1.0e-6 / 1.2e-6 of the gradient's
// scale (128 -> 128 / 256 -> 512 convs, test_wino_weight_gradient_accuracy),
// whole-step gradients at 128^3 median 1.2e-6 vs float64; step 30.9 -> 29.7 ms.
// M3D_WINO_WGRAD_NZ=2 restores F(2x2x2).
static int wino_wgrad_nz() {
    static constexpr int v = M3D_TUNE_WINO_WGRAD_NZ;
    return v;
}
// the data gradient's z tile: the forward's
static int wino_dgrad_nz() { return wino_nz(); }
// The data gradient's y tile (round 5): F(2,3) along y by default, i.e.
// F(2x2x4) tiles, while the forward and the weight gradient keep F(4x2x4).
// The data gradients carry the step's gradient error (every layer's dx feeds
// all earlier layers): F(4,3) on two axes amplifies the point GEMMs' fp32
// accumulation error ~4x over F(2x2x4) (scripts/wino_stage_error.py), and the
// 128^3 step's gradient median against float64 was 6.6e-6 with F(4x2x4) data
// gradients, 2.3e-6 with F(2x2x4) (scripts/grad_table.py, gpurun_out/r05grad).
// M3D_TUNE_WINO_DGRAD_NY=0: the forward's tile.
static int wino_dgrad_ny() {
    static constexpr int v = M3D_TUNE_WINO_DGRAD_NY;
    return v ? v : WNY;
}
static int wino_points(int nz, int ny = WNY) { return (ny + 2) * 4 * (nz + 2); }
static int wino_points() { return wino_points(wino_nz()); }

static WinoGeom wino_geom(int64_t B, int64_t H, int64_t W, int64_t D, int64_t Din, int pz,
                          int nz = -1, int ny = WNY) {
    WinoGeom g{};
    if (nz < 0) nz = wino_nz();
    g.B = (int)B; g.H = (int)H; g.W = (int)W; g.D = (int)D; g.Din = (int)Din; g.pz = pz;
    g.TY = (int)((H + ny - 1) / ny); g.TX = (int)((W + 1) / 2); g.TZ = (int)((D + nz - 1) / nz);
    g.T = B * g.TY * g.TX * g.TZ;
    g.halo = nullptr;
    g.hlo = g.hhi = 0;
    g.tz_mode = 0;
    g.xcd = 0;
    return g;
}

// batched GEMM view over the 64 Winograd points: rows = tiles
static ConvP wino_gemm_p(const float* A, int64_t T, int K, const float* V, int N) {
    ConvP p{};
    p.a = A; p.B = 1; p.H = 1; p.W = 1; p.D = (int)T; p.C = K;      // tiles along "z":
    p.OH = 1; p.OW = 1; p.OD = (int)T;                                // no carries in m loops
    p.kh = p.kw = p.kd = 1; p.sy = p.sx = p.sz = 1;
    p.M = T; p.K = K; p.w = V; p.N = N;
    p.bsa = T * K; p.bsw = (int64_t)K * N; p.bsy = T * N;
    return p;
}

}  // namespace m3d

using namespace m3d;

// Plain batched fp32 GEMM on the conv MFMA kernel: C[b] (+)= act(A[b] B[b] + bias).
// A [M][K], B [K][N], C [M][N] row-major, batches contiguous.  Runs the same
// conv_gemm_kernel instantiations as the Winograd point-wise GEMMs (a GEMM is
// a 1x1x1 conv whose voxels lie along "z").
extern "C" int m3d_gemm_f32(const float* A, const float* Bm, float* C, int64_t batch, int64_t M,
                            int64_t K, int64_t N, const float* bias, int32_t relu,
                            int32_t accumulate, m3d_stream_t s) {
    if (batch <= 0 || M <= 0 || K <= 0 || N <= 0) return einval("gemm: dimensions must be positive");
    if (N % 4) return einval("gemm: N must be a multiple of 4");
    if (M > 0x7FFFFFFF || K > 0x7FFFFFFF || N > 0x7FFFFFFF)
        return einval("gemm: dimension larger than 2^31");
    const int64_t lim = (int64_t)0xFFFFFFF0 / 4;
    if (M * K >= lim || K * N >= lim || M * N >= lim)
        return einval("gemm: operand larger than 4 GiB (32-bit buffer offsets)");
    ConvP p = wino_gemm_p(A, M, (int)K, Bm, (int)N);
    Epi e{};
    e.bias = bias; e.relu = relu; e.accumulate = accumulate;
    e.y = C; e.ldy = N; e.simple = 1; e.YH = 1; e.YW = 1; e.YD = (int)M;
    e.ysy = e.ysx = e.ysz = 1;
    if (K % 32 == 0) dispatch_gemm<false, true>(p, e, st(s), (int)batch);
    else dispatch_gemm<false, false>(p, e, st(s), (int)batch);
    return check_launch("m3d_gemm_f32");
}

extern "C" int m3d_gemm_wgrad_f32(const float* A, const float* Bm, float* C, int64_t batch, int64_t M,
                                  int64_t K, int64_t N, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    if (batch <= 0 || M <= 0 || K <= 0 || N <= 0) return einval("gemm_wgrad: dimensions must be positive");
    if (K % 4 || N % 4) return einval("gemm_wgrad: K and N must be multiples of 4");
    const int64_t lim = (int64_t)0xFFFFFFF0 / 4;
    if (M >= 0x7FFFFFFF || M * K >= lim || M * N >= lim || K * N >= lim)
        return einval("gemm_wgrad: operand larger than 4 GiB (32-bit buffer offsets)");
    if (wgrad_x3_env() && N > 64) {
        launch_wgrad_x3(A, Bm, C, M, (int)K, (int)N, (int)batch, M * K, M * N, K * N, st(s));
        return check_launch("m3d_gemm_wgrad_f32 (x3)");
    }
    ConvP p = wino_gemm_p(A, M, (int)K, nullptr, (int)N);
    p.bsw = M * N;                      // B batch stride
    p.bsy = K * N;                      // C batch stride
    if (N <= 64) launch_wgrad<128, 64, 2, 2, true>(p, Bm, C, st(s), (int)batch);
    else launch_wgrad<128, 128, 2, 2, true>(p, Bm, C, st(s), (int)batch);
    return check_launch("m3d_gemm_wgrad_f32");
}

// The loaders address x / w / dz through 32-bit buffer offsets and the GEMM
// row index m through 32-bit division: an operand the kernels read must stay
// below 4 GiB and 2^31 voxels.  The conv entry points check that per batch item
// and run a batch whose whole tensors pass it one item at a time (the
// epilogues store through 64-bit pointers).  M3D_OPERAND_LIMIT (bytes) lowers
// the bound, to exercise the per-item path at test sizes.
static int64_t op_lim() {
    static const int64_t v = [] {
        const char* e = getenv("M3D_OPERAND_LIMIT");
        const long long l = e ? atoll(e) : 0;
        return (int64_t)((l > 0 && l < 0xFFFFFFF0LL) ? l : 0xFFFFFFF0LL) / 4;
    }();
    return v;
}

// batch of B items of in-voxels vin x cin and out-voxels vout x cout: one item at a time?
static bool per_item(int64_t B, int64_t vin, int64_t cin, int64_t vout, int64_t cout) {
    return B > 1 && (B * vin * cin >= op_lim() || B * vout * cout >= op_lim() || B * vin > 0x7FFFFFFF ||
                     B * vout > 0x7FFFFFFF);
}

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
    if (H * W * D > 0x7FFFFFFF || OH * OW * OD > 0x7FFFFFFF)
        return einval("conv3d: more than 2^31 voxels per batch item");
    const int64_t lim = op_lim();
    if (H * W * D * Cin >= lim || OH * OW * OD * Cout >= lim || (int64_t)kh * kw * kd * Cin * Cout >= lim)
        return einval("conv3d: operand of one batch item larger than 4 GiB (32-bit buffer offsets)");
    return M3D_OK;
}

// Strided batched GEMM: C[b] (+)= act(A[b] B[b] + bias), A[b] rows of stride
// lda (K <= lda) at A + b*bsa, B[b] = B + b*bsb [K][N], C[b] = C + b*bsc [M][N].
// Split-K is this call with batch = #K-slices (bsa = slice width, bsb =
// slice*N) into a workspace, then m3d_splitk_reduce.
extern "C" int m3d_gemm_f32_ex(const float* A, int64_t lda, int64_t bsa, const float* Bm,
                               int64_t bsb, float* C, int64_t bsc, int64_t batch, int64_t M,
                               int64_t K, int64_t N, const float* bias, int32_t act_code,
                               int32_t accumulate, m3d_stream_t s) {
    if (batch <= 0 || M <= 0 || K <= 0 || N <= 0) return einval("gemm: dimensions must be positive");
    if (N % 4) return einval("gemm: N must be a multiple of 4");
    if (lda < K) return einval("gemm: lda < K");
    if (M > 0x7FFFFFFF || lda > 0x7FFFFFFF || N > 0x7FFFFFFF)
        return einval("gemm: dimension larger than 2^31");
    const int64_t lim = (int64_t)0xFFFFFFF0 / 4;
    if (M * lda >= lim || K * N >= lim || M * N >= lim)
        return einval("gemm: operand larger than 4 GiB (32-bit buffer offsets)");
    ConvP p{};
    p.a = A; p.B = 1; p.H = 1; p.W = (int)M; p.D = 1; p.C = (int)lda;   // rows along "x"
    p.OH = 1; p.OW = (int)M; p.OD = 1;
    p.kh = p.kw = p.kd = 1; p.sy = p.sx = p.sz = 1;
    p.M = M; p.K = (int)K; p.w = Bm; p.N = (int)N;
    p.bsa = bsa; p.bsw = bsb; p.bsy = bsc;
    Epi e{};
    e.bias = bias; e.relu = act_code; e.accumulate = accumulate;
    e.y = C; e.ldy = N; e.simple = 1; e.YH = 1; e.YW = 1; e.YD = (int)M;
    e.ysy = e.ysx = e.ysz = 1;
    const bool vec = K % 32 == 0 && lda % 4 == 0 && bsa % 4 == 0 && ((uintptr_t)A & 15) == 0;
    if (vec) dispatch_gemm<false, true>(p, e, st(s), (int)batch);
    else dispatch_gemm<false, false>(p, e, st(s), (int)batch);
    return check_launch("m3d_gemm_f32_ex");
}

// out[m][n] = act((sum_z ws[z][m][n] + bias[n]) * scale[n] + shift[n]), z in
// order (deterministic).
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, int splits,
                                                            int64_t M, int N,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift,
                                                            int act_code, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M * N) return;
    const int n = (int)(i % N);
    float v = ws[i];
    for (int z = 1; z < splits; ++z) v += ws[(int64_t)z * M * N + i];
    if (bias) v += bias[n];
    if (scale) v = v * scale[n] + shift[n];
    out[i] = act(act_code, v);
}

extern "C" int m3d_splitk_reduce(const float* ws, int32_t splits, int64_t M, int64_t N,
                                 const float* bias, const float* bn_scale, const float* bn_shift,
                                 int32_t act_code, float* out, m3d_stream_t s) {
    if (splits <= 0 || M < 0 || N <= 0) return einval("splitk_reduce: bad dimensions");
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("splitk_reduce: bn_scale and bn_shift must be given together");
    if (M == 0) return M3D_OK;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(grid_for(M * N, 256)), dim3(256), 0, st(s), ws, splits,
                       M, (int)N, bias, bn_scale, bn_shift, act_code, out);
    return check_launch("splitk_reduce_kernel");
}

// Conv3DTranspose(Cout, (2,2,2), strides=2, 'valid') (mrcnn_mask_deconv,
// core/models.py:1228-1232): y[2i+a, 2j+b, 2k+c, o] = act(bias[o] +
// sum_c x[i,j,k,c] w[a,b,c,o,cin]), Keras kernel [2,2,2,Cout,Cin].  One GEMM
// rows = input voxels, K = Cin, columns = (tap, o) read from the kernel as
// B^T, scattered by the epilogue to the 8 output voxels of each input voxel.
extern "C" int m3d_deconv3d_k2s2(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                 int64_t Cin, const float* w, int64_t Cout, const float* bias,
                                 int32_t act_code, float* y, m3d_stream_t s) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0 || Cin <= 0 || Cout <= 0)
        return einval("deconv3d: tensor dimensions must be positive");
    if (Cout % 4 || Cin % 32) return einval("deconv3d: Cout % 4 == 0 and Cin % 32 == 0 required");
    const int64_t lim = (int64_t)0xFFFFFFF0 / 4;
    if (B * H * W * D * Cin >= lim || B * H * W * D * 8 * Cout >= lim)
        return einval("deconv3d: operand larger than 4 GiB (32-bit buffer offsets)");
    ConvP p{};
    p.a = x; p.B = (int)B; p.H = (int)H; p.W = (int)W; p.D = (int)D; p.C = (int)Cin;
    p.OH = (int)H; p.OW = (int)W; p.OD = (int)D;
    p.kh = p.kw = p.kd = 1; p.sy = p.sx = p.sz = 1;
    p.M = B * H * W * D; p.K = (int)Cin; p.w = w; p.N = (int)(8 * Cout);
    Epi e{};
    e.bias = bias; e.relu = act_code; e.y = y; e.ldy = Cout;
    e.YH = (int)(2 * H); e.YW = (int)(2 * W); e.YD = (int)(2 * D);
    e.ysy = e.ysx = e.ysz = 1; e.simple = 0; e.deconv = (int)Cout;
    dispatch_gemm<true, true>(p, e, st(s));
    return check_launch("conv_gemm_kernel(deconv)");
}

// ---- the one-channel 7^3 stem: conv1 (core/models.py:242, Conv3D(64, (7,7,7),
// strides (2,2,1)) after ZeroPadding3D(3)) -------------------------------------
// The implicit GEMM's scalar loader reaches 0.27 of the f32 MFMA peak here
// (K = 343 taps of ONE channel: no channel vector to load).  This kernel keeps
// the whole K operand on chip: the 343 x 64 weights live in LDS for the life
// of a workgroup that loops over many tiles (about 4 per CU), and every wave owns one
// output column (oy, ox) x 32 z x 64 channels with its own input window (the
// 49 (ky, kx) rows x 38 z voxels, + one zero row) in its own LDS region,
// refilled from registers prefetched during the previous tile's MFMAs.  No
// barrier after the weight load: the waves of a CU run out of phase.
// K order: the two MFMA k-slots (lane halves h) walk (ky, kx) rows R = rp and
// R = rp + 25 in step, 7 taps kz each -- so a lane's window offset is
// R * 38 + kz: one add per row, the 7 taps as ds_read immediates (a
// per-tap index walk cost more issue than the MFMAs).  Row R = 49 is the
// padding (zero weights, zero window row).  Epilogue: each 32-channel
// accumulator is staged in the wave's LDS region (row stride 40 floats:
// the lane halves, 4 rows apart, land 32 banks apart) and leaves as
// row-contiguous float4s through epi_store4 (bias, z, frozen BN, ReLU).
// Summation order: K in the (R pair, kz) order above -- an exact f32 FMA
// chain, a different order than the implicit GEMM (parity 1e-4).
constexpr int STEM_TZ = 32;
constexpr int STEM_WZ = STEM_TZ + 6;                             // 38
constexpr int STEM_WIN = 50 * STEM_WZ;                           // 49 rows + the zero row: 1900 floats
constexpr int STEM_RP = 25;                                      // row pairs (R, R + 25)
constexpr int STEM_NP = STEM_RP * 7;                             // 175 k pairs
constexpr int STEM_PER = (49 * STEM_WZ + 63) / 64;               // window values per lane (30)
constexpr int STEM_SLD = 40;                                     // epilogue staging row stride

__global__ __launch_bounds__(512) void stem_fwd_kernel(ConvP p, Epi e, int tz_n, int64_t ntiles) {
    __shared__ float wsh[STEM_NP * 128];          // [pair][h*32+l32][nb]  (89.6 KB)
    __shared__ float win[8][STEM_WIN];            // one window / staging region per wave (60.8 KB)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int l32 = lane & 31, h = lane >> 5;
    for (int i = tid; i < STEM_NP * 128; i += 512) {
        const int kp = i >> 7, r = i & 127, nb = r & 1, hl = r >> 1, hh = hl >> 5, ll = hl & 31;
        const int R = kp / 7 + STEM_RP * hh, kz = kp % 7;
        wsh[i] = R < 49 ? p.w[(R * 7 + kz) * 64 + nb * 32 + ll] : 0.0f;
    }
    float* ww = win[wave];
    if (lane < STEM_WZ) ww[49 * STEM_WZ + lane] = 0.0f;   // the padding row
    __syncthreads();                              // the only barrier: waves run free below
    const size_t plane = (size_t)(p.halo ? p.hdl : p.D), row = (size_t)p.W * plane, img = (size_t)p.H * row;
    auto decode = [&](int64_t t, int& b, int& oy, int& ox, int& tz) {
        tz = (int)(t % tz_n); t /= tz_n;
        ox = (int)(t % p.OW); t /= p.OW;
        oy = (int)(t % p.OH);
        b = (int)(t / p.OH);
    };
    auto fetch = [&](int64_t tile, float* v) {
        int b, oy, ox, tz;
        decode(tile, b, oy, ox, tz);
        const int gy0 = 2 * oy - p.py, gx0 = 2 * ox - p.px, gz0 = tz * STEM_TZ - p.pz;
        const float* xb = p.a + b * img;
#pragma unroll
        for (int q = 0; q < STEM_PER; ++q) {
            const int i = lane + 64 * q;
            float val = 0.0f;
            if (i < 49 * STEM_WZ) {
                const int R = i / STEM_WZ, iz = i - R * STEM_WZ;
                const int gy = gy0 + R / 7, gx = gx0 + R % 7, gz = gz0 + iz;
                if (gy >= 0 && gy < p.H && gx >= 0 && gx < p.W && gz >= 0 && gz < p.D) {
                    if (p.halo) {     // virtual z grid: slab planes from x, the others from the halo
                        const int zl = gz - p.hnlo;
                        if ((unsigned)zl < (unsigned)p.hdl)
                            val = xb[gy * row + gx * plane + zl];
                        else
                            val = p.halo[(((size_t)b * p.H + gy) * p.W + gx) * (2 * p.hr) +
                                         (zl < 0 ? zl + p.hr : p.hr + zl - p.hdl)];
                    } else {
                        val = xb[gy * row + gx * plane + gz];
                    }
                }
            }
            v[q] = val;
        }
    };
    const int64_t w0 = (int64_t)blockIdx.x * 8 + wave, wstride = (int64_t)gridDim.x * 8;
    float4 ebias[2], escale[2], eshift[2];
    for (int nb = 0; nb < 2; ++nb) {
        const int n = nb * 32 + 4 * (lane & 7);
        ebias[nb] = e.bias ? ld4(e.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        escale[nb] = e.scale ? ld4(e.scale + n) : make_float4(1.f, 1.f, 1.f, 1.f);
        eshift[nb] = e.scale ? ld4(e.shift + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float pre[STEM_PER];
    if (w0 < ntiles) fetch(w0, pre);
    for (int64_t tile = w0; tile < ntiles; tile += wstride) {
#pragma unroll
        for (int q = 0; q < STEM_PER; ++q)
            if (lane + 64 * q < 49 * STEM_WZ) ww[lane + 64 * q] = pre[q];
        __builtin_amdgcn_wave_barrier();
        if (tile + wstride < ntiles) fetch(tile + wstride, pre);      // next window in flight
        int b, oy, ox, tz;
        decode(tile, b, oy, ox, tz);
        floatx16 acc0 = {}, acc1 = {};
        const float* wa = ww + STEM_RP * STEM_WZ * h + l32;           // row R = rp + 25 h
        const float* wb = wsh + lane * 2;
        for (int rp = 0; rp < STEM_RP; ++rp) {
#pragma unroll
            for (int kz = 0; kz < 7; ++kz) {
                const float a = wa[kz];
                const float2 bv = *reinterpret_cast<const float2*>(wb + kz * 128);
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv.x, acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv.y, acc1, 0, 0, 0);
            }
            wa += STEM_WZ;
            wb += 7 * 128;
        }
        __builtin_amdgcn_wave_barrier();          // window reads done before the staging writes
        const int64_t mbase = (((int64_t)b * p.OH + oy) * p.OW + ox) * p.OD;
        const int oz0 = tz * STEM_TZ;
#pragma unroll
        for (int nb = 0; nb < 2; ++nb) {
            const floatx16& acc = nb ? acc1 : acc0;
#pragma unroll
            for (int r = 0; r < 16; ++r) ww[((r & 3) + 8 * (r >> 2) + 4 * h) * STEM_SLD + l32] = acc[r];
            __builtin_amdgcn_wave_barrier();
            // a lane's 4 channels are the same in every row it stores (c4 = lane & 7):
            // the epilogue parameters are held in registers (epi_store4's order of ops)
            const int n = nb * 32 + 4 * (lane & 7);
            const float4 bb = ebias[nb], sc = escale[nb], sh = eshift[nb];
#pragma unroll
            for (int q = 0; q < 4; ++q) {                 // 32 rows x 8 float4 = 4 per lane
                const int rr = (lane >> 3) + 8 * q;
                float4 v = *reinterpret_cast<const float4*>(ww + rr * STEM_SLD + 4 * (lane & 7));
                if (oz0 + rr >= p.OD) continue;
                const int64_t m = mbase + oz0 + rr;
                if (e.bias) { v.x += bb.x; v.y += bb.y; v.z += bb.z; v.w += bb.w; }
                if (e.z) st4(e.z + m * 64 + n, v);
                if (e.scale) {
                    v.x = v.x * sc.x + sh.x; v.y = v.y * sc.y + sh.y;
                    v.z = v.z * sc.z + sh.z; v.w = v.w * sc.w + sh.w;
                }
                if (e.relu) {
                    v.x = act(e.relu, v.x); v.y = act(e.relu, v.y); v.z = act(e.relu, v.z); v.w = act(e.relu, v.w);
                }
                st4(e.y + m * 64 + n, v);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
}


static bool stem_ok(int64_t Cin, int kh, int kw, int kd, int64_t Cout, int sy, int sx, int sz, int dly, int dlx,
                    int dlz, int res_mode, int64_t split_n, int64_t ldy) {
    // the kernel's own epilogue covers bias / z / frozen BN / activation, plain
    // [M, 64] stores (no residual, split or accumulate)
    return Cin == 1 && kh == 7 && kw == 7 && kd == 7 && Cout == 64 && sy == 2 && sx == 2 && sz == 1 &&
           dly == 1 && dlx == 1 && dlz == 1 && res_mode == 0 && split_n <= 0 && (ldy <= 0 || ldy == 64);
}

// ---- the stem's weight gradient: dW[343][64] += sum_m window(m)[tap] dz[m][ch] ----
// The implicit-GEMM weight gradient reads the one-channel window through its
// scalar loader (0.27 of the f32 MFMA peak).  Here a workgroup (8 waves) loops
// over a contiguous range of m-tiles (one output column (oy, ox) x 32 z); per
// tile the 49 x 38 input window (the same fetch as stem_fwd_kernel, halo planes
// included) and the 32 x 64 dz rows are staged in LDS (double-buffered, one
// barrier per tile) and every wave accumulates its 11 of the 88 16 x 16 dW
// tiles (v_mfma_f32_16x16x4_f32: one n-tile of 16 channels x 11 k-tiles of 16
// taps) over the tile's 32 m in steps of 4.  A lane's window offset per k-tile
// is precomputed (tap -> R * 38 + kz), so every operand read is a ds_read_b32
// with an immediate offset.  Taps 343..351 read the zero row.  The partial dW
// leaves through wg_put (fp32 atomics, or the deterministic-mode partials).
constexpr int SWG_STR = 80;                                      // dz staging row stride (floats)
__global__ __launch_bounds__(512) void stem_wgrad_kernel(ConvP p, const float* __restrict__ dz,
                                                         float* __restrict__ dw, WgOut wo, int tz_n,
                                                         int64_t ntiles, int64_t per_block) {
    __shared__ float win[2][STEM_WIN];            // 49 rows x 38 z + the zero row
    __shared__ float dzs[2][STEM_TZ * SWG_STR];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t t_begin = (int64_t)blockIdx.x * per_block;
    const int64_t t_end = t_begin + per_block < ntiles ? t_begin + per_block : ntiles;
    if (t_begin >= t_end) return;
    float* const wp = wo.part ? wo.part + (int64_t)blockIdx.x * wo.pstride : nullptr;
    if (tid < STEM_WZ) { win[0][49 * STEM_WZ + tid] = 0.0f; win[1][49 * STEM_WZ + tid] = 0.0f; }
    const size_t plane = (size_t)(p.halo ? p.hdl : p.D), row = (size_t)p.W * plane, img = (size_t)p.H * row;
    // per tile: window values i = tid + 512 q (q < 4), dz float4 tid
    float wv[4];
    float4 dv;
    auto fetch = [&](int64_t tile) {
        int64_t t = tile;
        const int tz = (int)(t % tz_n); t /= tz_n;
        const int ox = (int)(t % p.OW); t /= p.OW;
        const int oy = (int)(t % p.OH);
        const int b = (int)(t / p.OH);
        const int gy0 = 2 * oy - p.py, gx0 = 2 * ox - p.px, gz0 = tz * STEM_TZ - p.pz;
        const float* xb = p.a + b * img;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int i = tid + 512 * q;
            float val = 0.0f;
            if (i < 49 * STEM_WZ) {
                const int R = i / STEM_WZ, iz = i - R * STEM_WZ;
                const int gy = gy0 + R / 7, gx = gx0 + R % 7, gz = gz0 + iz;
                if (gy >= 0 && gy < p.H && gx >= 0 && gx < p.W && gz >= 0 && gz < p.D) {
                    if (p.halo) {
                        const int zl = gz - p.hnlo;
                        if ((unsigned)zl < (unsigned)p.hdl)
                            val = xb[gy * row + gx * plane + zl];
                        else
                            val = p.halo[(((size_t)b * p.H + gy) * p.W + gx) * (2 * p.hr) +
                                         (zl < 0 ? zl + p.hr : p.hr + zl - p.hdl)];
                    } else {
                        val = xb[gy * row + gx * plane + gz];
                    }
                }
            }
            wv[q] = val;
        }
        const int zi = tid >> 4, c4 = tid & 15;          // 32 rows x 16 float4
        const int oz = tz * STEM_TZ + zi;
        dv = oz < p.OD ? *reinterpret_cast<const float4*>(
                             dz + ((((int64_t)b * p.OH + oy) * p.OW + ox) * p.OD + oz) * 64 + c4 * 4)
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto stage = [&](int buf) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            if (tid + 512 * q < 49 * STEM_WZ) win[buf][tid + 512 * q] = wv[q];
        *reinterpret_cast<float4*>(&dzs[buf][(tid >> 4) * SWG_STR + (tid & 15) * 4]) = dv;
    };
    // this wave: n-tile nt (16 channels), k-tiles kt = kg + 2 j (j < 11) of 16 taps
    const int nt = wave & 3, kg = wave >> 2;
    const int l16 = lane & 15, lq = lane >> 4;
    int abase[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) {
        const int tap = 16 * (kg + 2 * j) + l16;
        const int R = tap < 343 ? tap / 7 : 49, kz = tap < 343 ? tap % 7 : 0;
        abase[j] = R * STEM_WZ + kz + lq;
    }
    const int bbase = lq * SWG_STR + nt * 16 + l16;
    floatx4 acc[11];
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
    fetch(t_begin);
    stage(0);
    __syncthreads();
    int buf = 0;
    for (int64_t t = t_begin; t < t_end; ++t) {
        if (t + 1 < t_end) fetch(t + 1);
        const float* W = win[buf];
        const float* Z = dzs[buf];
#pragma unroll
        for (int s = 0; s < STEM_TZ / 4; ++s) {
            const float bv = Z[bbase + 4 * s * SWG_STR];
#pragma unroll
            for (int j = 0; j < 11; ++j)
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(W[abase[j] + 4 * s], bv, acc[j], 0, 0, 0);
        }
        if (t + 1 < t_end) stage(buf ^ 1);
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int j = 0; j < 11; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int tap = 16 * (kg + 2 * j) + 4 * lq + r;
            if (tap < 343) wg_put(wo, dw, wp, (int64_t)tap * 64 + nt * 16 + l16, acc[j][r]);
        }
}


static int launch_stem_wgrad(const ConvP& p, const float* dz, float* dw, hipStream_t s) {
    const int ncu = num_cus();
    const int tz_n = (p.OD + STEM_TZ - 1) / STEM_TZ;
    const int64_t ntiles = (int64_t)p.B * p.OH * p.OW * tz_n;
    // two workgroups per CU (LDS 2 x 23.4 KB each, 8 waves), >= 8 m-tiles each
    int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(2 * (int64_t)ncu, (ntiles + 7) / 8));
    const WgOut wo = wg_out(blocks, 1, 343, 64);
    const int64_t per = (ntiles + blocks - 1) / blocks;
    blocks = (ntiles + per - 1) / per;
    hipLaunchKernelGGL(stem_wgrad_kernel, dim3((unsigned)blocks), dim3(512), 0, s, p, dz, dw, wo, tz_n, ntiles, per);
    wg_finish(wo, blocks, 1, 343, 64, 343 * 64, dw, s);
    return check_launch("stem_wgrad_kernel");
}

static int launch_stem(const ConvP& p, const Epi& e, hipStream_t s) {
    const int ncu = num_cus();
    const int tz_n = (p.OD + STEM_TZ - 1) / STEM_TZ;
    const int64_t ntiles = (int64_t)p.B * p.OH * p.OW * tz_n;
    // about four workgroups per CU, not one persistent workgroup per CU: the
    // stem opens the step while the previous step's side-stream work (the
    // one-CU NMS reduce) may still hold a CU, and a persistent block waiting
    // for that CU would stall the whole launch (measured 1.5 ms in the step
    // vs 0.28 ms alone at 128^3); with 4 per CU the others absorb its share
    // M3D_STEM_X3=1 / 2: the bf16-split forms (measured slower than the f32 kernel: 2.65 / 2.24-2.5 vs
    // 2.2 ms at 256^3, DESIGN.md round-3 list); default the f32 MFMA kernel
    const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>((ntiles + 7) / 8, 4 * (int64_t)ncu));
    hipLaunchKernelGGL(stem_fwd_kernel, dim3(grid), dim3(512), 0, s, p, e, tz_n, ntiles);
    return check_launch("stem_fwd_kernel");
}

extern "C" int m3d_conv3d_fwd_dil(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                  int64_t Cin, const float* w, int32_t kh, int32_t kw, int32_t kd,
                                  int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                                  int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                                  int32_t dly, int32_t dlx, int32_t dlz, const float* bias,
                                  const float* bn_scale, const float* bn_shift,
                                  const float* residual, int32_t res_mode, int32_t act_code,
                                  float* z_out, float* y, int64_t ldy, float* y2, int64_t ldy2,
                                  int64_t split_n, m3d_stream_t s) {
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (dly <= 0 || dlx <= 0 || dlz <= 0) return einval("conv3d: dilation must be positive");
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("conv3d: bn_scale and bn_shift must be given together");
    if (res_mode < 0 || res_mode > 3) return einval("conv3d: res_mode must be 0..3");
    if (act_code < 0 || act_code > 2) return einval("conv3d: activation must be 0 (none), 1 (relu), 2 (sigmoid)");
    if (res_mode != 0 && residual == nullptr) return einval("conv3d: residual missing");
    if (res_mode == 2 && ((OH & 1) || (OW & 1))) return einval("conv3d: upsampled residual needs even OH/OW");
    if (split_n > 0 && y2 == nullptr) return einval("conv3d: split output needs y2");
    if (per_item(B, H * W * D, Cin, OH * OW * OD, Cout)) {
        const int64_t xs = H * W * D * Cin, os = OH * OW * OD, ld = ldy > 0 ? ldy : Cout;
        const int64_t rs = res_mode == 2 ? (OH / 2) * (OW / 2) * OD * Cout : os * ld;
        for (int64_t b = 0; b < B; ++b) {
            rc = m3d_conv3d_fwd_dil(x + b * xs, 1, H, W, D, Cin, w, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz, py, px,
                                    pz, dly, dlx, dlz, bias, bn_scale, bn_shift,
                                    residual ? residual + b * rs : nullptr, res_mode, act_code,
                                    z_out ? z_out + b * os * Cout : nullptr, y + b * os * ld, ldy,
                                    y2 ? y2 + b * os * ldy2 : nullptr, ldy2, split_n, s);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    ConvP p{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), w, (int)Cout, 0, 0, 0, 0};
    p.dly = dly; p.dlx = dlx; p.dlz = dlz;
    Epi e{bias, bn_scale, bn_shift, residual, res_mode, act_code, z_out, y, ldy > 0 ? ldy : Cout,
          y2, ldy2, (int)split_n, (int)OH, (int)OW, (int)OD, 1, 1, 1, 0, 1};
    if (stem_ok(Cin, kh, kw, kd, Cout, sy, sx, sz, dly, dlx, dlz, res_mode, split_n, ldy)) return launch_stem(p, e, st(s));
    if (Cin % 32 == 0) dispatch_gemm<false, true>(p, e, st(s));
    else dispatch_gemm<false, false>(p, e, st(s));
    return check_launch("conv_gemm_kernel(fwd)");
}

extern "C" int m3d_conv3d_fwd(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                              int64_t Cin, const float* w, int32_t kh, int32_t kw, int32_t kd,
                              int64_t Cout, int64_t OH, int64_t OW, int64_t OD, int32_t sy,
                              int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                              const float* bias, const float* bn_scale, const float* bn_shift,
                              const float* residual, int32_t res_mode, int32_t relu, float* z_out,
                              float* y, int64_t ldy, float* y2, int64_t ldy2, int64_t split_n,
                              m3d_stream_t s) {
    return m3d_conv3d_fwd_dil(x, B, H, W, D, Cin, w, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz, py, px,
                              pz, 1, 1, 1, bias, bn_scale, bn_shift, residual, res_mode, relu, z_out,
                              y, ldy, y2, ldy2, split_n, s);
}

static int bwd_data_direct(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                           int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                           int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz, float* dx,
                           int32_t accumulate, hipStream_t s, const Epi* fb, int64_t* fb_rows);

extern "C" int m3d_conv3d_bwd_data(const float* dz, const float* w, int64_t B, int64_t H,
                                   int64_t W, int64_t D, int64_t Cin, int32_t kh, int32_t kw,
                                   int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                   int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px,
                                   int32_t pz, float* dx, int32_t accumulate, m3d_stream_t s) {
    return bwd_data_direct(dz, w, B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz, py, px, pz, dx,
                           accumulate, st(s), nullptr, nullptr);
}

// the output-tile height dispatch_gemm picks for a GEMM of N columns (rows of
// the fused BN backward's channel partials: one per tile row)
static int dispatch_bm(const ConvP& p, int nbatch = 1) {
    if (p.N <= 64) return 128;
    const int64_t blocks128 = ((p.M + 127) / 128) * ((p.N + 127) / 128) * nbatch;
    return blocks128 < 512 ? 64 : 128;
}

static int bwd_data_direct(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                           int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                           int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz, float* dx,
                           int32_t accumulate, hipStream_t hs, const Epi* fb, int64_t* fb_rows) {
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (Cout % 32) return einval("conv3d bwd-data: Cout must be a multiple of 32");
    if (Cin % 4) return einval("conv3d bwd-data: Cin must be a multiple of 4");
    const bool unit = kh == 1 && kw == 1 && kd == 1;
    if (!unit && (sy != 1 || sx != 1 || sz != 1))
        return einval("conv3d bwd-data: strided convs supported for 1x1x1 kernels only");
    if (per_item(B, H * W * D, Cin, OH * OW * OD, Cout)) {
        if (fb) return einval("conv3d bwd-data (fused BN backward): batch past the 32-bit operand bound");
        for (int64_t b = 0; b < B; ++b) {
            rc = bwd_data_direct(dz + b * OH * OW * OD * Cout, w, 1, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD,
                                 sy, sx, sz, py, px, pz, dx + b * H * W * D * Cin, accumulate, hs, nullptr, nullptr);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    ConvP p{};
    Epi e{};
    if (fb) e = *fb;
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
    if (fb) {
        if (!e.simple) return einval("conv3d bwd-data (fused BN backward): strided convs unsupported");
        e.fprows = (p.M + dispatch_bm(p) - 1) / dispatch_bm(p);
        if (fb_rows) *fb_rows = e.fprows;
    }
    dispatch_gemm<true, true>(p, e, hs);
    return check_launch("conv_gemm_kernel(bwd-data)");
}

// ---- data gradients with the fused BN-ReLU backward of the producing unit -----
static int bn_fuse_epi(const m3d_bn_bwd_t* bn, int64_t C, void* ws, size_t ws_bytes, int64_t rows, Epi& e) {
    if (!bn) return einval("bwd-data (fused BN backward): null descriptor");
    if (bn->relu && !bn->y) return einval("bwd-data (fused BN backward): relu needs y");
    if (bn->sum_dpre_xhat && !(bn->z && bn->mean && bn->rstd))
        return einval("bwd-data (fused BN backward): xhat sums need z, mean and rstd");
    if (C % 4) return einval("bwd-data (fused BN backward): C must be a multiple of 4");
    const bool sums = bn->sum_dpre || bn->sum_dpre_xhat || bn->sum_dz;
    if (sums && ws_bytes < sizeof(float) * 3 * (size_t)rows * (size_t)C)
        return einval("bwd-data (fused BN backward): workspace too small");
    e.fbn = 1;
    e.frelu = bn->relu ? 1 : 0;
    e.fy = bn->y;
    e.fz = bn->sum_dpre_xhat ? bn->z : nullptr;
    e.fscale = bn->scale;
    e.fmean = bn->mean;
    e.frstd = bn->rstd;
    e.fdres = bn->dres;
    e.fpart = sums ? (float*)ws : nullptr;
    e.fprows = rows;
    return M3D_OK;
}

// rows of channel partials either fused form writes for an input grid of M voxels (upper bound)
static int64_t bn_fuse_rows(int64_t B, int64_t H, int64_t W, int64_t D, int64_t C) {
    const int64_t M = B * H * W * D;
    const int64_t t2 = B * ((H + 1) / 2) * ((W + 1) / 2) * ((D + 1) / 2);   // Winograd tiles, NZ >= 2
    return std::max<int64_t>(std::max<int64_t>((M + 63) / 64, t2), bn_act_bwd_rows(M, C));
}

extern "C" size_t m3d_bn_bwd_fused_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D, int64_t C) {
    if (C <= 0) C = 4;
    return sizeof(float) * 3 * (size_t)bn_fuse_rows(B, H, W, D, C) * (size_t)C;
}

extern "C" int m3d_conv3d_bwd_data_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                                      int64_t Cin, int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH,
                                      int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz, int32_t py,
                                      int32_t px, int32_t pz, float* dx, int32_t accumulate, const m3d_bn_bwd_t* bn,
                                      void* workspace, size_t ws_bytes, m3d_stream_t s) {
    Epi e{};
    int rc = bn_fuse_epi(bn, Cin, workspace, ws_bytes, bn_fuse_rows(B, H, W, D, Cin), e);
    if (rc) return rc;
    int64_t rows = 0;
    rc = bwd_data_direct(dz, w, B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz, py, px, pz, dx, accumulate,
                         st(s), &e, &rows);
    if (rc) return rc;
    return bn_sums_reduce(e.fpart, rows, Cin, bn->sum_dpre, bn->sum_dpre_xhat, bn->sum_dz, st(s));
}

// ---- split-K form of the 1x1x1 direct convs whose tiles do not fill the chip --
// The deep stages' 1x1x1 convs have few output rows (res5: 2048 voxels at
// 128^3), so their 128x128 output tiles occupy a quarter of the CUs, each
// walking K = Cin (up to 2048) alone.  Split-K: `splits` K-slices run as the
// batch of one launch (the slice's channels are an offset into the rows of x /
// dz and of w), each writing its partial tile plainly into the workspace; one
// reduce kernel sums the slices in slice order (deterministic) and applies the
// conv's epilogue (bias, z, BN, residual, ReLU, strided or accumulated store)
// through the same epi_store4 as the one-pass kernel.
__global__ __launch_bounds__(256) void splitk_epi_kernel(const float* ws, int splits,   // (may be e.y: in place)
                                                         ConvP p, Epi e) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int N4 = p.N >> 2;
    if (i >= p.M * N4) return;
    const int64_t m = i / N4;
    const int n = (int)(i - m * N4) * 4;
    const int64_t plane = p.M * p.N;
    float4 v = ld4(ws + m * p.N + n);
    for (int z = 1; z < splits; ++z) {
        const float4 t = ld4(ws + z * plane + m * p.N + n);
        v.x += t.x; v.y += t.y; v.z += t.z; v.w += t.w;
    }
    epi_store4(p, e, m, n, v);
}

// K-slices for a 1x1x1 conv GEMM of M rows, reduction K, N columns (1: no split).
// Only where the 128x128 tiles leave CUs idle AND each walks a long K (>= 1024),
// or the tiles are very few (<= 32); doubled while the tiles times the slices
// stay under two per CU and a slice keeps >= 128 channels (4 k-tiles).
// Measured per layer at 128^3 (scripts/conv_layers.py): res5 2048 -> 512
// 117 -> 67 us, the P5 lateral 2048 -> 256 106 -> 39 us; K = 512 with 128-256
// tiles lost 10-25 % (the extra partial-sum traffic, no idle CUs to gain).
static int splitk_count(int64_t M, int64_t K, int64_t N) {
    if (N % 4 || K % 32) return 1;
    const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
    if (tiles >= num_cus() || (K < 1024 && tiles > 32)) return 1;
    int s = 1;
    while (s < 8 && tiles * s < 2 * num_cus() && K % (64 * s) == 0 && K / (2 * s) >= 128) s *= 2;
    return s;
}

extern "C" int32_t m3d_conv3d_splitk_count(int64_t M, int64_t K, int64_t N) {
    if (M <= 0 || K <= 0 || N <= 0) return 1;
    return splitk_count(M, K, N);
}

// fwd: x [B,H,W,D,Cin] (strided rows), w [Cin][Cout]; the epilogue of m3d_conv3d_fwd
extern "C" int m3d_conv3d_fwd_splitk(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                                     const float* w, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                     int32_t sy, int32_t sx, int32_t sz, const float* bias, const float* bn_scale,
                                     const float* bn_shift, const float* residual, int32_t res_mode, int32_t relu,
                                     float* z_out, float* y, int32_t splits, void* workspace, size_t ws_bytes,
                                     m3d_stream_t s) {
    const int64_t M = B * OH * OW * OD;
    if (splits <= 1 || per_item(B, H * W * D, Cin, OH * OW * OD, Cout))
        return m3d_conv3d_fwd(x, B, H, W, D, Cin, w, 1, 1, 1, Cout, OH, OW, OD, sy, sx, sz, 0, 0, 0, bias,
                              bn_scale, bn_shift, residual, res_mode, relu, z_out, y, Cout, nullptr, 0, 0, s);
    int rc = conv_check(B, H, W, D, Cin, 1, 1, 1, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("conv3d: bn_scale and bn_shift must be given together");
    if (res_mode < 0 || res_mode > 3) return einval("conv3d: res_mode must be 0..3");
    if (relu < 0 || relu > 2) return einval("conv3d: activation must be 0 (none), 1 (relu), 2 (sigmoid)");
    if (res_mode != 0 && residual == nullptr) return einval("conv3d: residual missing");
    if (res_mode == 2 && ((OH & 1) || (OW & 1))) return einval("conv3d: upsampled residual needs even OH/OW");
    if (splits > 64 || Cin % (32 * splits)) return einval("conv3d split-K: Cin must be a multiple of 32 * splits");
    if (!workspace || ws_bytes < sizeof(float) * (size_t)splits * (size_t)M * (size_t)Cout)
        return einval("conv3d split-K: workspace smaller than splits * M * Cout floats");
    const int sp = splits;
    const int64_t slice = Cin / sp;
    float* part = static_cast<float*>(workspace);
    // the K-slices as the batch: channel offset into x's rows and w's rows
    ConvP q{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, 1, 1, 1,
            sy, sx, sz, 0, 0, 0, M, (int)slice, w, (int)Cout, 0, slice, slice * Cout, M * Cout};
    Epi pe{};
    pe.y = part; pe.ldy = Cout; pe.simple = 1; pe.YH = (int)OH; pe.YW = (int)OW; pe.YD = (int)OD;
    pe.ysy = pe.ysx = pe.ysz = 1;
    dispatch_gemm<false, true>(q, pe, st(s), sp);
    rc = check_launch("conv_gemm_kernel(fwd split-K)");
    if (rc) return rc;
    ConvP p{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, 1, 1, 1,
            sy, sx, sz, 0, 0, 0, M, (int)Cin, w, (int)Cout, 0, 0, 0, 0};
    Epi e{bias, bn_scale, bn_shift, residual, res_mode, relu, z_out, y, Cout,
          nullptr, 0, 0, (int)OH, (int)OW, (int)OD, 1, 1, 1, 0, 1};
    hipLaunchKernelGGL(splitk_epi_kernel, dim3(grid_for(M * Cout / 4, 256)), dim3(256), 0, st(s), part, sp, p, e);
    return check_launch("splitk_epi_kernel(fwd)");
}

// bwd-data of a 1x1x1 conv: dx (+)= dz w^T, dz [B,OH,OW,OD,Cout]; the store of m3d_conv3d_bwd_data
extern "C" int m3d_conv3d_bwd_data_splitk(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                          int64_t D, int64_t Cin, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                          int32_t sy, int32_t sx, int32_t sz, float* dx, int32_t accumulate,
                                          int32_t splits, void* workspace, size_t ws_bytes, m3d_stream_t s) {
    const int64_t M = B * OH * OW * OD;
    if (splits <= 1 || per_item(B, H * W * D, Cin, OH * OW * OD, Cout))
        return m3d_conv3d_bwd_data(dz, w, B, H, W, D, Cin, 1, 1, 1, Cout, OH, OW, OD, sy, sx, sz, 0, 0, 0, dx,
                                   accumulate, s);
    int rc = conv_check(B, H, W, D, Cin, 1, 1, 1, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (Cout % 32) return einval("conv3d bwd-data: Cout must be a multiple of 32");
    if (Cin % 4) return einval("conv3d bwd-data: Cin must be a multiple of 4");
    if (splits > 64 || Cout % (32 * splits)) return einval("conv3d split-K: Cout must be a multiple of 32 * splits");
    if (!workspace || ws_bytes < sizeof(float) * (size_t)splits * (size_t)M * (size_t)Cin)
        return einval("conv3d split-K: workspace smaller than splits * M * Cin floats");
    const int sp = splits;
    const int64_t slice = Cout / sp;
    float* part = static_cast<float*>(workspace);
    // M grid = dz grid; B(k = c', n) = w[n][c'] (Keras [Cin][Cout]), slice = channel offset of dz and w
    ConvP q{};
    q.a = dz; q.B = (int)B; q.H = (int)OH; q.W = (int)OW; q.D = (int)OD; q.C = (int)Cout;
    q.OH = (int)OH; q.OW = (int)OW; q.OD = (int)OD;
    q.kh = q.kw = q.kd = 1; q.sy = q.sx = q.sz = 1;
    q.M = M; q.K = (int)slice; q.w = w; q.N = (int)Cin; q.flip = 1;
    q.bsa = slice; q.bsw = slice; q.bsy = M * Cin;
    Epi pe{};
    pe.y = part; pe.ldy = Cin; pe.simple = 1; pe.YH = (int)OH; pe.YW = (int)OW; pe.YD = (int)OD;
    pe.ysy = pe.ysx = pe.ysz = 1;
    dispatch_gemm<true, true>(q, pe, st(s), sp);
    rc = check_launch("conv_gemm_kernel(bwd-data split-K)");
    if (rc) return rc;
    ConvP p = q;
    p.K = (int)Cout; p.bsa = p.bsw = p.bsy = 0;
    Epi e{};
    e.y = dx; e.ldy = Cin; e.accumulate = accumulate;
    e.YH = (int)H; e.YW = (int)W; e.YD = (int)D;
    e.ysy = sy; e.ysx = sx; e.ysz = sz;
    e.simple = (sy == 1 && sx == 1 && sz == 1 && H == OH && W == OW && D == OD);
    hipLaunchKernelGGL(splitk_epi_kernel, dim3(grid_for(M * Cin / 4, 256)), dim3(256), 0, st(s), part, sp, p, e);
    return check_launch("splitk_epi_kernel(bwd-data)");
}

// the split-K form with the fused BN-ReLU backward of the unit whose output dx
// is: the K-slice reduce is bn_act_bwd_kernel summing the slices (stride 1 only)
extern "C" int m3d_conv3d_bwd_data_splitk_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                             int64_t D, int64_t Cin, int64_t Cout, float* dx, int32_t accumulate,
                                             int32_t splits, void* workspace, size_t ws_bytes,
                                             const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes,
                                             m3d_stream_t s) {
    Epi chk{};
    int rc = bn_fuse_epi(bn, Cin, bn_ws, bn_ws_bytes, bn_fuse_rows(B, H, W, D, Cin), chk);
    if (rc) return rc;
    const int64_t M = B * H * W * D;
    if (splits <= 1) return m3d_conv3d_bwd_data_bn(dz, w, B, H, W, D, Cin, 1, 1, 1, Cout, H, W, D, 1, 1, 1, 0, 0,
                                                   0, dx, accumulate, bn, bn_ws, bn_ws_bytes, s);
    if (per_item(B, H * W * D, Cin, H * W * D, Cout))
        return einval("conv3d bwd-data split-K (fused BN backward): batch past the 32-bit operand bound");
    rc = conv_check(B, H, W, D, Cin, 1, 1, 1, Cout, H, W, D, 1, 1, 1);
    if (rc) return rc;
    if (Cout % 32) return einval("conv3d bwd-data: Cout must be a multiple of 32");
    if (splits > 64 || Cout % (32 * splits)) return einval("conv3d split-K: Cout must be a multiple of 32 * splits");
    if (!workspace || ws_bytes < sizeof(float) * (size_t)splits * (size_t)M * (size_t)Cin)
        return einval("conv3d split-K: workspace smaller than splits * M * Cin floats");
    const int64_t slice = Cout / splits;
    ConvP q{};
    q.a = dz; q.B = (int)B; q.H = (int)H; q.W = (int)W; q.D = (int)D; q.C = (int)Cout;
    q.OH = (int)H; q.OW = (int)W; q.OD = (int)D;
    q.kh = q.kw = q.kd = 1; q.sy = q.sx = q.sz = 1;
    q.M = M; q.K = (int)slice; q.w = w; q.N = (int)Cin; q.flip = 1;
    q.bsa = slice; q.bsw = slice; q.bsy = M * Cin;
    Epi pe{};
    pe.y = static_cast<float*>(workspace); pe.ldy = Cin; pe.simple = 1;
    pe.YH = (int)H; pe.YW = (int)W; pe.YD = (int)D;
    pe.ysy = pe.ysx = pe.ysz = 1;
    dispatch_gemm<true, true>(q, pe, st(s), splits);
    rc = check_launch("conv_gemm_kernel(bwd-data split-K, fused BN)");
    if (rc) return rc;
    return bn_act_bwd_splitk(static_cast<const float*>(workspace), splits, M, Cin, bn, dx, accumulate, bn_ws,
                             bn_ws_bytes, st(s));
}

extern "C" int m3d_conv3d_bwd_weight(const float* x, const float* dz, int64_t B, int64_t H,
                                     int64_t W, int64_t D, int64_t Cin, int32_t kh, int32_t kw,
                                     int32_t kd, int64_t Cout, int64_t OH, int64_t OW, int64_t OD,
                                     int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px,
                                     int32_t pz, float* dw, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    int rc = conv_check(B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (per_item(B, H * W * D, Cin, OH * OW * OD, Cout)) {      // dw accumulates over the items
        for (int64_t b = 0; b < B; ++b) {
            rc = m3d_conv3d_bwd_weight(x + b * H * W * D * Cin, dz + b * OH * OW * OD * Cout, 1, H, W, D, Cin, kh,
                                       kw, kd, Cout, OH, OW, OD, sy, sx, sz, py, px, pz, dw, det, s);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    ConvP p{x, (int)B, (int)H, (int)W, (int)D, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), nullptr,
            (int)Cout, 0, 0, 0, 0};
    const bool vec = (Cin % 4) == 0;
    if (stem_ok(Cin, kh, kw, kd, Cout, sy, sx, sz, 1, 1, 1, 0, 0, 0))
        return launch_stem_wgrad(p, dz, dw, st(s));
    // 1x1x1 stride-1 convs: im2col is x itself, the plain weight-gradient GEMM
    // dW += x^T dz -- on the exact bf16 split like the Winograd ones
    // M3D_WGRAD1_X3_MIN_N: smallest Cout taking this path (A/B: 65 = round 2's Cout > 64)
    static constexpr int min_n = M3D_TUNE_WGRAD1_X3_MIN_N;
    if (vec && ((x3_mask() >> 3) & 1) && kh == 1 && kw == 1 && kd == 1 && sy == 1 && sx == 1 && sz == 1 &&
        py == 0 && px == 0 && pz == 0 && OH == H && OW == W && OD == D && Cout >= min_n) {
        launch_wgrad_x3(x, dz, dw, p.M, (int)Cin, (int)Cout, 1, 0, 0, 0, st(s));
        return check_launch("x3_wgrad_kernel (1x1x1)");
    }
    if (vec && p.K <= 64) {        // e.g. the 64 -> 256 1x1 convs of stage 2
        if (Cout <= 64) launch_wgrad<64, 64, 2, 2, true>(p, dz, dw, st(s));
        else launch_wgrad<64, 128, 2, 2, true>(p, dz, dw, st(s));
    } else if (Cout <= 64) {
        if (vec) launch_wgrad<128, 64, 2, 2, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 64, 2, 2, false>(p, dz, dw, st(s));
    } else {
        if (vec) launch_wgrad<128, 128, 2, 2, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 128, 2, 2, false>(p, dz, dw, st(s));
    }
    return check_launch("conv_wgrad_kernel");
}

// ---- depth-slab forms of the direct convs: halo planes beside the slab ---------
// x [B,H,W,Dl,Cin] is the local slab, halo [B,H,W,2r,Cin] the neighbours' r
// boundary planes (has_lo / has_hi: that neighbour exists); the conv is the
// 'same' z window kd = 2r+1 at z-stride 1 with pad pz = r where the volume ends,
// OD = Dl -- the same taps and sums as on the halo-extended copy of the slab.
static int conv_halo_geom(ConvP& p, const float* halo, int32_t has_lo, int32_t has_hi, int32_t r, int64_t Dl,
                          int32_t kd, int32_t sz, int32_t pz, int64_t OD) {
    if (!halo) return einval("conv3d halo: null halo planes");
    if (r <= 0 || kd != 2 * r + 1 || sz != 1 || pz != r || OD != Dl || Dl < r)
        return einval("conv3d halo: z window must be 'same' 2r+1 at stride 1 on a slab of >= r planes");
    const int nlo = has_lo ? r : 0, nhi = has_hi ? r : 0;
    p.D = (int)(Dl + nlo + nhi);
    p.pz = pz - nlo;
    p.halo = halo;
    p.hnlo = nlo;
    p.hdl = (int)Dl;
    p.hr = r;
    return M3D_OK;
}

// The one-channel 7^3 stem (stem_fwd_kernel) on a depth slab.
extern "C" int m3d_conv3d_fwd_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi, int32_t r,
                                   int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin, const float* w,
                                   int32_t kh, int32_t kw, int32_t kd, int64_t Cout, int64_t OH, int64_t OW,
                                   int64_t OD, int32_t sy, int32_t sx, int32_t sz, int32_t py, int32_t px, int32_t pz,
                                   const float* bias, const float* bn_scale, const float* bn_shift, int32_t relu,
                                   float* z_out, float* y, m3d_stream_t s) {
    int rc = conv_check(B, H, W, Dl, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (!stem_ok(Cin, kh, kw, kd, Cout, sy, sx, sz, 1, 1, 1, 0, 0, 0))
        return einval("conv3d_fwd_halo: only the one-channel 7^3 stem (1 -> 64, strides (2,2,1)) has a halo form");
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("conv3d: bn_scale and bn_shift must be given together");
    if (relu < 0 || relu > 2) return einval("conv3d: activation must be 0 (none), 1 (relu), 2 (sigmoid)");
    if (B * H * W * (Dl + 2 * r) * Cin >= op_lim() || B * OH * OW * OD * Cout >= op_lim())
        return einval("conv3d_fwd_halo: operand larger than 4 GiB (32-bit buffer offsets)");
    ConvP p{x, (int)B, (int)H, (int)W, (int)Dl, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), w, (int)Cout, 0, 0, 0, 0};
    if ((rc = conv_halo_geom(p, halo, has_lo, has_hi, r, Dl, kd, sz, pz, OD))) return rc;
    Epi e{bias, bn_scale, bn_shift, nullptr, 0, relu, z_out, y, Cout, nullptr, 0, 0, (int)OH, (int)OW, (int)OD,
          1, 1, 1, 0, 1};
    return launch_stem(p, e, st(s));
}

// The direct weight gradient (conv_wgrad_kernel) on a depth slab: the stem's
// and the 64-channel 3^3 convs' (whose weight gradient is not Winograd).
extern "C" int m3d_conv3d_bwd_weight_halo(const float* x, const float* halo, int32_t has_lo, int32_t has_hi,
                                          int32_t r, const float* dz, int64_t B, int64_t H, int64_t W, int64_t Dl,
                                          int64_t Cin, int32_t kh, int32_t kw, int32_t kd, int64_t Cout,
                                          int64_t OH, int64_t OW, int64_t OD, int32_t sy, int32_t sx, int32_t sz,
                                          int32_t py, int32_t px, int32_t pz, float* dw, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    int rc = conv_check(B, H, W, Dl, Cin, kh, kw, kd, Cout, OH, OW, OD, sy, sx, sz);
    if (rc) return rc;
    if (B * H * W * (Dl + 2 * r) * Cin >= op_lim() || B * OH * OW * OD * Cout >= op_lim())
        return einval("conv3d_bwd_weight_halo: operand larger than 4 GiB (32-bit buffer offsets)");
    ConvP p{x, (int)B, (int)H, (int)W, (int)Dl, (int)Cin, (int)OH, (int)OW, (int)OD, kh, kw, kd,
            sy, sx, sz, py, px, pz, B * OH * OW * OD, (int)(kh * kw * kd * Cin), nullptr,
            (int)Cout, 0, 0, 0, 0};
    if ((rc = conv_halo_geom(p, halo, has_lo, has_hi, r, Dl, kd, sz, pz, OD))) return rc;
    if (stem_ok(Cin, kh, kw, kd, Cout, sy, sx, sz, 1, 1, 1, 0, 0, 0))
        return launch_stem_wgrad(p, dz, dw, st(s));
    const bool vec = (Cin % 4) == 0;
    if (Cout <= 64) {
        if (vec) launch_wgrad<128, 64, 2, 2, true, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 64, 2, 2, false, true>(p, dz, dw, st(s));
    } else {
        if (vec) launch_wgrad<128, 128, 2, 2, true, true>(p, dz, dw, st(s));
        else launch_wgrad<128, 128, 2, 2, false, true>(p, dz, dw, st(s));
    }
    return check_launch("conv_wgrad_kernel<halo>");
}

// ---- Winograd entry points -------------------------------------------------
// x depth D, output depth OD, z pad-before pz: 'same' is OD == D, pz == 1; a
// z-halo-extended depth slab has D = OD + halos and pz = 1 - (lower halo).
static int wino_check(int64_t B, int64_t H, int64_t W, int64_t D, int64_t OD, int32_t pz,
                      int64_t Cin, int64_t Cout) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0 || OD <= 0 || Cin <= 0 || Cout <= 0)
        return einval("conv3d winograd: tensor dimensions must be positive");
    if (Cin % 32 || Cout % 32) return einval("conv3d winograd: Cin and Cout must be multiples of 32");
    if (pz < 0 || pz > 1 || D - OD < 0 || D - OD > 2)
        return einval("conv3d winograd: z geometry must be pz in {0,1} and 0 <= D - OD <= 2");
    if (H * W * (D > OD ? D : OD) > 0x7FFFFFFF) return einval("conv3d winograd: more than 2^31 voxels");
    // the input transform reads x / dz through 32-bit buffer offsets (per batch
    // item: a larger batch runs one item at a time, see op_lim)
    if (H * W * (D > OD ? D : OD) * (Cin > Cout ? Cin : Cout) >= op_lim())
        return einval("conv3d winograd: operand of one batch item larger than 4 GiB (32-bit buffer offsets)");
    return M3D_OK;
}

static bool wino_per_item(int64_t B, int64_t H, int64_t W, int64_t D, int64_t OD, int64_t Cin, int64_t Cout) {
    return per_item(B, H * W * (D > OD ? D : OD), Cin > Cout ? Cin : Cout, 0, 0);
}
// Workspace: V [P][Cin][Cout] + U [P][T][C1] + M [P][T][C2] (P = 16*(NZ+2) points) with
// {C1, C2} = {Cin, Cout} (fwd / wgrad) or {Cout, Cin} (bwd-data), T the larger
// of the fwd (tiles over OD) and bwd-data (tiles over D) tile counts.
// launch the F(2x2xNZ) instantiation of a Winograd transform kernel
#define WINO_LAUNCH_NZ(nz, kern, ...)                                            \
    do {                                                                         \
        if ((nz) == 4) hipLaunchKernelGGL(kern<4>, __VA_ARGS__);                 \
        else hipLaunchKernelGGL(kern<2>, __VA_ARGS__);                           \
    } while (0)
#define WINO_LAUNCH(kern, ...) WINO_LAUNCH_NZ(wino_nz(), kern, __VA_ARGS__)

extern "C" int32_t m3d_conv3d_wino_tile_z(void) { return wino_nz(); }
extern "C" int32_t m3d_conv3d_wino_wgrad_tile_z(void) { return wino_wgrad_nz(); }
extern "C" int32_t m3d_conv3d_wino_tile_y(void) { return WNY; }
extern "C" int32_t m3d_conv3d_wino_dgrad_tile_y(void) { return wino_dgrad_ny(); }
extern "C" int32_t m3d_conv3d_wino_dgrad_tile_z(void) { return wino_dgrad_nz(); }

extern "C" size_t m3d_conv3d_wino_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D,
                                                  int64_t OD, int64_t Cin, int64_t Cout) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    if (wino_per_item(B, H, W, D, OD, Cin, Cout)) B = 1;     // run one batch item at a time
    size_t best = 0;
    // the data gradient's y tile is a per-call argument (m3d_conv3d_bwd_data_wino_vy / _bny): both sizes
    const int tiles[4][2] = {{wino_nz(), WNY}, {wino_wgrad_nz(), WNY}, {wino_dgrad_nz(), 2}, {wino_dgrad_nz(), 4}};
    for (const auto& zy : tiles) {
        const int nz = zy[0], ny = zy[1];
        const WinoGeom g = wino_geom(B, H, W, D > OD ? D : OD, D, 1, nz, ny);
        const size_t P = (size_t)wino_points(nz, ny);
        const size_t eb = gemm_x3_env() ? 6 : 4;      // X3: V and U hold three bf16 planes
        const size_t wt = gemm_x3_env() ? al(sizeof(float) * 27 * (size_t)Cin * Cout) : 0;
        // U (eb bytes / element) then M (fp32), in either role order (fwd: U over
        // Cin, M over Cout; bwd-data: the reverse)
        const size_t um1 = al(eb * P * (size_t)g.T * Cin) + al(4 * P * (size_t)g.T * Cout);
        const size_t um2 = al(eb * P * (size_t)g.T * Cout) + al(4 * P * (size_t)g.T * Cin);
        const size_t b = wt + al(eb * P * (size_t)Cin * Cout) + (um1 > um2 ? um1 : um2);
        best = b > best ? b : best;
    }
    return best;
}

struct WinoWs { float *V, *U, *M, *WT; };
// bytes wino_ws lays out for geometry g, operand widths C1 (U) / C2 (M) and the tile (nz, ny)
static size_t wino_ws_need(const WinoGeom& g, int64_t C1, int64_t C2, int nz, int ny) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t P = (size_t)wino_points(nz, ny);
    const size_t eb = gemm_x3_env() ? 6 : 4;
    const size_t wt = gemm_x3_env() ? al(sizeof(float) * 27 * (size_t)C1 * C2) : 0;
    return wt + al(eb * P * (size_t)C1 * C2) + al(eb * P * (size_t)g.T * C1) + al(4 * P * (size_t)g.T * C2);
}
// the data gradient's own workspace at tile_y (0: the library default): the
// layout bwd_data_wino checks (dz transformed over Cout, dx's points over Cin)
extern "C" size_t m3d_conv3d_wino_dgrad_workspace_bytes(int64_t B, int64_t H, int64_t W, int64_t D, int64_t OD,
                                                        int64_t Cin, int64_t Cout, int32_t tile_y) {
    if (tile_y != 0 && tile_y != 2 && tile_y != 4) return 0;
    if (wino_per_item(B, H, W, D, OD, Cin, Cout)) B = 1;
    const int nz = wino_dgrad_nz(), ny = tile_y ? tile_y : wino_dgrad_ny();
    return wino_ws_need(wino_geom(B, H, W, D, OD, 1, nz, ny), Cout, Cin, nz, ny);
}
// [WT: X3 only, the transposed kernel][V][U][M]
static WinoWs wino_ws(void* ws, const WinoGeom& g, int64_t Cin, int64_t Cout, int nz = -1, int ny = WNY) {
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t P = (size_t)wino_points(nz < 0 ? wino_nz() : nz, ny);
    char* p = (char*)ws;
    WinoWs w{};
    w.WT = (float*)p;
    if (gemm_x3_env()) p += al(sizeof(float) * 27 * (size_t)Cin * Cout);
    const size_t eb = gemm_x3_env() ? 6 : 4;
    w.V = (float*)p; p += al(eb * P * (size_t)Cin * Cout);
    w.U = (float*)p; p += al(eb * P * (size_t)g.T * Cin);
    w.M = (float*)p;
    return w;
}

#define WINO_LAUNCH_NZ_X3(nz, kern, ...)                                         \
    do {                                                                         \
        if ((nz) == 4) hipLaunchKernelGGL((kern<4, true>), __VA_ARGS__);         \
        else hipLaunchKernelGGL((kern<2, true>), __VA_ARGS__);                   \
    } while (0)
// the input transform, reading a depth slab's halo planes when g.halo is set
#define WINO_INPUT(nz, x3o, grid, s, x, g, C, U)                                                          \
    do {                                                                                                   \
        const bool h_ = (g).halo != nullptr;                                                               \
        if ((nz) == 4) {                                                                                   \
            if (x3o) { if (h_) hipLaunchKernelGGL((wino_input_kernel<4, true, true>), grid, dim3(256), 0, s, x, g, C, U); \
                       else hipLaunchKernelGGL((wino_input_kernel<4, true, false>), grid, dim3(256), 0, s, x, g, C, U); } \
            else { if (h_) hipLaunchKernelGGL((wino_input_kernel<4, false, true>), grid, dim3(256), 0, s, x, g, C, U); \
                   else hipLaunchKernelGGL((wino_input_kernel<4, false, false>), grid, dim3(256), 0, s, x, g, C, U); } \
        } else {                                                                                           \
            if (x3o) { if (h_) hipLaunchKernelGGL((wino_input_kernel<2, true, true>), grid, dim3(256), 0, s, x, g, C, U); \
                       else hipLaunchKernelGGL((wino_input_kernel<2, true, false>), grid, dim3(256), 0, s, x, g, C, U); } \
            else { if (h_) hipLaunchKernelGGL((wino_input_kernel<2, false, true>), grid, dim3(256), 0, s, x, g, C, U); \
                   else hipLaunchKernelGGL((wino_input_kernel<2, false, false>), grid, dim3(256), 0, s, x, g, C, U); } \
        }                                                                                                  \
    } while (0)

static int x3_af32_env() { return (x3_mask() >> 4) & 1; }

// the P point GEMMs M[xi] = U[xi] V[xi] on split planes (U: T x K, V: N x K);
// af32: U is fp32 [P][T][K] (split in the GEMM's LDS store)
static void wino_gemm_x3(const WinoWs& ws, int64_t T, int K, int N, int P, hipStream_t s,
                         bool af32 = false) {
    X3G q{};                   // (value-initialised: q.ep.on = 0, the plain C store)
    q.a = reinterpret_cast<const unsigned short*>(ws.U);
    q.af = ws.U;
    q.b = reinterpret_cast<const unsigned short*>(ws.V);
    q.c = ws.M;
    q.M = T; q.K = K; q.N = N; q.nbatch = P;
    q.psa = (int64_t)P * T * K; q.psb = (int64_t)P * K * N;
    q.bsa = T * K; q.bsb = (int64_t)K * N; q.bsc = T * N;
    // the 256x256 kernels where N fills whole 256-column tiles (x3_gemm256_kernel:
    // 1.345 vs 1.368 ms on the priced launch against the 128x128 kernel)
    if (N % 256 == 0 && T >= 256) {
        const int64_t t256 = ((T + 255) / 256) * (N / 256) * P;
        const dim3 grid((unsigned)(t256 < 65536 ? t256 : 65536), (unsigned)((t256 + 65535) / 65536));
        if (af32) hipLaunchKernelGGL(x3_gemm256_af_kernel<0>, grid, dim3(512), 0, s, q);
        else hipLaunchKernelGGL(x3_gemm256_kernel<0>, grid, dim3(512), 0, s, q);
        return;
    }
    if (N == 64) {             // 128x64 tiles (the res2 64-channel layers)
        const int64_t tiles = ((T + 127) / 128) * P;
        if (af32) hipLaunchKernelGGL((x3_gemm_kernel<32, false, 2, true, 64>), dim3((unsigned)tiles), dim3(256), 0, s, q);
        else hipLaunchKernelGGL((x3_gemm_kernel<32, false, 3, false, 64>), dim3((unsigned)tiles), dim3(256), 0, s, q);
        return;
    }
    // 128x128 tiles, BK 32, 3 blocks per CU (2 with A in fp32)
    const int64_t tiles = ((T + 127) / 128) * ((N + 127) / 128) * P;
    if (af32) hipLaunchKernelGGL((x3_gemm_kernel<32, false, 2, true>), dim3((unsigned)tiles), dim3(256), 0, s, q);
    else hipLaunchKernelGGL((x3_gemm_kernel<32, false, 3>), dim3((unsigned)tiles), dim3(256), 0, s, q);
}

// x -> three bf16 planes of split3 (planes at x3 + p * n), one element per thread
__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, int64_t n,
                                                     unsigned short* __restrict__ x3) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t h, m, l;
    split3(x[i], h, m, l);
    x3[i] = (unsigned short)h;
    x3[n + i] = (unsigned short)m;
    x3[2 * n + i] = (unsigned short)l;
}

extern "C" int m3d_split3_f32(const float* x, int64_t n, uint16_t* x3, m3d_stream_t s) {
    if (n <= 0) return einval("split3: n must be positive");
    hipLaunchKernelGGL(split3_kernel, dim3(grid_for(n, 256)), dim3(256), 0, st(s), x, n,
                       reinterpret_cast<unsigned short*>(x3));
    return check_launch("split3_kernel");
}

extern "C" int m3d_gemm_x3(const uint16_t* A3, const uint16_t* B3, float* C, int64_t batch, int64_t M,
                           int64_t K, int64_t N, m3d_stream_t s) {
    if (batch <= 0 || M <= 0 || K <= 0 || N <= 0) return einval("gemm_x3: dimensions must be positive");
    if (K % 32 || N % 4) return einval("gemm_x3: K must be a multiple of 32 and N of 4");
    if (M > 0x7FFFFFFF || M * K * 2 >= 0xFFFFFFF0LL || N * K * 2 >= 0xFFFFFFF0LL || M * N * 4 >= 0xFFFFFFF0LL)
        return einval("gemm_x3: operand larger than 4 GiB (32-bit buffer offsets)");
    WinoWs ws{};
    ws.U = (float*)const_cast<uint16_t*>(A3);
    ws.V = (float*)const_cast<uint16_t*>(B3);
    ws.M = C;
    ws.WT = nullptr;
    wino_gemm_x3(ws, M, (int)K, (int)N, (int)batch, st(s));
    return check_launch("m3d_gemm_x3");
}

extern "C" int m3d_gemm_x3_af(const float* A, const uint16_t* B3, float* C, int64_t batch, int64_t M, int64_t K,
                              int64_t N, m3d_stream_t s) {
    if (batch <= 0 || M <= 0 || K <= 0 || N <= 0) return einval("gemm_x3_af: dimensions must be positive");
    if (K % 32 || N % 4) return einval("gemm_x3_af: K must be a multiple of 32 and N of 4");
    if (!A || !B3 || !C) return einval("gemm_x3_af: null operand");
    if (M > 0x7FFFFFFF || M * K * 4 >= 0xFFFFFFF0LL || N * K * 2 >= 0xFFFFFFF0LL || M * N * 4 >= 0xFFFFFFF0LL)
        return einval("gemm_x3_af: operand larger than 4 GiB (32-bit buffer offsets)");
    WinoWs ws{};
    ws.U = const_cast<float*>(A);
    ws.V = (float*)const_cast<uint16_t*>(B3);
    ws.M = C;
    ws.WT = nullptr;
    wino_gemm_x3(ws, M, (int)K, (int)N, (int)batch, st(s), true);
    return check_launch("m3d_gemm_x3_af");
}


// ---- 1x1x1 stride-1 convs as one GEMM on the exact bf16 split --------------
// The big-K 1x1x1 convs at the finest level (rpn_conv_shared2 512 -> 256, the
// P2 lateral 256 -> 256 and their data gradients) are f32-MFMA-bound in the
// direct kernel; as a GEMM rows = voxels, A = x (or dz) rows of K fp32
// channels split in registers, B = the weight as split planes, they run on
// x3_gemm256_af_kernel, the conv epilogue applied by a second pass.
// planes[p][n][k] = split3_p(w[k][n]) (transpose = 1: the forward, K = Cin,
// N = Cout) or split3_p(w[n][k]) (transpose = 0: the data gradient, N = Cin,
// K = Cout); w is the Keras [Cin][Cout] kernel.
__global__ __launch_bounds__(256) void x3_wplanes_kernel(const float* __restrict__ w, int Cin, int Cout,
                                                         int transpose, unsigned short* __restrict__ pl) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_el = (int64_t)Cin * Cout;
    if (i >= n_el) return;
    const int c = (int)(i / Cout), o = (int)(i % Cout);   // w[c][o]
    uint32_t h, m, l;
    split3(w[i], h, m, l);
    const int64_t at = transpose ? (int64_t)o * Cin + c : i;
    pl[at] = (unsigned short)h;
    pl[n_el + at] = (unsigned short)m;
    pl[2 * n_el + at] = (unsigned short)l;
}

extern "C" int m3d_conv1_x3_planes(const float* w, int64_t Cin, int64_t Cout, int32_t transpose, uint16_t* planes,
                                   m3d_stream_t s) {
    if (Cin <= 0 || Cout <= 0 || !w || !planes) return einval("conv1_x3_planes: bad arguments");
    hipLaunchKernelGGL(x3_wplanes_kernel, dim3(grid_for(Cin * Cout, 256)), dim3(256), 0, st(s), w, (int)Cin,
                       (int)Cout, transpose ? 1 : 0, reinterpret_cast<unsigned short*>(planes));
    return check_launch("x3_wplanes_kernel");
}

// Both orientations of every listed kernel in one launch (grid (ceil(max
// Cin*Cout / 256), n)): each element split once, its three planes stored
// transposed into fwd and in place into bwd (either may be NULL) -- the same
// bits as x3_wplanes_kernel per orientation.
__global__ __launch_bounds__(256) void x3_wplanes_batched_kernel(const m3d_x3_planes_item_t* __restrict__ items) {
    const m3d_x3_planes_item_t it = items[blockIdx.y];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t n_el = (int64_t)it.cin * it.cout;
    if (i >= n_el) return;
    const int c = (int)(i / it.cout), o = (int)(i % it.cout);
    uint32_t h, m, l;
    split3(it.w[i], h, m, l);
    if (it.fwd) {
        unsigned short* pl = reinterpret_cast<unsigned short*>(it.fwd);
        const int64_t at = (int64_t)o * it.cin + c;
        pl[at] = (unsigned short)h;
        pl[n_el + at] = (unsigned short)m;
        pl[2 * n_el + at] = (unsigned short)l;
    }
    if (it.bwd) {
        unsigned short* pl = reinterpret_cast<unsigned short*>(it.bwd);
        pl[i] = (unsigned short)h;
        pl[n_el + i] = (unsigned short)m;
        pl[2 * n_el + i] = (unsigned short)l;
    }
}

extern "C" int m3d_conv1_x3_planes_batched(const m3d_x3_planes_item_t* items, int32_t n, int64_t max_el,
                                           m3d_stream_t s) {
    if (n <= 0 || n > 65535 || max_el <= 0 || max_el > 0x7FFFFFFF || !items)
        return einval("conv1_x3_planes_batched: bad arguments");
    hipLaunchKernelGGL(x3_wplanes_batched_kernel, dim3(grid_for(max_el, 256), (unsigned)n), dim3(256), 0, st(s),
                       items);
    return check_launch("x3_wplanes_batched_kernel");
}

// the GEMM on x3_gemm256_af_kernel (plain C = out [M][N]), then -- when the
// conv has an epilogue -- splitk_epi_kernel over `out` in place (one slice):
// each element read once and rewritten through epi_store4.  (The epilogue
// inside the GEMM kernel spilled: its 222 VGPRs leave no room.)
static int conv1_x3_launch(const float* a, const uint16_t* planes, int64_t M, int64_t K, int64_t N, int64_t H,
                           int64_t W, int64_t D, float* out, const Epi* e, hipStream_t s) {
    if (M <= 0 || K <= 0 || N <= 0) return einval("conv1 x3: dimensions must be positive");
    if (K % 32 || N % 256) return einval("conv1 x3: K must be a multiple of 32 and N of 256");
    if (M > 0x7FFFFFFF || M * K >= op_lim() || M * N >= op_lim() || N * K * 2 >= 0xFFFFFFF0LL)
        return einval("conv1 x3: operand larger than 4 GiB (32-bit buffer offsets)");
    X3G q{};
    q.af = a;
    q.b = reinterpret_cast<const unsigned short*>(planes);
    q.c = out;
    q.M = M; q.K = (int)K; q.N = (int)N; q.nbatch = 1;
    q.psb = K * N;
    const int64_t t256 = ((M + 255) / 256) * (N / 256);
    const dim3 grid((unsigned)(t256 < 65536 ? t256 : 65536), (unsigned)((t256 + 65535) / 65536));
    // the epilogue in the GEMM's own stores when it is element-local (same-shape
    // residual); the FPN's upsampled residual (res_mode 2) takes the second pass
    const bool fuse = e && e->res_mode <= 1 && !e->accumulate && e->split <= 0 &&
                      e->ldy == N && e->simple;
    if (fuse) {
        q.ep.bias = e->bias; q.ep.scale = e->scale; q.ep.shift = e->shift;
        q.ep.res = e->res_mode == 1 ? e->res : nullptr; q.ep.z = e->z; q.ep.act = e->relu; q.ep.on = 1;
    }
    if (fuse) hipLaunchKernelGGL(x3_gemm256_af_kernel<1>, grid, dim3(512), 0, s, q);
    else hipLaunchKernelGGL(x3_gemm256_af_kernel<0>, grid, dim3(512), 0, s, q);
    int rc = check_launch("x3_gemm256_af_kernel(conv1)");
    if (rc || !e || fuse) return rc;
    ConvP p{};
    p.M = M; p.N = (int)N; p.K = (int)K; p.OH = (int)H; p.OW = (int)W; p.OD = (int)D;
    hipLaunchKernelGGL(splitk_epi_kernel, dim3(grid_for(M * N / 4, 256)), dim3(256), 0, s, out, 1, p, *e);
    return check_launch("splitk_epi_kernel(conv1 x3)");
}

extern "C" int m3d_conv3d_fwd_x3(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                                 const uint16_t* planes, int64_t Cout, const float* bias, const float* bn_scale,
                                 const float* bn_shift, const float* residual, int32_t res_mode, int32_t relu,
                                 float* z_out, float* y, m3d_stream_t s) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0) return einval("conv3d x3: tensor dimensions must be positive");
    if ((bn_scale == nullptr) != (bn_shift == nullptr))
        return einval("conv3d: bn_scale and bn_shift must be given together");
    if (res_mode < 0 || res_mode > 2) return einval("conv3d x3: res_mode must be 0..2");
    if (relu < 0 || relu > 2) return einval("conv3d: activation must be 0 (none), 1 (relu), 2 (sigmoid)");
    if (res_mode != 0 && residual == nullptr) return einval("conv3d: residual missing");
    if (res_mode == 2 && ((H & 1) || (W & 1))) return einval("conv3d: upsampled residual needs even OH/OW");
    Epi e{};
    e.bias = bias; e.scale = bn_scale; e.shift = bn_shift; e.res = residual; e.res_mode = res_mode;
    e.relu = relu; e.z = z_out; e.y = y; e.ldy = Cout; e.simple = 1;
    e.YH = (int)H; e.YW = (int)W; e.YD = (int)D; e.ysy = e.ysx = e.ysz = 1;
    const bool plain = !bias && !bn_scale && !residual && !relu && !z_out;
    return conv1_x3_launch(x, planes, B * H * W * D, Cin, Cout, H, W, D, y, plain ? nullptr : &e, st(s));
}

// dx = dz w^T (accumulate = 0 only: the GEMM's plain store)
extern "C" int m3d_conv3d_bwd_data_x3(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W,
                                      int64_t D, int64_t Cin, int64_t Cout, float* dx, m3d_stream_t s) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0) return einval("conv3d x3: tensor dimensions must be positive");
    return conv1_x3_launch(dz, planes, B * H * W * D, Cout, Cin, H, W, D, dx, nullptr, st(s));
}

// m3d_conv3d_bwd_data_x3 with the fused BN-ReLU backward of the unit that made
// x (m3d_conv3d_bwd_data_bn's contract, accumulate 0): the GEMM's epilogue
// applies it to each element (dz into dx, dpre into bn->dres) and writes the
// channel sums of each 128-row half tile; bn_sums_reduce folds them in row order.
static int bwd_data_x3_bn(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W, int64_t D,
                          int64_t Cin, int64_t Cout, float* dx, int32_t accumulate, const m3d_bn_bwd_t* bn,
                          void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s) {
    if (B <= 0 || H <= 0 || W <= 0 || D <= 0) return einval("conv3d x3: tensor dimensions must be positive");
    const int64_t M = B * H * W * D;
    if (Cout % 32 || Cin % 256) return einval("conv1 x3: K must be a multiple of 32 and N of 256");
    if (M > 0x7FFFFFFF || M * Cout >= op_lim() || M * Cin >= op_lim() || Cin * Cout * 2 >= 0xFFFFFFF0LL)
        return einval("conv1 x3: operand larger than 4 GiB (32-bit buffer offsets)");
    const int64_t rows = 2 * ((M + 255) / 256);           // one partial row per 128-row half tile
    Epi e{};
    int rc = bn_fuse_epi(bn, Cin, bn_ws, bn_ws_bytes, rows, e);
    if (rc) return rc;
    X3G q{};
    q.af = dz;
    q.b = reinterpret_cast<const unsigned short*>(planes);
    q.c = dx;
    q.M = M; q.K = (int)Cout; q.N = (int)Cin; q.nbatch = 1;
    q.psb = Cout * Cin;
    q.ep.on = 2;
    q.ep.fy = e.fy; q.ep.fz = e.fz; q.ep.fscale = e.fscale; q.ep.fmean = e.fmean; q.ep.frstd = e.frstd;
    q.ep.fdres = e.fdres; q.ep.fpart = e.fpart; q.ep.fprows = rows; q.ep.frelu = e.frelu;
    q.ep.facc = accumulate ? 1 : 0;
    const int64_t t256 = (rows / 2) * (Cin / 256);
    const dim3 grid((unsigned)(t256 < 65536 ? t256 : 65536), (unsigned)((t256 + 65535) / 65536));
    hipLaunchKernelGGL(x3_gemm256_af_kernel<2>, grid, dim3(512), 0, st(s), q);
    rc = check_launch("x3_gemm256_af_kernel(conv1 bwd-data, fused BN backward)");
    if (rc || !e.fpart) return rc;
    return bn_sums_reduce(e.fpart, rows, Cin, bn->sum_dpre, bn->sum_dpre_xhat, bn->sum_dz, st(s));
}

extern "C" int m3d_conv3d_bwd_data_x3_bn(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W,
                                         int64_t D, int64_t Cin, int64_t Cout, float* dx, const m3d_bn_bwd_t* bn,
                                         void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s) {
    return bwd_data_x3_bn(dz, planes, B, H, W, D, Cin, Cout, dx, 0, bn, bn_ws, bn_ws_bytes, s);
}

extern "C" int m3d_conv3d_bwd_data_x3_bna(const float* dz, const uint16_t* planes, int64_t B, int64_t H, int64_t W,
                                          int64_t D, int64_t Cin, int64_t Cout, float* dx, int32_t accumulate,
                                          const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes, m3d_stream_t s) {
    return bwd_data_x3_bn(dz, planes, B, H, W, D, Cin, Cout, dx, accumulate, bn, bn_ws, bn_ws_bytes, s);
}

extern "C" size_t m3d_conv3d_wino_u_bytes(int64_t B, int64_t H, int64_t W, int64_t OD, int64_t Cin) {
    if (wino_nz() != wino_wgrad_nz()) return 0;       // forward tiles differ from the wgrad's: nothing to keep
    if (gemm_x3_env() && !x3_af32_env()) return 0;     // the forward's U is in bf16 planes
    return sizeof(float) * wino_points() * (size_t)wino_geom(B, H, W, OD, OD, 1).T * (size_t)Cin;
}

static int fwd_wino(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                    const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                    const float* bn_scale, const float* bn_shift, const float* residual,
                    int32_t relu, float* z_out, float* y, float* u_keep, void* workspace,
                    size_t ws_bytes, hipStream_t s, const float* halo = nullptr, int hlo = 0, int hhi = 0,
                    bool v_ready = false, int phase = 0, const void* v_ext = nullptr) {
    int rc = wino_check(B, H, W, D, OD, pz, Cin, Cout);
    if (rc) return rc;
    if (ws_bytes < m3d_conv3d_wino_workspace_bytes(B, H, W, D, OD, Cin, Cout))
        return einval("conv3d winograd: workspace too small");
    if (phase && wino_per_item(B, H, W, D, OD, Cin, Cout))
        return einval("conv3d winograd: a phased launch needs a batch within the 32-bit operand bound");
    if (wino_per_item(B, H, W, D, OD, Cin, Cout)) {
        if (u_keep) return einval("conv3d winograd: u_keep with a batch past the 32-bit operand bound");
        const int64_t os = H * W * OD * Cout;
        for (int64_t b = 0; b < B; ++b) {
            rc = fwd_wino(x + b * H * W * D * Cin, 1, H, W, D, Cin, w, Cout, OD, pz, bias, bn_scale, bn_shift,
                          residual ? residual + b * os : nullptr, relu, z_out ? z_out + b * os : nullptr, y + b * os,
                          nullptr, workspace, ws_bytes, s, halo ? halo + b * H * W * 2 * Cin : nullptr, hlo, hhi,
                          v_ready || b > 0, 0, v_ext);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    WinoGeom g = wino_geom(B, H, W, OD, D, pz);
    g.halo = halo; g.hlo = hlo; g.hhi = hhi;
    WinoWs ws = wino_ws(workspace, g, Cin, Cout);
    // phase 1 (depth slab, halo exchange in flight): weight transform + the
    // interior z tiles' input transform (no halo plane in their windows);
    // phase 2: the first / last z tiles (halo planes now present), GEMM, output
    WinoGeom gi = g, ge = g;
    if (phase) {
        gi.tz_mode = 1; gi.halo = nullptr; gi.hlo = gi.hhi = 0;
        ge.tz_mode = 2;
    }
    if (gemm_x3_env() && (!u_keep || x3_af32_env())) {
        // (the fp32-A GEMM reads U in fp32: a kept U is written in place for the weight gradient)
        if (u_keep) ws.U = u_keep;
        if (v_ext) ws.V = static_cast<float*>(const_cast<void*>(v_ext));   // transformed by m3d_conv3d_wino_weight_v
        float* wt = ws.WT;
        if (!v_ready && !v_ext && phase != 2) {   // v_ready: V already holds this w's transform (an earlier call, same workspace)
            hipLaunchKernelGGL(x3_wt_kernel, dim3((unsigned)((Cout + 31) / 32), (unsigned)((Cin + 31) / 32), 27),
                               dim3(256), 0, s, w, (int)Cin, (int)Cout, wt);
            WINO_LAUNCH_NZ_X3(wino_nz(), wino_weight_kernel, dim3(grid_for(Cin * Cout, 256)), dim3(256), 0, s, wt,
                              (int)Cin, (int)Cout, 0, ws.V);
        }
        const bool af32 = x3_af32_env();
        if (phase == 1) {
            WINO_INPUT(wino_nz(), !af32, dim3(grid_for(g.T * Cin, 256)), s, x, gi, (int)Cin, ws.U);
            return check_launch("conv3d winograd fwd (x3, phase 1)");
        }
        if (phase == 2) WINO_INPUT(wino_nz(), !af32, dim3(grid_for(g.T * Cin, 256)), s, x, ge, (int)Cin, ws.U);
        else WINO_INPUT(wino_nz(), !af32, dim3(grid_for(g.T * Cin, 256)), s, x, g, (int)Cin, ws.U);
        wino_gemm_x3(ws, g.T, (int)Cin, (int)Cout, wino_points(), s, af32);
        Epi o{};
        o.bias = bias; o.scale = bn_scale; o.shift = bn_shift; o.res = residual;
        o.res_mode = residual ? 1 : 0; o.relu = relu; o.z = z_out; o.y = y; o.ldy = Cout;
        WINO_LAUNCH(wino_output_kernel, dim3(grid_for(g.T * Cout, 256)), dim3(256), 0, s, ws.M,
                    g, (int)Cout, o);
        return check_launch("conv3d winograd fwd (x3)");
    }
    if (u_keep) ws.U = u_keep;
    if (phase != 2)
        WINO_LAUNCH(wino_weight_kernel, dim3(grid_for(Cin * Cout, 256)), dim3(256), 0, s, w,
                           (int)Cin, (int)Cout, 0, ws.V);
    if (phase == 1) {
        WINO_INPUT(wino_nz(), false, dim3(grid_for(g.T * Cin, 256)), s, x, gi, (int)Cin, ws.U);
        return check_launch("conv3d winograd fwd (phase 1)");
    }
    WINO_INPUT(wino_nz(), false, dim3(grid_for(g.T * Cin, 256)), s, x, phase == 2 ? ge : g, (int)Cin, ws.U);
    ConvP p = wino_gemm_p(ws.U, g.T, (int)Cin, ws.V, (int)Cout);
    Epi e{};
    e.y = ws.M; e.ldy = Cout; e.simple = 1; e.YH = 1; e.YW = 1; e.YD = (int)g.T;
    e.ysy = e.ysx = e.ysz = 1;
    dispatch_gemm<false, true>(p, e, s, wino_points());
    Epi o{};
    o.bias = bias; o.scale = bn_scale; o.shift = bn_shift; o.res = residual;
    o.res_mode = residual ? 1 : 0; o.relu = relu; o.z = z_out; o.y = y; o.ldy = Cout;
    WINO_LAUNCH(wino_output_kernel, dim3(grid_for(g.T * Cout, 256)), dim3(256), 0, s, ws.M,
                       g, (int)Cout, o);
    return check_launch("conv3d winograd fwd");
}

extern "C" int m3d_conv3d_fwd_wino(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                   int64_t Cin, const float* w, int64_t Cout, int64_t OD,
                                   int32_t pz, const float* bias, const float* bn_scale,
                                   const float* bn_shift, const float* residual, int32_t relu,
                                   float* z_out, float* y, void* workspace, size_t ws_bytes,
                                   m3d_stream_t s) {
    return fwd_wino(x, B, H, W, D, Cin, w, Cout, OD, pz, bias, bn_scale, bn_shift, residual, relu,
                    z_out, y, nullptr, workspace, ws_bytes, st(s));
}

extern "C" int m3d_conv3d_fwd_wino_keep(const float* x, int64_t B, int64_t H, int64_t W, int64_t D,
                                        int64_t Cin, const float* w, int64_t Cout, int64_t OD,
                                        int32_t pz, const float* bias, const float* bn_scale,
                                        const float* bn_shift, const float* residual, int32_t relu,
                                        float* z_out, float* y, float* u_keep, void* workspace,
                                        size_t ws_bytes, m3d_stream_t s) {
    if (!u_keep) return einval("conv3d winograd: u_keep must not be NULL");
    if (wino_nz() != wino_wgrad_nz())
        return einval("conv3d winograd: forward and weight-gradient tiles differ (m3d_conv3d_wino_u_bytes == 0)");
    return fwd_wino(x, B, H, W, D, Cin, w, Cout, OD, pz, bias, bn_scale, bn_shift, residual, relu,
                    z_out, y, u_keep, workspace, ws_bytes, st(s));
}

// dx [B,H,W,D,Cin] = conv_transpose(dz [B,H,W,OD,Cout]): a 'same'-type 3x3x3
// correlation of dz with the flipped, transposed kernel, tiles over dx's grid,
// dz read at z = 2tz - (2 - pz) + k.
static int bwd_data_wino(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                         int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                         void* workspace, size_t ws_bytes, hipStream_t s, float* dx_halo = nullptr,
                         int hlo = 0, bool v_ready = false, const Epi* fb = nullptr, int ny = 0,
                         const void* v_ext = nullptr);

// The same two entry points for convs that share one kernel across calls (the
// RPN head's rpn_conv_shared1 on P2..P6, core/models.py:512-557): with
// v_ready = 1 the workspace's V region already holds this w's transform from
// an earlier call on the same stream (same Cin, Cout, workspace), and the
// weight transform is skipped.
extern "C" int m3d_conv3d_fwd_wino_v(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                                     const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                                     const float* bn_scale, const float* bn_shift, const float* residual,
                                     int32_t relu, float* z_out, float* y, void* workspace, size_t ws_bytes,
                                     int32_t v_ready, m3d_stream_t s) {
    return fwd_wino(x, B, H, W, D, Cin, w, Cout, OD, pz, bias, bn_scale, bn_shift, residual, relu, z_out, y,
                    nullptr, workspace, ws_bytes, st(s), nullptr, 0, 0, v_ready != 0);
}
extern "C" int m3d_conv3d_bwd_data_wino_v(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                          int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx,
                                          int32_t accumulate, void* workspace, size_t ws_bytes, int32_t v_ready,
                                          m3d_stream_t s) {
    return bwd_data_wino(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, st(s), nullptr,
                         0, v_ready != 0);
}

// tile_y: the data gradient's y tile for this call (2: F(2x2xNZ), 4: F(4x2xNZ);
// 0: the library's, m3d_conv3d_wino_dgrad_tile_y).  The V region a v_ready
// call reuses must have been transformed with the same tile_y.
static int dgrad_tile_arg(int32_t tile_y, int& ny) {
    if (tile_y != 0 && tile_y != 2 && tile_y != 4) return einval("conv3d winograd bwd-data: tile_y must be 0, 2 or 4");
    ny = tile_y ? tile_y : wino_dgrad_ny();
    return M3D_OK;
}

extern "C" int m3d_conv3d_bwd_data_wino_vy(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                           int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx,
                                           int32_t accumulate, void* workspace, size_t ws_bytes, int32_t v_ready,
                                           int32_t tile_y, m3d_stream_t s) {
    int ny;
    int rc = dgrad_tile_arg(tile_y, ny);
    if (rc) return rc;
    return bwd_data_wino(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, st(s), nullptr,
                         0, v_ready != 0, nullptr, ny);
}

extern "C" int m3d_conv3d_bwd_data_wino(const float* dz, const float* w, int64_t B, int64_t H,
                                        int64_t W, int64_t D, int64_t Cin, int64_t Cout,
                                        int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                                        void* workspace, size_t ws_bytes, m3d_stream_t s) {
    return bwd_data_wino(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, st(s));
}

static int bwd_data_wino_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                            int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                            void* workspace, size_t ws_bytes, int32_t v_ready, const m3d_bn_bwd_t* bn, void* bn_ws,
                            size_t bn_ws_bytes, int ny, hipStream_t hs, const void* v_ext = nullptr) {
    if (Cin % 256 != 0 && 256 % Cin != 0)
        return einval("conv3d winograd bwd-data (fused BN backward): Cin must divide 256 or be a multiple of it");
    if (wino_per_item(B, H, W, D, OD, Cin, Cout))
        return einval("conv3d winograd bwd-data (fused BN backward): batch past the 32-bit operand bound");
    const WinoGeom g = wino_geom(B, H, W, D, OD, 2 - pz, wino_dgrad_nz(), ny);
    const int64_t rows = Cin % 256 == 0 ? g.T : (g.T * Cin + 255) / 256;
    Epi e{};
    int rc = bn_fuse_epi(bn, Cin, bn_ws, bn_ws_bytes, rows, e);
    if (rc) return rc;
    rc = bwd_data_wino(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, hs, nullptr, 0,
                       v_ready != 0, &e, ny, v_ext);
    if (rc) return rc;
    return bn_sums_reduce(e.fpart, rows, Cin, bn->sum_dpre, bn->sum_dpre_xhat, bn->sum_dz, hs);
}

extern "C" int m3d_conv3d_bwd_data_wino_bn(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                           int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx,
                                           int32_t accumulate, void* workspace, size_t ws_bytes, int32_t v_ready,
                                           const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes,
                                           m3d_stream_t s) {
    return bwd_data_wino_bn(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, v_ready, bn,
                            bn_ws, bn_ws_bytes, wino_dgrad_ny(), st(s));
}

extern "C" int m3d_conv3d_bwd_data_wino_bny(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                            int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx,
                                            int32_t accumulate, void* workspace, size_t ws_bytes, int32_t v_ready,
                                            const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes, int32_t tile_y,
                                            m3d_stream_t s) {
    int ny;
    int rc = dgrad_tile_arg(tile_y, ny);
    if (rc) return rc;
    return bwd_data_wino_bn(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, v_ready, bn,
                            bn_ws, bn_ws_bytes, ny, st(s));
}

// ---- Winograd weight transforms into caller memory ----------------------------
// The transformed weights depend only on w, so a caller can produce them ahead
// of the convs (e.g. on a side stream at the start of a model's forward) and
// hand them to m3d_conv3d_fwd_wino_kv / m3d_conv3d_bwd_data_wino_xv.  Layout:
// the bf16-split planes the point GEMMs read, [3][points][n'][k'] uint16, at
// offset 0; the forward's form also uses a 27*Cin*Cout fp32 scratch behind them
// (the transposed weights, x3_wt_kernel).
static size_t wino_v_planes_bytes(int64_t Cin, int64_t Cout, int dgrad, int ny) {
    const int P = dgrad ? wino_points(wino_dgrad_nz(), ny) : wino_points();
    return (6 * (size_t)P * (size_t)Cin * (size_t)Cout + 255) & ~(size_t)255;
}
static int wino_v_tile(int32_t dgrad, int32_t tile_y, int& ny) {
    if (!gemm_x3_env()) return einval("conv3d winograd: external transformed weights need the bf16-split GEMMs");
    if (dgrad) return dgrad_tile_arg(tile_y, ny);
    ny = WNY;
    return M3D_OK;
}
extern "C" size_t m3d_conv3d_wino_v_bytes(int64_t Cin, int64_t Cout, int32_t dgrad, int32_t tile_y) {
    int ny;
    if (Cin <= 0 || Cout <= 0 || wino_v_tile(dgrad, tile_y, ny)) return 0;
    return wino_v_planes_bytes(Cin, Cout, dgrad, ny) + (dgrad ? 0 : sizeof(float) * 27 * (size_t)Cin * Cout);
}
extern "C" int m3d_conv3d_wino_weight_v(const float* w, int64_t Cin, int64_t Cout, int32_t dgrad, int32_t tile_y,
                                        void* v, size_t v_bytes, m3d_stream_t s) {
    int ny;
    if (Cin <= 0 || Cout <= 0) return einval("conv3d winograd: channel counts must be positive");
    if (int rc = wino_v_tile(dgrad, tile_y, ny)) return rc;
    if (!w || !v || v_bytes < m3d_conv3d_wino_v_bytes(Cin, Cout, dgrad, tile_y))
        return einval("conv3d winograd: transformed-weight buffer missing or too small (m3d_conv3d_wino_v_bytes)");
    const dim3 grid(grid_for(Cin * Cout, 256));
    if (!dgrad) {
        float* wt = reinterpret_cast<float*>(static_cast<char*>(v) + wino_v_planes_bytes(Cin, Cout, 0, ny));
        hipLaunchKernelGGL(x3_wt_kernel, dim3((unsigned)((Cout + 31) / 32), (unsigned)((Cin + 31) / 32), 27),
                           dim3(256), 0, st(s), w, (int)Cin, (int)Cout, wt);
        WINO_LAUNCH_NZ_X3(wino_nz(), wino_weight_kernel, grid, dim3(256), 0, st(s), wt, (int)Cin, (int)Cout, 0,
                          static_cast<float*>(v));
        return check_launch("conv3d winograd weight transform (fwd)");
    }
    const int nz = wino_dgrad_nz();
    float* V = static_cast<float*>(v);
    if (nz == 4 && ny == 4) hipLaunchKernelGGL((wino_weight_kernel<4, true, 4>), grid, dim3(256), 0, st(s), w, (int)Cin, (int)Cout, 1, V);
    else if (nz == 4) hipLaunchKernelGGL((wino_weight_kernel<4, true, 2>), grid, dim3(256), 0, st(s), w, (int)Cin, (int)Cout, 1, V);
    else if (ny == 4) hipLaunchKernelGGL((wino_weight_kernel<2, true, 4>), grid, dim3(256), 0, st(s), w, (int)Cin, (int)Cout, 1, V);
    else hipLaunchKernelGGL((wino_weight_kernel<2, true, 2>), grid, dim3(256), 0, st(s), w, (int)Cin, (int)Cout, 1, V);
    return check_launch("conv3d winograd weight transform (dgrad)");
}
extern "C" int m3d_conv3d_fwd_wino_kv(const float* x, int64_t B, int64_t H, int64_t W, int64_t D, int64_t Cin,
                                      const float* w, int64_t Cout, int64_t OD, int32_t pz, const float* bias,
                                      const float* bn_scale, const float* bn_shift, const float* residual,
                                      int32_t relu, float* z_out, float* y, float* u_keep, const void* v,
                                      void* workspace, size_t ws_bytes, m3d_stream_t s) {
    int ny;
    if (int rc = wino_v_tile(0, 0, ny)) return rc;
    if (!v) return einval("conv3d winograd: v must not be NULL (m3d_conv3d_wino_weight_v)");
    if (u_keep && wino_nz() != wino_wgrad_nz())
        return einval("conv3d winograd: forward and weight-gradient tiles differ (m3d_conv3d_wino_u_bytes == 0)");
    return fwd_wino(x, B, H, W, D, Cin, w, Cout, OD, pz, bias, bn_scale, bn_shift, residual, relu, z_out, y, u_keep,
                    workspace, ws_bytes, st(s), nullptr, 0, 0, false, 0, v);
}
extern "C" int m3d_conv3d_bwd_data_wino_xv(const float* dz, const float* w, int64_t B, int64_t H, int64_t W,
                                           int64_t D, int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx,
                                           int32_t accumulate, void* workspace, size_t ws_bytes, const void* v,
                                           int32_t tile_y, const m3d_bn_bwd_t* bn, void* bn_ws, size_t bn_ws_bytes,
                                           m3d_stream_t s) {
    int ny;
    if (int rc = wino_v_tile(1, tile_y, ny)) return rc;
    if (!v) return einval("conv3d winograd bwd-data: v must not be NULL (m3d_conv3d_wino_weight_v)");
    if (bn)
        return bwd_data_wino_bn(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, 0, bn, bn_ws,
                                bn_ws_bytes, ny, st(s), v);
    return bwd_data_wino(dz, w, B, H, W, D, Cin, Cout, OD, pz, dx, accumulate, workspace, ws_bytes, st(s), nullptr, 0,
                         false, nullptr, ny, v);
}

// the data-gradient output transform: dx over the (halo-extended) grid, or,
// for a depth slab with dx_halo, interior planes into dx (depth dl) and the
// neighbours' planes into dx_halo [B][H][W][2][C]
template <int NZ, int NY>
static void wino_dgrad_out(const float* Mt, const WinoGeom& g, int C, float* dx, int accumulate,
                           float* dx_halo, int hlo, int dl, hipStream_t hs, const Epi* fb) {
    Epi o{};
    if (fb) o = *fb;                 // the fused BN backward's fields
    o.y = dx; o.ldy = C; o.accumulate = accumulate;
    const dim3 grid(grid_for(g.T * C, 256));
    if (fb) {
        hipLaunchKernelGGL((wino_output_bn_kernel<NZ, NY>), grid, dim3(256), 0, hs, Mt, g, C, o);
        return;
    }
    if (dx_halo) {
        o.yh = dx_halo; o.hlo = hlo; o.dl = dl;
        hipLaunchKernelGGL((wino_output_halo_kernel<NZ, NY>), grid, dim3(256), 0, hs, Mt, g, C, o);
        return;
    }
    hipLaunchKernelGGL((wino_output_kernel<NZ, NY>), grid, dim3(256), 0, hs, Mt, g, C, o);
}

// the data gradient's launches on F(NY x 2 x NZ) tiles (geometry g, workspace ws)
template <int NZ, int NY>
static void bwd_data_wino_launch(const float* dz, const float* w, const WinoGeom& g, const WinoWs& ws, int Cin,
                                 int Cout, float* dx, int32_t accumulate, float* dx_halo, int hlo, int dl,
                                 bool v_ready, const Epi* fb, hipStream_t hs) {
    const int P = wino_points(NZ, NY);
    const dim3 wgrid(grid_for((int64_t)Cin * Cout, 256)), igrid(grid_for(g.T * Cout, 256));
    if (gemm_x3_env()) {
        if (!v_ready)
            hipLaunchKernelGGL((wino_weight_kernel<NZ, true, NY>), wgrid, dim3(256), 0, hs, w, Cin, Cout, 1, ws.V);
        const bool af32 = x3_af32_env();
        if (af32)
            hipLaunchKernelGGL((wino_input_kernel<NZ, false, false, NY>), igrid, dim3(256), 0, hs, dz, g, Cout, ws.U);
        else
            hipLaunchKernelGGL((wino_input_kernel<NZ, true, false, NY>), igrid, dim3(256), 0, hs, dz, g, Cout, ws.U);
        wino_gemm_x3(ws, g.T, Cout, Cin, P, hs, af32);
    } else {
        hipLaunchKernelGGL((wino_weight_kernel<NZ, false, NY>), wgrid, dim3(256), 0, hs, w, Cin, Cout, 1, ws.V);
        hipLaunchKernelGGL((wino_input_kernel<NZ, false, false, NY>), igrid, dim3(256), 0, hs, dz, g, Cout, ws.U);
        ConvP p = wino_gemm_p(ws.U, g.T, Cout, ws.V, Cin);
        Epi e{};
        e.y = ws.M; e.ldy = Cin; e.simple = 1; e.YH = 1; e.YW = 1; e.YD = (int)g.T;
        e.ysy = e.ysx = e.ysz = 1;
        dispatch_gemm<false, true>(p, e, hs, P);
    }
    wino_dgrad_out<NZ, NY>(ws.M, g, Cin, dx, accumulate, dx_halo, hlo, dl, hs, fb);
}

static int bwd_data_wino(const float* dz, const float* w, int64_t B, int64_t H, int64_t W, int64_t D,
                         int64_t Cin, int64_t Cout, int64_t OD, int32_t pz, float* dx, int32_t accumulate,
                         void* workspace, size_t ws_bytes, hipStream_t hs, float* dx_halo, int hlo, bool v_ready,
                         const Epi* fb, int ny_arg, const void* v_ext) {
    int rc = wino_check(B, H, W, D, OD, pz, Cin, Cout);
    if (rc) return rc;
    if (wino_per_item(B, H, W, D, OD, Cin, Cout)) {
        const int64_t dxd = dx_halo ? OD : D;          // dx depth: the slab's interior, or the full grid
        for (int64_t b = 0; b < B; ++b) {
            rc = bwd_data_wino(dz + b * H * W * OD * Cout, w, 1, H, W, D, Cin, Cout, OD, pz, dx + b * H * W * dxd * Cin,
                               accumulate, workspace, ws_bytes, hs,
                               dx_halo ? dx_halo + b * H * W * 2 * Cin : nullptr, hlo, v_ready || b > 0, nullptr,
                               ny_arg, v_ext);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    const int nz = wino_dgrad_nz(), ny = ny_arg ? ny_arg : wino_dgrad_ny();
    const WinoGeom g = wino_geom(B, H, W, D, OD, 2 - pz, nz, ny);
    // the layout this call uses (its tile_y may differ from the library's default)
    if (ws_bytes < wino_ws_need(g, Cout, Cin, nz, ny))
        return einval("conv3d winograd: workspace too small");
    // same layout with the roles of Cin/Cout swapped (V'[P][Cout][Cin], U'[P][T][Cout])
    WinoWs ws = wino_ws(workspace, g, Cout, Cin, nz, ny);
    if (v_ext) {                        // transformed by m3d_conv3d_wino_weight_v (dgrad 1, this tile_y)
        ws.V = static_cast<float*>(const_cast<void*>(v_ext));
        v_ready = true;
    }
    const int ci = (int)Cin, co = (int)Cout, dl = (int)OD;
    if (nz == 4 && ny == 4)
        bwd_data_wino_launch<4, 4>(dz, w, g, ws, ci, co, dx, accumulate, dx_halo, hlo, dl, v_ready, fb, hs);
    else if (nz == 4)
        bwd_data_wino_launch<4, 2>(dz, w, g, ws, ci, co, dx, accumulate, dx_halo, hlo, dl, v_ready, fb, hs);
    else if (ny == 4)
        bwd_data_wino_launch<2, 4>(dz, w, g, ws, ci, co, dx, accumulate, dx_halo, hlo, dl, v_ready, fb, hs);
    else
        bwd_data_wino_launch<2, 2>(dz, w, g, ws, ci, co, dx, accumulate, dx_halo, hlo, dl, v_ready, fb, hs);
    return check_launch("conv3d winograd bwd-data");
}

static int bwd_weight_wino(const float* x, const float* u_in, const float* dz, int64_t B,
                           int64_t H, int64_t W, int64_t D, int64_t Cin, int64_t Cout, int64_t OD,
                           int32_t pz, float* dw, void* workspace, size_t ws_bytes, m3d_stream_t s,
                           const float* halo = nullptr, int hlo = 0, int hhi = 0) {
    int rc = wino_check(B, H, W, D, OD, pz, Cin, Cout);
    if (rc) return rc;
    if (ws_bytes < m3d_conv3d_wino_workspace_bytes(B, H, W, D, OD, Cin, Cout))
        return einval("conv3d winograd: workspace too small");
    if (wino_per_item(B, H, W, D, OD, Cin, Cout)) {           // dw accumulates over the items
        if (u_in) return einval("conv3d winograd: kept U with a batch past the 32-bit operand bound");
        for (int64_t b = 0; b < B; ++b) {
            rc = bwd_weight_wino(x + b * H * W * D * Cin, nullptr, dz + b * H * W * OD * Cout, 1, H, W, D, Cin, Cout,
                                 OD, pz, dw, workspace, ws_bytes, s, halo ? halo + b * H * W * 2 * Cin : nullptr, hlo,
                                 hhi);
            if (rc) return rc;
        }
        return M3D_OK;
    }
    const int nz = wino_wgrad_nz();
    WinoGeom g = wino_geom(B, H, W, OD, D, pz, nz);
    g.halo = halo; g.hlo = hlo; g.hhi = hhi;
    WinoWs ws = wino_ws(workspace, g, Cin, Cout, nz);   // V <- dW_hat, U <- B^T x, M <- A dz
    if (hipMemsetAsync(ws.V, 0, sizeof(float) * wino_points(nz) * (size_t)Cin * Cout, st(s)) != hipSuccess)
        return check_launch("memset dW_hat");
    if (u_in)
        ws.U = const_cast<float*>(u_in);       // the forward's transformed input, kept
    else
        WINO_INPUT(nz, false, dim3(grid_for(g.T * Cin, 256)), st(s), x, g, (int)Cin, ws.U);
    // M3D_WINO_GRAD4=1: the float4 form (measured slower: 278 vs 253 us avg, write-bound)
        WINO_LAUNCH_NZ(nz, wino_grad_kernel, dim3(grid_for(g.T * Cout, 256)), dim3(256), 0, st(s), dz, g,
                       (int)Cout, ws.M);
    // (Cin, Cout <= 64: x3_wgrad64_kernel, the whole 64x64 product per workgroup)
    if (wgrad_x3_env() && (Cout > 64 || Cin <= 64)) {
        launch_wgrad_x3(ws.U, ws.M, ws.V, g.T, (int)Cin, (int)Cout, wino_points(nz), g.T * Cin, g.T * Cout,
                        (int64_t)Cin * Cout, st(s));
    } else {
        ConvP p = wino_gemm_p(ws.U, g.T, (int)Cin, nullptr, (int)Cout);
        p.bsw = g.T * Cout;                 // dz (DY) batch stride
        p.bsy = (int64_t)Cin * Cout;        // dW_hat batch stride
        if (Cout <= 64) launch_wgrad<128, 64, 2, 2, true>(p, ws.M, ws.V, st(s), wino_points(nz));
        else launch_wgrad<128, 128, 2, 2, true>(p, ws.M, ws.V, st(s), wino_points(nz));
    }
    WINO_LAUNCH_NZ(nz, wino_wgrad_out_kernel, dim3(grid_for(Cin * Cout, 256)), dim3(256), 0, st(s),
                       ws.V, (int)Cin, (int)Cout, dw);
    return check_launch("conv3d winograd bwd-weight");
}

extern "C" int m3d_conv3d_bwd_weight_wino(const float* x, const float* dz, int64_t B, int64_t H,
                                          int64_t W, int64_t D, int64_t Cin, int64_t Cout,
                                          int64_t OD, int32_t pz, float* dw, void* workspace,
                                          size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    return bwd_weight_wino(x, nullptr, dz, B, H, W, D, Cin, Cout, OD, pz, dw, workspace, ws_bytes, s);
}

// ---- depth-slab forms: interior slab + separate halo planes -----------------
// x [B,H,W,Dl,C] is this rank's slab, x_halo [B,H,W,2,C] the neighbours'
// boundary planes (plane 0 = z -1 from the lower rank, valid if has_lo;
// plane 1 = z Dl from the upper rank, valid if has_hi).  The same tiles and
// arithmetic as the halo-extended tensor (bit-identical results) without
// materialising it.  workspace: m3d_conv3d_wino_workspace_bytes(B, H, W,
// Dl + has_lo + has_hi, Dl, Cin, Cout).
static int halo_check(const void* x_halo, int32_t has_lo, int32_t has_hi) {
    if ((has_lo | has_hi) & ~1) return einval("conv3d winograd halo: has_lo / has_hi must be 0 or 1");
    if ((has_lo || has_hi) && !x_halo) return einval("conv3d winograd halo: halo planes missing");
    return M3D_OK;
}

extern "C" int m3d_conv3d_fwd_wino_halo(const float* x, const float* x_halo, int32_t has_lo, int32_t has_hi,
                                        int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin,
                                        const float* w, int64_t Cout, const float* bias, const float* bn_scale,
                                        const float* bn_shift, const float* residual, int32_t relu, float* z_out,
                                        float* y, float* u_keep, void* workspace, size_t ws_bytes,
                                        m3d_stream_t s) {
    int rc = halo_check(x_halo, has_lo, has_hi);
    if (rc) return rc;
    if (u_keep && wino_nz() != wino_wgrad_nz())
        return einval("conv3d winograd: forward and weight-gradient tiles differ (m3d_conv3d_wino_u_bytes == 0)");
    return fwd_wino(x, B, H, W, Dl, Cin, w, Cout, Dl, 1, bias, bn_scale, bn_shift, residual, relu, z_out, y,
                    u_keep, workspace, ws_bytes, st(s), x_halo, has_lo, has_hi);
}

// The same conv in two launches around the halo exchange: phase 1 (before the
// halo planes arrive; x_halo is not read) transforms the weights and the
// interior z tiles, phase 2 (after) the first / last z tiles, then the GEMM
// and the output transform -- the caller overlaps the exchange with phase 1.
// Both phases take the same arguments and workspace; bit-identical to
// m3d_conv3d_fwd_wino_halo.
extern "C" int m3d_conv3d_fwd_wino_halo_phase(const float* x, const float* x_halo, int32_t has_lo, int32_t has_hi,
                                              int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin,
                                              const float* w, int64_t Cout, const float* bias, const float* bn_scale,
                                              const float* bn_shift, const float* residual, int32_t relu,
                                              float* z_out, float* y, float* u_keep, void* workspace,
                                              size_t ws_bytes, int32_t phase, m3d_stream_t s) {
    if (phase != 1 && phase != 2) return einval("conv3d winograd halo: phase must be 1 or 2");
    int rc = phase == 2 ? halo_check(x_halo, has_lo, has_hi) : M3D_OK;
    if (rc) return rc;
    if (u_keep && wino_nz() != wino_wgrad_nz())
        return einval("conv3d winograd: forward and weight-gradient tiles differ (m3d_conv3d_wino_u_bytes == 0)");
    return fwd_wino(x, B, H, W, Dl, Cin, w, Cout, Dl, 1, bias, bn_scale, bn_shift, residual, relu, z_out, y,
                    u_keep, workspace, ws_bytes, st(s), phase == 2 ? x_halo : nullptr, has_lo, has_hi, false,
                    phase);
}

// dx [B,H,W,Dl,Cin] (interior, accumulate as m3d_conv3d_bwd_data_wino) and
// dx_halo [B,H,W,2,Cin] = the gradient of the neighbours' halo planes (always
// written; planes of absent neighbours are left untouched)
extern "C" int m3d_conv3d_bwd_data_wino_halo(const float* dz, const float* w, int32_t has_lo, int32_t has_hi,
                                             int64_t B, int64_t H, int64_t W, int64_t Dl, int64_t Cin,
                                             int64_t Cout, float* dx, float* dx_halo, int32_t accumulate,
                                             void* workspace, size_t ws_bytes, m3d_stream_t s) {
    int rc = halo_check(dx_halo, has_lo, has_hi);
    if (rc) return rc;
    return bwd_data_wino(dz, w, B, H, W, Dl + has_lo + has_hi, Cin, Cout, Dl, 1 - has_lo, dx, accumulate,
                         workspace, ws_bytes, st(s), (has_lo || has_hi) ? dx_halo : nullptr, has_lo);
}

extern "C" int m3d_conv3d_bwd_weight_wino_halo(const float* x, const float* x_halo, int32_t has_lo,
                                               int32_t has_hi, const float* dz, int64_t B, int64_t H, int64_t W,
                                               int64_t Dl, int64_t Cin, int64_t Cout, float* dw, void* workspace,
                                               size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    int rc = halo_check(x_halo, has_lo, has_hi);
    if (rc) return rc;
    return bwd_weight_wino(x, nullptr, dz, B, H, W, Dl, Cin, Cout, Dl, 1, dw, workspace, ws_bytes, s, x_halo,
                           has_lo, has_hi);
}

extern "C" int m3d_conv3d_bwd_weight_wino_u(const float* u, const float* dz, int64_t B, int64_t H,
                                            int64_t W, int64_t D, int64_t Cin, int64_t Cout,
                                            int64_t OD, int32_t pz, float* dw, void* workspace,
                                            size_t ws_bytes, const m3d_det_t* det, m3d_stream_t s) {
    M3D_DET_SCOPE(det);
    if (!u) return einval("conv3d winograd: u must not be NULL");
    return bwd_weight_wino(nullptr, u, dz, B, H, W, D, Cin, Cout, OD, pz, dw, workspace, ws_bytes, s);
}
