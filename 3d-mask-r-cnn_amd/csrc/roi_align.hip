// 3-D CropAndResize / PyramidROIAlign kernels for gfx950.
//
// Replaces the CPU-only TF ops CropAndResize3D{,GradImage,GradBoxes} of the
// vendored wheel and the PyramidROIAlign
// layer glue (core/models.py:597-687).
//
// Mapping: one wave64 per output sample (n, y, x, z); the 64 lanes walk the
// channel vector (C innermost, channels-last) with float4 accesses, so every
// one of the 8 trilinear corner reads is a contiguous C*4-byte row (1 KiB per
// wave-instruction at C=256) and every output store is coalesced.  The
// coordinate maths runs redundantly in all lanes (wave-uniform values).
//
// Exactness: compiled with -ffp-contract=off; the coordinate / lerp op order
// is the reference's, so trilinear outputs are bit-identical
// to the CPU restatement (oracle/oracle.c).
#include "common.h"

namespace m3d {

// ---- coordinate maths (whl @0x499a-0x4a62, @0x4abd, @0x5287) ----
__device__ __forceinline__ float axis_scale(float b1, float b2, int S, int n) {
    return n > 1 ? ((b2 - b1) * (float)(S - 1)) / (float)(n - 1) : 0.0f;
}
__device__ __forceinline__ float axis_coord(float b1, float b2, int S, int n, int i, float sc) {
    if (n > 1) return b1 * (float)(S - 1) + (float)i * sc;
    return (float)(0.5 * (double)(b1 + b2) * (double)(S - 1));
}

struct Sample {
    int oob;              // 1 if the sample lies outside the image (extrapolate)
    int ty, by, lx, rx, fz, kz;
    float yl, xl, zl;
    int ny, nx, nz;       // nearest indices
};

__device__ __forceinline__ Sample make_sample(const float* box, int H, int W, int D, int ch, int cw,
                                              int cd, int y, int x, int z) {
    Sample s{};
    const float y1 = box[0], x1 = box[1], z1 = box[2], y2 = box[3], x2 = box[4], z2 = box[5];
    const float in_y = axis_coord(y1, y2, H, ch, y, axis_scale(y1, y2, H, ch));
    const float in_x = axis_coord(x1, x2, W, cw, x, axis_scale(x1, x2, W, cw));
    const float in_z = axis_coord(z1, z2, D, cd, z, axis_scale(z1, z2, D, cd));
    s.oob = (in_y < 0 || in_y > (float)(H - 1)) || (in_x < 0 || in_x > (float)(W - 1)) ||
            (in_z < 0 || in_z > (float)(D - 1));
    if (s.oob) return s;
    s.ty = (int)floorf(in_y); s.by = (int)ceilf(in_y); s.yl = in_y - (float)s.ty;
    s.lx = (int)floorf(in_x); s.rx = (int)ceilf(in_x); s.xl = in_x - (float)s.lx;
    s.fz = (int)floorf(in_z); s.kz = (int)ceilf(in_z); s.zl = in_z - (float)s.fz;
    s.ny = (int)roundf(in_y); s.nx = (int)roundf(in_x); s.nz = (int)roundf(in_z);
    return s;
}

__device__ __forceinline__ float tri(float tlf, float tlk, float trf, float trk, float blf,
                                     float blk, float brf, float brk, float yl, float xl,
                                     float zl) {
    // lerp order @0x4f88-0x5011: z first, then x, then y
    const float tl = tlf + (tlk - tlf) * zl;
    const float bl = blf + (blk - blf) * zl;
    const float tr = trf + (trk - trf) * zl;
    const float br = brf + (brk - brf) * zl;
    const float top = tl + (tr - tl) * xl;
    const float bot = bl + (br - bl) * xl;
    return top + (bot - top) * yl;
}

__device__ __forceinline__ float scrub(float v) { return isfinite(v) ? v : 0.0f; }

// Writes one output sample's C channels (lane-strided).  img points at image b.
template <bool SCRUB>
__device__ __forceinline__ void emit_sample(const float* __restrict__ img, int W, int D, int C,
                                            const Sample& s, int method, float extrap,
                                            float* __restrict__ o, int lane) {
    if (s.oob) {
        if ((C & 3) == 0) {
            const float4 e = make_float4(extrap, extrap, extrap, extrap);
            for (int c = lane; c < (C >> 2); c += 64) reinterpret_cast<float4*>(o)[c] = e;
        } else {
            for (int c = lane; c < C; c += 64) o[c] = extrap;
        }
        return;
    }
    const size_t rowD = (size_t)D * C, rowW = (size_t)W * rowD;
    if (method == 1) {
        const float* v = img + s.ny * rowW + s.nx * rowD + (size_t)s.nz * C;
        for (int c = lane; c < C; c += 64) o[c] = SCRUB ? scrub(v[c]) : v[c];
        return;
    }
    const float* tl = img + s.ty * rowW + s.lx * rowD;
    const float* tr = img + s.ty * rowW + s.rx * rowD;
    const float* bl = img + s.by * rowW + s.lx * rowD;
    const float* br = img + s.by * rowW + s.rx * rowD;
    const size_t f = (size_t)s.fz * C, k = (size_t)s.kz * C;
    if ((C & 3) == 0) {
        const float4 *tlf = (const float4*)(tl + f), *tlk = (const float4*)(tl + k);
        const float4 *trf = (const float4*)(tr + f), *trk = (const float4*)(tr + k);
        const float4 *blf = (const float4*)(bl + f), *blk = (const float4*)(bl + k);
        const float4 *brf = (const float4*)(br + f), *brk = (const float4*)(br + k);
        for (int c = lane; c < (C >> 2); c += 64) {
            const float4 a = tlf[c], b = tlk[c], cc = trf[c], d = trk[c];
            const float4 e = blf[c], g = blk[c], h = brf[c], i = brk[c];
            float4 r;
            r.x = tri(a.x, b.x, cc.x, d.x, e.x, g.x, h.x, i.x, s.yl, s.xl, s.zl);
            r.y = tri(a.y, b.y, cc.y, d.y, e.y, g.y, h.y, i.y, s.yl, s.xl, s.zl);
            r.z = tri(a.z, b.z, cc.z, d.z, e.z, g.z, h.z, i.z, s.yl, s.xl, s.zl);
            r.w = tri(a.w, b.w, cc.w, d.w, e.w, g.w, h.w, i.w, s.yl, s.xl, s.zl);
            if (SCRUB) { r.x = scrub(r.x); r.y = scrub(r.y); r.z = scrub(r.z); r.w = scrub(r.w); }
            reinterpret_cast<float4*>(o)[c] = r;
        }
    } else {
        for (int c = lane; c < C; c += 64) {
            float r = tri(tl[f + c], tl[k + c], tr[f + c], tr[k + c], bl[f + c], bl[k + c],
                          br[f + c], br[k + c], s.yl, s.xl, s.zl);
            o[c] = SCRUB ? scrub(r) : r;
        }
    }
}

// Atomic scatter of one sample's gradient into the 8 corners (A.2 weights).
__device__ __forceinline__ void scatter_sample(float* __restrict__ img, int W, int D, int C,
                                               const Sample& s, int method,
                                               const float* __restrict__ g, int lane) {
    if (s.oob) return;
    const size_t rowD = (size_t)D * C, rowW = (size_t)W * rowD;
    if (method == 1) {
        float* v = img + s.ny * rowW + s.nx * rowD + (size_t)s.nz * C;
        for (int c = lane; c < C; c += 64) unsafeAtomicAdd(v + c, g[c]);
        return;
    }
    const float wy[2] = {1.0f - s.yl, s.yl}, wx[2] = {1.0f - s.xl, s.xl},
                wz[2] = {1.0f - s.zl, s.zl};
    const int iy[2] = {s.ty, s.by}, ix[2] = {s.lx, s.rx}, iz[2] = {s.fz, s.kz};
    float w[8];
    float* dst[8];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
#pragma unroll
            for (int c = 0; c < 2; ++c) {
                w[a * 4 + b * 2 + c] = (wy[a] * wx[b]) * wz[c];
                dst[a * 4 + b * 2 + c] = img + iy[a] * rowW + ix[b] * rowD + (size_t)iz[c] * C;
            }
    for (int c = lane; c < C; c += 64) {
        const float gv = g[c];
#pragma unroll
        for (int q = 0; q < 8; ++q) unsafeAtomicAdd(dst[q] + c, gv * w[q]);
    }
}

struct Pyr {
    const float* fmaps[4];
    float* gmaps[4];
    int H[4], W[4], D[4];
};

// ---- trilinear z-line kernel (C % 4 == 0) ---------------------------------
// One wave per output line (n, y, x): the wave walks the cd samples of the
// line in z.  The 4 (y, x) corner columns of a line are contiguous in memory
// along z ([H][W][D][C] layout), and a sample whose floor plane equals the
// previous sample's ceil plane reuses those 4 rows from registers.  The 4
// waves of a workgroup are 4 consecutive x of one y, so their corner columns
// overlap in L1/L2, and the block index is remapped XCD-contiguously so the
// lines of one ROI stay in one XCD's L2.  Per-sample arithmetic is exactly
// make_sample + tri (bit-identical to the per-sample kernels).
__device__ __forceinline__ int64_t xcd_block() {
    const int64_t nb = gridDim.x, L = blockIdx.x, xcd = L % 8, q8 = nb / 8, r8 = nb % 8;
    return (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + L / 8;
}

struct LineArgs {
    const float* image;          // crop: [B,H,W,D,C]
    const int32_t* box_ind;
    const float* boxes;          // crop: [N,6]; pyramid: boxes_adj [B*N,6]
    const int32_t* levels;       // pyramid
    int64_t N;                   // pyramid: boxes per image
    int64_t lines;               // (#boxes) * ch * cw
    int H, W, D, C, ch, cw, cd;
    float extrap;
    float* out;
};

__device__ __forceinline__ float4 tri4(const float4& a, const float4& b, const float4& c,
                                       const float4& d, const float4& e, const float4& g,
                                       const float4& h, const float4& i, float yl, float xl,
                                       float zl) {
    float4 r;
    r.x = tri(a.x, b.x, c.x, d.x, e.x, g.x, h.x, i.x, yl, xl, zl);
    r.y = tri(a.y, b.y, c.y, d.y, e.y, g.y, h.y, i.y, yl, xl, zl);
    r.z = tri(a.z, b.z, c.z, d.z, e.z, g.z, h.z, i.z, yl, xl, zl);
    r.w = tri(a.w, b.w, c.w, d.w, e.w, g.w, h.w, i.w, yl, xl, zl);
    return r;
}

typedef float f4v __attribute__((ext_vector_type(4)));
// Output rows are written once and never re-read here: non-temporal stores
// keep them from evicting the feature-map corner rows from L2.
__device__ __forceinline__ void st_nt(float4* p, const float4& v) {
    f4v t = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(t, reinterpret_cast<f4v*>(p));
}

template <bool PYR>
__global__ __launch_bounds__(256) void line_fwd_kernel(LineArgs a, Pyr P) {
    const int64_t line = xcd_block() * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (line >= a.lines) return;
    int64_t t = line;
    const int x = (int)(t % a.cw); t /= a.cw;
    const int y = (int)(t % a.ch);
    const int64_t n = t / a.ch;
    int H, W, D;
    const float* img;
    if (PYR) {
        const int l = a.levels[n] - 2;
        H = P.H[l]; W = P.W[l]; D = P.D[l];
        img = P.fmaps[l] + (size_t)(n / a.N) * H * W * D * a.C;
    } else {
        H = a.H; W = a.W; D = a.D;
        img = a.image + (size_t)a.box_ind[n] * H * W * D * a.C;
    }
    const float* box = a.boxes + n * 6;
    const float y1 = box[0], x1 = box[1], z1 = box[2], y2 = box[3], x2 = box[4], z2 = box[5];
    const float in_y = axis_coord(y1, y2, H, a.ch, y, axis_scale(y1, y2, H, a.ch));
    const float in_x = axis_coord(x1, x2, W, a.cw, x, axis_scale(x1, x2, W, a.cw));
    const float zsc = axis_scale(z1, z2, D, a.cd);
    const int C4 = a.C >> 2;
    float4* o = reinterpret_cast<float4*>(a.out + line * (int64_t)a.cd * a.C);
    const bool yx_oob = (in_y < 0 || in_y > (float)(H - 1)) || (in_x < 0 || in_x > (float)(W - 1));
    const float4 ex = make_float4(a.extrap, a.extrap, a.extrap, a.extrap);
    if (yx_oob) {
        for (int z = 0; z < a.cd; ++z)
            for (int c = lane; c < C4; c += 64) st_nt(o + (int64_t)z * C4 + c, ex);
        return;
    }
    const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
    const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
    const float yl = in_y - (float)ty, xl = in_x - (float)lx;
    const size_t rowD = (size_t)D * C4, rowW = (size_t)W * rowD;
    const float4* base = reinterpret_cast<const float4*>(img);
    const float4* col[4] = {base + ty * rowW + lx * rowD, base + ty * rowW + rx * rowD,
                            base + by * rowW + lx * rowD, base + by * rowW + rx * rowD};
    for (int c = lane; c < C4; c += 64) {
        int pk = -1;
        float4 kv[4];
        for (int z = 0; z < a.cd; ++z) {
            const float in_z = axis_coord(z1, z2, D, a.cd, z, zsc);
            float4 r;
            if (in_z < 0 || in_z > (float)(D - 1)) {
                r = ex;
            } else {
                const int fz = (int)floorf(in_z), kz = (int)ceilf(in_z);
                const float zl = in_z - (float)fz;
                float4 fv[4];
                if (fz == pk) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) fv[q] = kv[q];
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) fv[q] = col[q][(size_t)fz * C4 + c];
                }
                if (kz != fz) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) kv[q] = col[q][(size_t)kz * C4 + c];
                } else {
#pragma unroll
                    for (int q = 0; q < 4; ++q) kv[q] = fv[q];
                }
                pk = kz;
                // tri(tlf, tlk, trf, trk, blf, blk, brf, brk): tl = (ty,lx), tr = (ty,rx), ...
                r = tri4(fv[0], kv[0], fv[1], kv[1], fv[2], kv[2], fv[3], kv[3], yl, xl, zl);
                if (PYR) { r.x = scrub(r.x); r.y = scrub(r.y); r.z = scrub(r.z); r.w = scrub(r.w); }
            }
            st_nt(o + (int64_t)z * C4 + c, r);
        }
    }
}

// owner voxel index of a sample coordinate along an axis of S voxels (samples
// outside the map go to the nearest end voxel: every sample has one owner)
__device__ __forceinline__ int owner_idx(float in, int S) {
    return in >= 0.0f ? (in <= (float)(S - 1) ? (int)floorf(in) : S - 1) : 0;
}

struct RegionBase {
    int64_t base[4];             // first (y, x) column bucket of each level (B-major inside)
};

// ---- PyramidROIAlign forward, channel-sliced line kernel --------------------------
// line_fwd_kernel<true> with the channels cut into SL slices and the grid
// ordered slice-major: while slice s runs, the feature-map bytes in play are
// 1/SL of the maps (P2 at 256^3: 1.07 GB -> 134 MB for SL = 8), so rows that
// overlapping ROIs read again come from the memory-side cache instead of HBM.
// A wave holds SL lines (consecutive x of one y) x one slice: 64/SL lanes per
// line, float4 each (C = 256: SL = 8 -> 128 B rows, one L2 line).  Per-sample
// arithmetic as line_fwd_kernel (bit-identical).  Needs C % (4 * 64 / SL) == 0
// ... and C/4 == 64 (C = 256) for the lane split below.
// PD > 0 (crop depth known at compile time, one z-part): the line's PD outputs
// are kept in registers and stored after the loop, so no corner load of the
// line waits behind an earlier output store (one vmcnt counter covers loads
// and stores) -- the z loop's loads can all be in flight at once.
template <int SL, int PD = 0>
__global__ __launch_bounds__(256) void line_fwd_sl_kernel(LineArgs a, Pyr P, const int32_t* __restrict__ perm,
                                                          int zs, const int32_t* __restrict__ wperm) {
    constexpr int LPL = 64 / SL;                      // lanes (float4) per line slice
    // blocks: SL slices in dispatch order, each a multiple of 8 blocks remapped
    // XCD-contiguously within the slice (hardware XCD = block % 8); a line is
    // cut into zs z-parts (more, shorter dependent load chains in flight)
    const int64_t items = a.lines * zs;
    const int64_t waves_per_slice = (items + SL - 1) / SL;
    const int64_t bs8 = ((waves_per_slice + 3) / 4 + 7) / 8 * 8;
    const int slice = (int)(blockIdx.x / bs8);
    const int64_t lr = blockIdx.x - (int64_t)slice * bs8;
    int64_t wv = ((lr % 8) * (bs8 / 8) + lr / 8) * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (slice >= SL || wv >= waves_per_slice) return;
    if (wperm) wv = wperm[wv];                        // spatially sorted wave order (lines stay per ROI)
    const int64_t item = wv * SL + lane / LPL;
    if (item >= items) return;
    int64_t line = item / zs;
    const int part = (int)(item - line * zs);
    const int zb = part * a.cd / zs, ze = (part + 1) * a.cd / zs;
    if (perm) line = perm[line];                      // spatially sorted line order
    const int c = slice * LPL + (lane % LPL);         // float4 index within the voxel
    int64_t t = line;
    const int x = (int)(t % a.cw); t /= a.cw;
    const int y = (int)(t % a.ch);
    const int64_t n = t / a.ch;
    const int l = a.levels[n] - 2;
    const int H = P.H[l], W = P.W[l], D = P.D[l];
    const float* img = P.fmaps[l] + (size_t)(n / a.N) * H * W * D * a.C;
    const float* box = a.boxes + n * 6;
    const float y1 = box[0], x1 = box[1], z1 = box[2], y2 = box[3], x2 = box[4], z2 = box[5];
    const float in_y = axis_coord(y1, y2, H, a.ch, y, axis_scale(y1, y2, H, a.ch));
    const float in_x = axis_coord(x1, x2, W, a.cw, x, axis_scale(x1, x2, W, a.cw));
    const float zsc = axis_scale(z1, z2, D, a.cd);
    const int C4 = a.C >> 2;
    float4* o = reinterpret_cast<float4*>(a.out + line * (int64_t)a.cd * a.C);
    const bool yx_oob = (in_y < 0 || in_y > (float)(H - 1)) || (in_x < 0 || in_x > (float)(W - 1));
    const float4 ex = make_float4(a.extrap, a.extrap, a.extrap, a.extrap);
    if (yx_oob) {
        for (int z = zb; z < ze; ++z) st_nt(o + (int64_t)z * C4 + c, ex);
        return;
    }
    const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
    const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
    const float yl = in_y - (float)ty, xl = in_x - (float)lx;
    const size_t rowD = (size_t)D * C4, rowW = (size_t)W * rowD;
    const float4* base = reinterpret_cast<const float4*>(img);
    const float4* col[4] = {base + ty * rowW + lx * rowD, base + ty * rowW + rx * rowD,
                            base + by * rowW + lx * rowD, base + by * rowW + rx * rowD};
    int pk = -1;
    float4 kv[4];
    // (no lambda around the body: capturing col / kv by reference put them in scratch)
    // PD > 0: this wave's z part (at most PD samples, zs = ceil(cd / PD) parts per
    // line) with its outputs held in registers and stored after the loop, so no
    // corner load waits behind an output store: loads and stores share vmcnt, and
    // with both kinds in flight the compiler can only wait with vmcnt(0)
    float4 res[PD > 0 ? PD : 1];
    const int n_it = PD > 0 ? PD : ze - zb;
#pragma unroll
    for (int zz = 0; zz < n_it; ++zz) {
        const int z = zb + zz;
        if (PD > 0 && z >= ze) break;
        const float in_z = axis_coord(z1, z2, D, a.cd, z, zsc);
        float4 r;
        if (in_z < 0 || in_z > (float)(D - 1)) {
            r = ex;
        } else {
            const int fz = (int)floorf(in_z), kz = (int)ceilf(in_z);
            const float zl = in_z - (float)fz;
            float4 fv[4];
#if defined(M3D_ROI_DBG) && M3D_ROI_DBG == 2
            // timing probe: no corner loads (values from the coordinates)
#pragma unroll
            for (int q = 0; q < 4; ++q) fv[q] = make_float4(in_z, yl, xl, (float)(fz + q));
            if (kz != fz) {
#pragma unroll
                for (int q = 0; q < 4; ++q) kv[q] = make_float4(yl, in_z, (float)(kz + q), xl);
            } else {
#else
            if (fz == pk) {
#pragma unroll
                for (int q = 0; q < 4; ++q) fv[q] = kv[q];
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) fv[q] = col[q][(size_t)fz * C4 + c];
            }
            if (kz != fz) {
#pragma unroll
                for (int q = 0; q < 4; ++q) kv[q] = col[q][(size_t)kz * C4 + c];
            } else {
#endif
#pragma unroll
                for (int q = 0; q < 4; ++q) kv[q] = fv[q];
            }
            pk = kz;
            r = tri4(fv[0], kv[0], fv[1], kv[1], fv[2], kv[2], fv[3], kv[3], yl, xl, zl);
            r.x = scrub(r.x); r.y = scrub(r.y); r.z = scrub(r.z); r.w = scrub(r.w);
        }
#if defined(M3D_ROI_DBG) && M3D_ROI_DBG == 1
        if (r.x == 1.2345f) st_nt(o + (int64_t)z * C4 + c, r);          // timing probe: no stores
        continue;
#endif
        if constexpr (PD > 0) res[zz] = r;
        else st_nt(o + (int64_t)z * C4 + c, r);
    }
    if constexpr (PD > 0) {
#pragma unroll
        for (int zz = 0; zz < PD; ++zz)
            if (zb + zz < ze) st_nt(o + (int64_t)(zb + zz) * C4 + c, res[zz]);
    }
}




// exclusive prefix sum of counts[0..n) into offs, one workgroup of 1024
__global__ __launch_bounds__(1024) void excl_scan_kernel(const int32_t* __restrict__ counts, int64_t n,
                                                         int32_t* __restrict__ offs) {
    __shared__ int32_t part[1024];
    const int tid = threadIdx.x;
    const int64_t per = (n + 1023) / 1024;
    const int64_t i0 = tid * per, i1 = min<int64_t>(n, i0 + per);
    int32_t sum = 0;
    for (int64_t i = i0; i < i1; ++i) sum += counts[i];
    part[tid] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int32_t v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int32_t run = part[tid] - sum;
    for (int64_t i = i0; i < i1; ++i) {
        offs[i] = run;
        run += counts[i];
    }
}

// Wave order (M3D_ROI_SORT=3): the SL consecutive lines of one wave (one ROI,
// consecutive x) stay together -- their z samples coincide, so the loop stays
// wave-uniform -- and the waves are counting-sorted by the owner (y, x) column
// of their first line, so waves of different, overlapping ROIs that read the
// same columns run next to each other on one XCD (band of rows per XCD).
__global__ void wave_key_kernel(LineArgs a, Pyr P, RegionBase rb, int sl, int64_t nwaves,
                                int32_t* __restrict__ keys, int32_t* __restrict__ counts) {
    const int64_t w = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwaves) return;
    int64_t t = w * sl;
    const int x = (int)(t % a.cw); t /= a.cw;
    const int y = (int)(t % a.ch);
    const int64_t n = t / a.ch;
    const int l = a.levels[n] - 2;
    const int H = P.H[l], W = P.W[l];
    const int64_t b = n / a.N;
    const float* box = a.boxes + n * 6;
    const int ty = owner_idx(axis_coord(box[0], box[3], H, a.ch, y, axis_scale(box[0], box[3], H, a.ch)), H);
    const int lx = owner_idx(axis_coord(box[1], box[4], W, a.cw, x, axis_scale(box[1], box[4], W, a.cw)), W);
    const int32_t k = (int32_t)(rb.base[l] + (b * H + ty) * W + lx);
    keys[w] = k;
    atomicAdd(counts + k, 1);
}

__global__ void line_scatter_kernel(const int32_t* __restrict__ keys, int64_t lines, int32_t* __restrict__ offs,
                                    int32_t* __restrict__ perm) {
    const int64_t L = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (L >= lines) return;
    perm[atomicAdd(offs + keys[L], 1)] = (int32_t)L;
}

static int roi_slices() {
    static constexpr int env = M3D_TUNE_ROI_SLICES;
    return env;
}

// ---- trilinear backward in gather form ----------------------------------------
// The 8-corner scatter of A.2 is separable: the gradient of voxel (Y,X,Z) is
// sum_{i,j,k} g[i][j][k] * ((wy(Y,i) * wx(X,j)) * wz(Z,k)), where wy(Y,i) is
// 1 - yl_i if ty_i == Y and yl_i if by_i == Y (two terms when ty_i == by_i),
// and samples outside the image along an axis contribute nothing (out of
// bounds along any axis = no contribution, so the validity is separable too).
// Corner slot s of an axis is corner s&1 (floor, ceil) of sample s>>1; lane s
// of every wave holds slot s of each axis (voxel, weight, validity), so the
// contributing slots of a voxel are one ballot.  One wave per (box, y slot,
// x slot); a slot whose voxel an earlier slot already names exits, so every
// touched (Y, X) column has one owner.  The wave walks the z slots the same
// way and per touched voxel sums the per-term products g * ((wy*wx)*wz) of the
// reference (only the summation order differs from the atomic scatter) from
// the box's gradient rows -- L2-resident, the box's waves are XCD-contiguous --
// and adds the sum with one atomic per channel instead of one per corner hit.
// Boxes whose sample spacing is below a voxel share corners: a 14^3 crop of a
// box spanning 8 voxels per axis makes 9*9*9 row atomics instead of 8*14^3.
// Needs ch, cw, cd <= 32 (slots <= 64 lanes) and C % 64 == 0 (lanes over C).
struct GatherArgs {
    const float* grads;          // [nbox, ch, cw, cd, C]
    const float* boxes;          // crop: [N,6]; pyramid: boxes_adj
    const int32_t* box_ind;      // crop
    const int32_t* levels;       // pyramid
    float* gimage;               // crop: [B,H,W,D,C]
    int64_t nbox, N;             // pyramid: N boxes per image
    int H, W, D, ch, cw, cd;
};

struct SlotTab {
    int vox;
    float w;
    bool ok;
};

// lane s: slot s of an axis with n samples over S voxels
__device__ __forceinline__ SlotTab slot_tab(float b1, float b2, int S, int n, int s) {
    SlotTab t{0, 0.0f, false};
    if (s >= 2 * n) return t;
    const float sc = axis_scale(b1, b2, S, n);
    const float in = axis_coord(b1, b2, S, n, s >> 1, sc);
    t.ok = !(in < 0 || in > (float)(S - 1));
    if (!t.ok) return t;
    const int lo = (int)floorf(in);
    const float l = in - (float)lo;
    t.vox = (s & 1) ? (int)ceilf(in) : lo;
    t.w = (s & 1) ? l : 1.0f - l;
    return t;
}

template <int CQ, bool PYR>
__global__ __launch_bounds__(256) void gather_bwd_kernel(GatherArgs a, Pyr P) {
    constexpr int C = 64 * CQ;
    const int64_t wv = xcd_block() * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int sxn = 2 * a.cw;
    const int64_t per_box = (int64_t)(2 * a.ch) * sxn;
    if (wv >= a.nbox * per_box) return;
    const int64_t n = wv / per_box;
    const int rem = (int)(wv - n * per_box);
    const int sy = rem / sxn, sx = rem - (rem / sxn) * sxn;
    int H, W, D;
    float* gimg;
    if (PYR) {
        const int l = a.levels[n] - 2;
        H = P.H[l]; W = P.W[l]; D = P.D[l];
        gimg = P.gmaps[l] + (size_t)(n / a.N) * H * W * D * C;
    } else {
        H = a.H; W = a.W; D = a.D;
        gimg = a.gimage + (size_t)a.box_ind[n] * H * W * D * C;
    }
    const float* box = a.boxes + n * 6;
    const SlotTab ty = slot_tab(box[0], box[3], H, a.ch, lane);
    const SlotTab tx = slot_tab(box[1], box[4], W, a.cw, lane);
    const SlotTab tz = slot_tab(box[2], box[5], D, a.cd, lane);
    // this wave's (Y, X) column, owned by its first slot
    if (!__builtin_amdgcn_readlane((int)ty.ok, sy) || !__builtin_amdgcn_readlane((int)tx.ok, sx)) return;
    const int Y = __builtin_amdgcn_readlane(ty.vox, sy), X = __builtin_amdgcn_readlane(tx.vox, sx);
    const uint64_t my = __ballot(ty.ok && ty.vox == Y), mx = __ballot(tx.ok && tx.vox == X);
    if ((my & ((1ull << sy) - 1)) || (mx & ((1ull << sx) - 1))) return;
    const float* g = a.grads + (size_t)n * a.ch * a.cw * a.cd * C + lane;
    float* dst = gimg + ((size_t)Y * W + X) * D * C + lane;
    const uint64_t zok = __ballot(tz.ok);
    for (int sz = 0; sz < 2 * a.cd; ++sz) {
        if (!((zok >> sz) & 1)) continue;
        const int Z = __builtin_amdgcn_readlane(tz.vox, sz);
        const uint64_t mz = __ballot(tz.ok && tz.vox == Z);
        if (mz & ((1ull << sz) - 1)) continue;            // voxel Z done at an earlier slot
        float acc[CQ];
#pragma unroll
        for (int q = 0; q < CQ; ++q) acc[q] = 0.0f;
        for (uint64_t m1 = my; m1; m1 &= m1 - 1) {
            const int s1 = __builtin_ctzll(m1);
            const float wy = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, ty.w), s1));
            for (uint64_t m2 = mx; m2; m2 &= m2 - 1) {
                const int s2 = __builtin_ctzll(m2);
                const float wx = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tx.w), s2));
                const float wyx = wy * wx;
                const float* gyx = g + ((size_t)(s1 >> 1) * a.cw + (s2 >> 1)) * a.cd * C;
                for (uint64_t m3 = mz; m3; m3 &= m3 - 1) {
                    const int s3 = __builtin_ctzll(m3);
                    const float wz = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, tz.w), s3));
                    const float w = wyx * wz;
                    const float* gr = gyx + (size_t)(s3 >> 1) * C;
#pragma unroll
                    for (int q = 0; q < CQ; ++q) acc[q] += gr[64 * q] * w;
                }
            }
        }
#pragma unroll
        for (int q = 0; q < CQ; ++q) unsafeAtomicAdd(dst + (size_t)Z * C + 64 * q, acc[q]);
    }
}

// the gather-form backward for C in {64, 128, 256, 512} and crops <= 32 per
// axis (the per-sample atomic scatter elsewhere)
static bool gather_bwd_ok(int64_t C, int ch, int cw, int cd) {
    return (C == 64 || C == 128 || C == 256 || C == 512) && ch <= 32 && cw <= 32 && cd <= 32;
}

template <bool PYR>
static void launch_gather_bwd(const GatherArgs& a, const Pyr& P, int64_t C, hipStream_t s) {
    const unsigned grid = grid_for(a.nbox * 4 * a.ch * a.cw, 4);
    switch (C) {
        case 64: hipLaunchKernelGGL((gather_bwd_kernel<1, PYR>), dim3(grid), dim3(256), 0, s, a, P); break;
        case 128: hipLaunchKernelGGL((gather_bwd_kernel<2, PYR>), dim3(grid), dim3(256), 0, s, a, P); break;
        case 256: hipLaunchKernelGGL((gather_bwd_kernel<4, PYR>), dim3(grid), dim3(256), 0, s, a, P); break;
        default: hipLaunchKernelGGL((gather_bwd_kernel<8, PYR>), dim3(grid), dim3(256), 0, s, a, P);
    }
}

// ------------------------------------------------------------------ kernels
__global__ __launch_bounds__(256) void crop_fwd_kernel(const float* __restrict__ image, int B,
                                                       int H, int W, int D, int C,
                                                       const float* __restrict__ boxes,
                                                       const int32_t* __restrict__ box_ind,
                                                       int64_t total, int ch, int cw, int cd,
                                                       int method, float extrap,
                                                       float* __restrict__ crops) {
    const int64_t sidx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sidx >= total) return;
    int64_t t = sidx;
    const int z = (int)(t % cd); t /= cd;
    const int x = (int)(t % cw); t /= cw;
    const int y = (int)(t % ch);
    const int64_t n = t / ch;
    const Sample s = make_sample(boxes + n * 6, H, W, D, ch, cw, cd, y, x, z);
    const float* img = image + (size_t)box_ind[n] * H * W * D * C;
    emit_sample<false>(img, W, D, C, s, method, extrap, crops + sidx * C, lane);
}

__global__ __launch_bounds__(256) void crop_bwd_atomic_kernel(
    const float* __restrict__ grads, const float* __restrict__ boxes,
    const int32_t* __restrict__ box_ind, int64_t total, int ch, int cw, int cd, int H, int W,
    int D, int C, int method, float* __restrict__ gimg) {
    const int64_t sidx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sidx >= total) return;
    int64_t t = sidx;
    const int z = (int)(t % cd); t /= cd;
    const int x = (int)(t % cw); t /= cw;
    const int y = (int)(t % ch);
    const int64_t n = t / ch;
    const Sample s = make_sample(boxes + n * 6, H, W, D, ch, cw, cd, y, x, z);
    float* img = gimg + (size_t)box_ind[n] * H * W * D * C;
    scatter_sample(img, W, D, C, s, method, grads + sidx * C, lane);
}

// Deterministic replay: one thread per (image b, channel c) walks every box of
// image b in the reference order box -> y -> x -> z and accumulates the 8
// corners sequentially (bit-identical to the reference summation order).
__global__ __launch_bounds__(256) void crop_bwd_serial_kernel(
    const float* __restrict__ grads, const float* __restrict__ boxes,
    const int32_t* __restrict__ box_ind, int64_t N, int ch, int cw, int cd, int B, int H, int W,
    int D, int C, int method, float* __restrict__ gimg) {
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (tid >= (int64_t)B * C) return;
    const int b = (int)(tid / C), c = (int)(tid % C);
    float* img = gimg + (size_t)b * H * W * D * C;
    const size_t rowD = (size_t)D * C, rowW = (size_t)W * rowD;
    for (int64_t n = 0; n < N; ++n) {
        if (box_ind[n] != b) continue;
        for (int y = 0; y < ch; ++y)
            for (int x = 0; x < cw; ++x)
                for (int z = 0; z < cd; ++z) {
                    const Sample s = make_sample(boxes + n * 6, H, W, D, ch, cw, cd, y, x, z);
                    if (s.oob) continue;
                    const float gv = grads[((((size_t)n * ch + y) * cw + x) * cd + z) * C + c];
                    if (method == 1) {
                        img[s.ny * rowW + s.nx * rowD + (size_t)s.nz * C + c] += gv;
                        continue;
                    }
                    const float wy[2] = {1.0f - s.yl, s.yl}, wx[2] = {1.0f - s.xl, s.xl},
                                wz[2] = {1.0f - s.zl, s.zl};
                    const int iy[2] = {s.ty, s.by}, ix[2] = {s.lx, s.rx}, iz[2] = {s.fz, s.kz};
                    for (int a = 0; a < 2; ++a)
                        for (int bb = 0; bb < 2; ++bb)
                            for (int cc = 0; cc < 2; ++cc) {
                                const float w = (wy[a] * wx[bb]) * wz[cc];
                                img[iy[a] * rowW + ix[bb] * rowD + (size_t)iz[cc] * C + c] +=
                                    gv * w;
                            }
                }
    }
}

// Deterministic grad_image, segmented by destination: every voxel row of the
// output is owned by one thread (its channels by a float4 / float lane), which
// walks the contributions it receives in the reference order and keeps the
// running fp32 sum in a register -- so no atomics, no zero fill (every voxel is
// stored once) and the same bits as crop_bwd_serial_kernel's sequential replay.
//
// Why the order is the replay's: restricted to one destination voxel, the
// replay adds terms in (box n, y, x, z, corner) order.  Per sample at most ONE
// corner with a nonzero weight lands on a given voxel (two corners coincide
// only when floor == ceil, i.e. the lerp is exactly 0 and the second corner's
// weight is 0), and adding a zero term to the running sum never changes it
// (the sum starts at +0 and round-to-nearest never produces -0 from +0, so
// x + (+-0) == x for every reachable x; non-finite gradients still propagate
// because every term is still added).  The thread therefore enumerates
// n ascending, then (y sample, corner side), (x sample, side), (z sample,
// side) ascending, which visits every nonzero term in replay order.
//
// Mapping: block = (image b, row Y, column X, 256 consecutive (Z, channel
// vector) destinations); lanes test 64 boxes at a time against the column
// (conservative per-axis voxel ranges from the end samples: the sample
// coordinate is monotone in the sample index), then per relevant box the
// exact hit masks come from one ballot per axis (lane = sample index).  The
// terms g * ((wy * wx) * wz) are formed exactly as the replay forms them
// (-ffp-contract=off).  Needs crop sizes <= 64 (one lane per sample).
template <int VEC>
__global__ __launch_bounds__(256) void crop_bwd_det_kernel(
    const float* __restrict__ grads, const float* __restrict__ boxes,
    const int32_t* __restrict__ box_ind, int64_t N, int ch, int cw, int cd, int B, int H, int W,
    int D, int C, int method, int64_t blocks_per_col, float* __restrict__ gimg) {
    const int CV = C / VEC;
    const int lane = threadIdx.x & 63;
    const int64_t ncols = (int64_t)B * H * W;
    // Z values per wave when every wave holds whole Z rows of channel vectors
    // (CV a multiple or a divisor of 64); 0: per-thread z sample loop
    const int zpw = CV % 64 == 0 ? 1 : (64 % CV == 0 ? 64 / CV : 0);
    auto rdl = [](float v, int l) {
        return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
    };
    for (int64_t blk = blockIdx.x; blk < ncols * blocks_per_col; blk += gridDim.x) {
        const int64_t col = blk / blocks_per_col;
        const int64_t idx = (blk - col * blocks_per_col) * 256 + threadIdx.x;
        const bool active = idx < (int64_t)D * CV;
        const int Z = active ? (int)(idx / CV) : 0;
        const int cv = active ? (int)(idx - (int64_t)Z * CV) : 0;
        const int X = (int)(col % W);
        const int Y = (int)((col / W) % H);
        const int b = (int)(col / ((int64_t)H * W));
        // this wave's destination Z range (for the conservative box test)
        const int64_t wbase = (blk - col * blocks_per_col) * 256 + (threadIdx.x & ~63);
        const int zw0 = (int)min<int64_t>(wbase / CV, D - 1);
        const int zw1 = (int)min<int64_t>((wbase + 63) / CV, D - 1);
        float acc[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
        for (int64_t n0 = 0; n0 < N; n0 += 64) {
            bool rel = false;
            const int64_t nl = n0 + lane;
            if (nl < N && box_ind[nl] == b) {
                const float* bx = boxes + nl * 6;
                auto cover = [](float b1, float b2, int S, int n, float lo_v, float hi_v) {
                    const float sc = axis_scale(b1, b2, S, n);
                    const float e0 = axis_coord(b1, b2, S, n, 0, sc);
                    const float e1 = axis_coord(b1, b2, S, n, n - 1, sc);
                    const float lo = fminf(e0, e1), hi = fmaxf(e0, e1);
                    // NaN coordinates keep the box (the exact test then finds no sample)
                    return !(hi_v < floorf(lo) || lo_v > ceilf(hi));
                };
                rel = cover(bx[0], bx[3], H, ch, (float)Y, (float)Y) &&
                      cover(bx[1], bx[4], W, cw, (float)X, (float)X) &&
                      cover(bx[2], bx[5], D, cd, (float)zw0, (float)zw1);
            }
            for (uint64_t rm = __ballot(rel); rm; rm &= rm - 1) {
                const int64_t n = n0 + __builtin_ctzll(rm);
                const float* bx = boxes + n * 6;
                const float y1 = bx[0], x1 = bx[1], z1 = bx[2], y2 = bx[3], x2 = bx[4], z2 = bx[5];
                // lane i: sample i of the y and x axes (make_sample's maths)
                const float in_y = axis_coord(y1, y2, H, ch, lane, axis_scale(y1, y2, H, ch));
                const float in_x = axis_coord(x1, x2, W, cw, lane, axis_scale(x1, x2, W, cw));
                const bool vy = lane < ch && !(in_y < 0 || in_y > (float)(H - 1));
                const bool vx = lane < cw && !(in_x < 0 || in_x > (float)(W - 1));
                const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
                const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
                const float yl = in_y - (float)ty, xl = in_x - (float)lx;
                uint64_t myt, myb, mxl, mxr;
                if (method == 1) {
                    myt = __ballot(vy && (int)roundf(in_y) == Y);
                    mxl = __ballot(vx && (int)roundf(in_x) == X);
                    myb = mxr = 0;
                } else {
                    myt = __ballot(vy && ty == Y);
                    myb = __ballot(vy && by == Y);
                    mxl = __ballot(vx && lx == X);
                    mxr = __ballot(vx && rx == X);
                }
                // (uniform from here to the per-thread z loops: the readlanes below
                // must run with every lane active, or a value the compiler sinks into
                // a divergent block is missing in the lanes that skipped it)
                if (!(myt | myb) || !(mxl | mxr)) continue;
                // this thread's z samples / corner sides
                const float zsc = axis_scale(z1, z2, D, cd);
                uint64_t mzf = 0, mzk = 0;
                if (zpw > 0) {
                    // the wave holds zpw consecutive Z values: lane i computes z sample i
                    // once, one ballot per (Z, side) gives every thread its masks (instead
                    // of cd coordinate evaluations per thread and box)
                    const float in_zl = axis_coord(z1, z2, D, cd, lane, zsc);
                    const bool vz = lane < cd && !(in_zl < 0 || in_zl > (float)(D - 1));
                    const int fzl = method == 1 ? (int)roundf(in_zl) : (int)floorf(in_zl);
                    const int kzl = (int)ceilf(in_zl);
                    for (int g = 0; g < zpw; ++g) {
                        const int Zg = zw0 + g;
                        const uint64_t f = __ballot(vz && fzl == Zg);
                        const uint64_t k = method == 1 ? 0ull : __ballot(vz && kzl == Zg);
                        if (active && Z == Zg) {
                            mzf = f;
                            mzk = k;
                        }
                    }
                    if (__ballot((mzf | mzk) != 0) == 0) continue;      // wave-uniform skip
                } else {
                    for (int i = 0; i < cd && active; ++i) {
                        const float in_z = axis_coord(z1, z2, D, cd, i, zsc);
                        if (in_z < 0 || in_z > (float)(D - 1)) continue;
                        if (method == 1) {
                            if ((int)roundf(in_z) == Z) mzf |= 1ull << i;
                            continue;
                        }
                        if ((int)floorf(in_z) == Z) mzf |= 1ull << i;
                        if ((int)ceilf(in_z) == Z) mzk |= 1ull << i;
                    }
                }
                const float* gn = grads + (size_t)n * ch * cw * cd * C + (size_t)cv * VEC;
                if (method == 1) {                          // nearest: img[ny,nx,nz] += g
                    for (uint64_t m1 = myt; m1; m1 &= m1 - 1)
                        for (uint64_t m2 = mxl; m2; m2 &= m2 - 1) {
                            const float* gyx = gn + ((size_t)__builtin_ctzll(m1) * cw + __builtin_ctzll(m2)) * cd * C;
                            for (uint64_t m3 = mzf; m3; m3 &= m3 - 1) {
                                const float* gr = gyx + (size_t)__builtin_ctzll(m3) * C;
#pragma unroll
                                for (int q = 0; q < VEC; ++q) acc[q] += gr[q];
                            }
                        }
                    continue;
                }
                for (uint64_t m1 = myt | myb; m1; m1 &= m1 - 1) {
                    const int iy = __builtin_ctzll(m1);
                    const float yli = rdl(yl, iy);
                    for (int a = 0; a < 2; ++a) {
                        if (!(((a ? myb : myt) >> iy) & 1)) continue;
                        const float wy = a ? yli : 1.0f - yli;
                        for (uint64_t m2 = mxl | mxr; m2; m2 &= m2 - 1) {
                            const int ix = __builtin_ctzll(m2);
                            const float xli = rdl(xl, ix);
                            for (int bb = 0; bb < 2; ++bb) {
                                if (!(((bb ? mxr : mxl) >> ix) & 1)) continue;
                                const float wyx = wy * (bb ? xli : 1.0f - xli);
                                const float* gyx = gn + ((size_t)iy * cw + ix) * cd * C;
                                for (uint64_t m3 = mzf | mzk; m3; m3 &= m3 - 1) {
                                    const int iz = __builtin_ctzll(m3);
                                    const float in_z = axis_coord(z1, z2, D, cd, iz, zsc);
                                    const float zli = in_z - floorf(in_z);
                                    const float* gr = gyx + (size_t)iz * C;
                                    float gv[VEC];
#pragma unroll
                                    for (int q = 0; q < VEC; ++q) gv[q] = gr[q];
                                    for (int cc = 0; cc < 2; ++cc) {
                                        if (!(((cc ? mzk : mzf) >> iz) & 1)) continue;
                                        const float w = wyx * (cc ? zli : 1.0f - zli);
#pragma unroll
                                        for (int q = 0; q < VEC; ++q) acc[q] += gv[q] * w;
                                    }
                                }
                            }
                        }
                    }
                }
            }
        }
        if (active) {
            float* dst = gimg + ((((size_t)b * H + Y) * W + X) * D + Z) * C + (size_t)cv * VEC;
            if constexpr (VEC == 4)
                *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
            else
                dst[0] = acc[0];
        }
    }
}

// Sample hit masks of one axis for one box (crop_bwd_det_col_kernel's list
// build): bit i of lo / hi set when sample i lies in the image and its floor /
// ceil voxel (nearest: its rounded voxel, in lo) is V.  The sample coordinate
// a + i*sc is monotone in i, so only indices within two of the range where it
// can lie in (V - 1, V + 1) are tested -- each with axis_coord, the kernels'
// own arithmetic; at spacings below 1e-3 voxel every sample is tested.
__device__ __forceinline__ void det_axis_hits(float b1, float b2, int S, int n, int V, int method, uint64_t& lo,
                                              uint64_t& hi) {
    lo = hi = 0;
    const float sc = axis_scale(b1, b2, S, n);
    int i0 = 0, i1 = n - 1;
    if (n > 1 && fabsf(sc) >= 1e-3f) {
        const float a = b1 * (float)(S - 1);
        float r0 = ((float)(V - 1) - a) / sc, r1 = ((float)(V + 1) - a) / sc;
        if (r0 > r1) { const float t = r0; r0 = r1; r1 = t; }
        if (!(r1 >= -2.0f) || !(r0 <= (float)(n + 1))) return;       // (NaN boxes: no sample)
        i0 = max(0, (int)floorf(r0) - 2);
        i1 = min(n - 1, (int)ceilf(r1) + 2);
    }
    for (int i = i0; i <= i1; ++i) {
        const float c = axis_coord(b1, b2, S, n, i, sc);
        if (c < 0 || c > (float)(S - 1)) continue;
        if (method == 1) {
            if ((int)roundf(c) == V) lo |= 1ull << i;
            continue;
        }
        if ((int)floorf(c) == V) lo |= 1ull << i;
        if ((int)ceilf(c) == V) hi |= 1ull << i;
    }
}

// Deterministic grad_image, column form (the default of mode 1 when the boxes
// fit the list): a workgroup owns one voxel column (b, Y, X) and a range of its
// (Z, channel-vector) chunks.  Wave 0 first scans the boxes once, in ascending
// order, and keeps in LDS only those whose y and x samples really hit the
// column (exact per-axis ballots, lane = sample index), with their hit masks;
// every chunk then walks that short list -- instead of re-testing all boxes,
// and re-deriving the y / x hits, for every 256 destinations of the column.
// Per destination the terms, their order (box -> y -> x -> z -> corner) and
// the arithmetic are crop_bwd_det_kernel's: bit-identical.
constexpr int DET_CAP = 512;        // boxes per column list (host falls back above N = DET_CAP)
constexpr int DET_CHUNKS = 8;       // 256-destination chunks per workgroup

template <int VEC>
__global__ __launch_bounds__(256) void crop_bwd_det_col_kernel(
    const float* __restrict__ grads, const float* __restrict__ boxes,
    const int32_t* __restrict__ box_ind, int64_t N, int ch, int cw, int cd, int B, int H, int W,
    int D, int C, int method, int64_t blocks_per_col, float* __restrict__ gimg) {
    __shared__ int32_t ln[DET_CAP];
    __shared__ uint64_t lm[DET_CAP][4];          // y top / bottom, x left / right hit masks
    __shared__ float lb[DET_CAP][8];             // the box, its z scale and first-sample z (broadcast reads)
    __shared__ int lcount;
    const int CV = C / VEC;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int zpw = CV % 64 == 0 ? 1 : (64 % CV == 0 ? 64 / CV : 0);
    const int64_t col = blockIdx.x / blocks_per_col;
    const int64_t part = blockIdx.x - col * blocks_per_col;
    const int X = (int)(col % W);
    const int Y = (int)((col / W) % H);
    const int b = (int)(col / ((int64_t)H * W));
    const int64_t nchunks = ((int64_t)D * CV + 255) / 256;
    const int64_t c0 = part * DET_CHUNKS;
    const int64_t c1 = c0 + DET_CHUNKS < nchunks ? c0 + DET_CHUNKS : nchunks;
    if (c0 >= c1) return;                        // (uniform per block)
    // this block's Z range, for the conservative z part of the box test
    const int zb0 = (int)min<int64_t>(c0 * 256 / CV, D - 1);
    const int zb1 = (int)min<int64_t>((c1 * 256 - 1) / CV, D - 1);
    // lane = box: per-axis hit masks of sample indices (exact: every sample in a
    // conservative index range is tested with the kernel's coordinate maths).
    // Wave w takes the 64-box groups w and w + 4 (DET_CAP = 8 groups), counts
    // its hits per group, and after a prefix over the groups writes them in
    // ascending box order.
    static_assert(DET_CAP == 8 * 64, "two 64-box groups per wave");
    __shared__ int gcnt[8];
    uint64_t hm[2], my[2][4];
    bool hit[2];
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int64_t nl = (int64_t)(wave + 4 * r) * 64 + lane;
        hit[r] = false;
        my[r][0] = my[r][1] = my[r][2] = my[r][3] = 0;
        if (nl < N && box_ind[nl] == b) {
            const float* bx = boxes + nl * 6;
            const float z1 = bx[2], z2 = bx[5];
            const float zsc = axis_scale(z1, z2, D, cd);
            const float ze0 = axis_coord(z1, z2, D, cd, 0, zsc), ze1 = axis_coord(z1, z2, D, cd, cd - 1, zsc);
            if (!((float)zb1 < floorf(fminf(ze0, ze1)) || (float)zb0 > ceilf(fmaxf(ze0, ze1)))) {
                det_axis_hits(bx[0], bx[3], H, ch, Y, method, my[r][0], my[r][1]);
                if (my[r][0] | my[r][1]) det_axis_hits(bx[1], bx[4], W, cw, X, method, my[r][2], my[r][3]);
                hit[r] = (my[r][0] | my[r][1]) && (my[r][2] | my[r][3]);
            }
        }
        hm[r] = __ballot(hit[r]);
        if (lane == 0) gcnt[wave + 4 * r] = __builtin_popcountll(hm[r]);
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 2; ++r) {
        const int g = wave + 4 * r;
        int base = 0;
        for (int q = 0; q < g; ++q) base += gcnt[q];
        if (hit[r]) {
            const int64_t nl = (int64_t)g * 64 + lane;
            const int slot = base + __builtin_popcountll(hm[r] & ((1ull << lane) - 1));
            ln[slot] = (int32_t)nl;
#pragma unroll
            for (int q = 0; q < 4; ++q) lm[slot][q] = my[r][q];
            const float* bx = boxes + nl * 6;
#pragma unroll
            for (int q = 0; q < 6; ++q) lb[slot][q] = bx[q];
            lb[slot][6] = axis_scale(bx[2], bx[5], D, cd);
        }
    }
    if (threadIdx.x == 0) {
        int t = 0;
        for (int q = 0; q < 8; ++q) t += gcnt[q];
        lcount = t;
    }
    __syncthreads();
    const int nlist = lcount;
    for (int64_t c = c0; c < c1; ++c) {
        const int64_t idx = c * 256 + threadIdx.x;
        const bool active = idx < (int64_t)D * CV;
        const int Z = active ? (int)(idx / CV) : 0;
        const int cv = active ? (int)(idx - (int64_t)Z * CV) : 0;
        const int zw0 = (int)min<int64_t>((c * 256 + wave * 64) / CV, D - 1);
        float acc[VEC];
#pragma unroll
        for (int q = 0; q < VEC; ++q) acc[q] = 0.0f;
        for (int e = 0; e < nlist; ++e) {
            const int64_t n = ln[e];
            const uint64_t myt = lm[e][0], myb = lm[e][1], mxl = lm[e][2], mxr = lm[e][3];
            const float y1 = lb[e][0], x1 = lb[e][1], z1 = lb[e][2], y2 = lb[e][3], x2 = lb[e][4], z2 = lb[e][5];
            const float zsc = lb[e][6];
            uint64_t mzf = 0, mzk = 0;
            if (zpw > 0) {
                const float in_zl = axis_coord(z1, z2, D, cd, lane, zsc);
                const bool vz = lane < cd && !(in_zl < 0 || in_zl > (float)(D - 1));
                const int fzl = method == 1 ? (int)roundf(in_zl) : (int)floorf(in_zl);
                const int kzl = (int)ceilf(in_zl);
                for (int g = 0; g < zpw; ++g) {
                    const int Zg = zw0 + g;
                    const uint64_t f = __ballot(vz && fzl == Zg);
                    const uint64_t k = method == 1 ? 0ull : __ballot(vz && kzl == Zg);
                    if (active && Z == Zg) {
                        mzf = f;
                        mzk = k;
                    }
                }
                if (__ballot((mzf | mzk) != 0) == 0) continue;      // wave-uniform skip
            } else {
                for (int i = 0; i < cd && active; ++i) {
                    const float in_z = axis_coord(z1, z2, D, cd, i, zsc);
                    if (in_z < 0 || in_z > (float)(D - 1)) continue;
                    if (method == 1) {
                        if ((int)roundf(in_z) == Z) mzf |= 1ull << i;
                        continue;
                    }
                    if ((int)floorf(in_z) == Z) mzf |= 1ull << i;
                    if ((int)ceilf(in_z) == Z) mzk |= 1ull << i;
                }
            }
            const float* gn = grads + (size_t)n * ch * cw * cd * C + (size_t)cv * VEC;
            if (method == 1) {                          // nearest: img[ny,nx,nz] += g
                for (uint64_t m1 = myt; m1; m1 &= m1 - 1)
                    for (uint64_t m2 = mxl; m2; m2 &= m2 - 1) {
                        const float* gyx = gn + ((size_t)__builtin_ctzll(m1) * cw + __builtin_ctzll(m2)) * cd * C;
                        for (uint64_t m3 = mzf; m3; m3 &= m3 - 1) {
                            const float* gr = gyx + (size_t)__builtin_ctzll(m3) * C;
#pragma unroll
                            for (int q = 0; q < VEC; ++q) acc[q] += gr[q];
                        }
                    }
                continue;
            }
            const float ysc = axis_scale(y1, y2, H, ch), xsc = axis_scale(x1, x2, W, cw);
            for (uint64_t m1 = myt | myb; m1; m1 &= m1 - 1) {
                const int iy = __builtin_ctzll(m1);
                const float in_y = axis_coord(y1, y2, H, ch, iy, ysc);
                const float yli = in_y - floorf(in_y);
                for (int a = 0; a < 2; ++a) {
                    if (!(((a ? myb : myt) >> iy) & 1)) continue;
                    const float wy = a ? yli : 1.0f - yli;
                    for (uint64_t m2 = mxl | mxr; m2; m2 &= m2 - 1) {
                        const int ix = __builtin_ctzll(m2);
                        const float in_x = axis_coord(x1, x2, W, cw, ix, xsc);
                        const float xli = in_x - floorf(in_x);
                        for (int bb = 0; bb < 2; ++bb) {
                            if (!(((bb ? mxr : mxl) >> ix) & 1)) continue;
                            const float wyx = wy * (bb ? xli : 1.0f - xli);
                            const float* gyx = gn + ((size_t)iy * cw + ix) * cd * C;
                            for (uint64_t m3 = mzf | mzk; m3; m3 &= m3 - 1) {
                                const int iz = __builtin_ctzll(m3);
                                const float in_z = axis_coord(z1, z2, D, cd, iz, zsc);
                                const float zli = in_z - floorf(in_z);
                                const float* gr = gyx + (size_t)iz * C;
                                float gv[VEC];
#pragma unroll
                                for (int q = 0; q < VEC; ++q) gv[q] = gr[q];
                                for (int cc = 0; cc < 2; ++cc) {
                                    if (!(((cc ? mzk : mzf) >> iz) & 1)) continue;
                                    const float w = wyx * (cc ? zli : 1.0f - zli);
#pragma unroll
                                    for (int q = 0; q < VEC; ++q) acc[q] += gv[q] * w;
                                }
                            }
                        }
                    }
                }
            }
        }
        if (active) {
            float* dst = gimg + ((((size_t)b * H + Y) * W + X) * D + Z) * C + (size_t)cv * VEC;
            if constexpr (VEC == 4)
                *reinterpret_cast<float4*>(dst) = make_float4(acc[0], acc[1], acc[2], acc[3]);
            else
                dst[0] = acc[0];
        }
    }
}

// launch of the deterministic grad_image into one image set: the column-list
// kernel when the boxes fit its list and its one-block-per-(column, chunk
// group) grid fits the launch limit (grid x * 256 threads < 2^32), else
// crop_bwd_det_kernel (block-strided, capped grid); both are bit-identical to
// the sequential replay
static void launch_det_bwd(const float* grads, const float* boxes, const int32_t* box_ind, int64_t N, int ch,
                           int cw, int cd, int64_t B, int64_t H, int64_t W, int64_t D, int64_t C, int method,
                           float* gimg, hipStream_t s) {
    const bool v4 = (C & 3) == 0;
    const int64_t cvn = v4 ? C / 4 : C;
    const int64_t nchunks = (D * cvn + 255) / 256;
    const int64_t bpc = (nchunks + DET_CHUNKS - 1) / DET_CHUNKS;
    if (N <= DET_CAP && B * H * W * bpc < ((int64_t)1 << 24)) {
        const int64_t nblk = B * H * W * bpc;
        if (v4)
            hipLaunchKernelGGL(crop_bwd_det_col_kernel<4>, dim3((unsigned)nblk), dim3(256), 0, s, grads, boxes,
                               box_ind, N, ch, cw, cd, (int)B, (int)H, (int)W, (int)D, (int)C, method, bpc, gimg);
        else
            hipLaunchKernelGGL(crop_bwd_det_col_kernel<1>, dim3((unsigned)nblk), dim3(256), 0, s, grads, boxes,
                               box_ind, N, ch, cw, cd, (int)B, (int)H, (int)W, (int)D, (int)C, method, bpc, gimg);
        return;
    }
    const int64_t nblk = B * H * W * nchunks;
    const unsigned grid = (unsigned)std::min<int64_t>(nblk, 1 << 20);
    if (v4)
        hipLaunchKernelGGL(crop_bwd_det_kernel<4>, dim3(grid), dim3(256), 0, s, grads, boxes, box_ind, N, ch, cw,
                           cd, (int)B, (int)H, (int)W, (int)D, (int)C, method, nchunks, gimg);
    else
        hipLaunchKernelGGL(crop_bwd_det_kernel<1>, dim3(grid), dim3(256), 0, s, grads, boxes, box_ind, N, ch, cw,
                           cd, (int)B, (int)H, (int)W, (int)D, (int)C, method, nchunks, gimg);
}

// CropAndResize3DGradBoxes with the wheel's compiled formulas (DESIGN.md A.4,
// whl _crop_and_resize_3d_grad_boxes_ops.so Compute @0x3980): ratios
// (S-1)/(n-1), the depth scale (z2 - y1)(H-1)/(ch-1) as compiled, image
// gradients in the compiled association, out[a] += ((S-1) - r i) g_a and
// out[a+3] += (g_a i) r, or the double-precision update for n == 1.  One wave
// per box: the sample loop is wave-uniform, lanes compute the terms of 64
// channels, and the six outputs take them one channel after the other in the
// reference order (box -> y -> x -> z -> c), so the result is bit-identical
// to the sequential CPU op (oracle_crop_and_resize3d_grad_boxes).
__device__ __forceinline__ float lanef(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double laned(double v, int l) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)u, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), l);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// per-channel terms of one axis: float pair (n > 1) or the double term (n == 1)
struct GbTerm {
    float lo, hi;
    double d;
};
__device__ __forceinline__ GbTerm gb_term(int n, int i, float g, float r, int S) {
    GbTerm t{};
    if (n > 1) {
        t.lo = ((float)(S - 1) - r * (float)i) * g;
        t.hi = (g * (float)i) * r;
        t.d = 0.0;
    } else {
        t.lo = t.hi = 0.0f;
        t.d = (double)g * 0.5 * (double)(S - 1);
    }
    return t;
}
__device__ __forceinline__ void gb_acc(int n, const GbTerm& t, int l, float& a, float& b) {
    if (n > 1) {
        a += lanef(t.lo, l);
        b += lanef(t.hi, l);
    } else {
        const double d = laned(t.d, l);
        a = (float)((double)a + d);
        b = (float)(d + (double)b);
    }
}

__global__ __launch_bounds__(64) void crop_bwd_boxes_kernel(
    const float* __restrict__ grads, const float* __restrict__ image, int B, int H, int W, int D,
    int C, const float* __restrict__ boxes, const int32_t* __restrict__ box_ind, int ch, int cw,
    int cd, float* __restrict__ gboxes) {
    const int n = blockIdx.x, lane = threadIdx.x;
    const float* bx = boxes + (size_t)n * 6;
    const float y1 = bx[0], x1 = bx[1], z1 = bx[2], y2 = bx[3], x2 = bx[4], z2 = bx[5];
    const float* img = image + (size_t)box_ind[n] * H * W * D * C;
    const float hr = ch > 1 ? (float)(H - 1) / (float)(ch - 1) : 0.0f;
    const float wr = cw > 1 ? (float)(W - 1) / (float)(cw - 1) : 0.0f;
    const float dr = cd > 1 ? (float)(D - 1) / (float)(cd - 1) : 0.0f;
    const float hs = ch > 1 ? (y2 - y1) * hr : 0.0f;
    const float ws = cw > 1 ? (x2 - x1) * wr : 0.0f;
    const float ds = cd > 1 ? (z2 - y1) * hr : 0.0f;       // sic: the compiled depth scale (A.4)
    float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f, a3 = 0.0f, a4 = 0.0f, a5 = 0.0f;
    const size_t rowD = (size_t)D * C, rowW = (size_t)W * rowD;
    for (int y = 0; y < ch; ++y) {
        const float in_y = axis_coord(y1, y2, H, ch, y, hs);
        if (in_y < 0 || in_y > (float)(H - 1)) continue;
        const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
        const float yl = in_y - (float)ty, yl1 = 1.0f - yl;
        for (int x = 0; x < cw; ++x) {
            const float in_x = axis_coord(x1, x2, W, cw, x, ws);
            if (in_x < 0 || in_x > (float)(W - 1)) continue;
            const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
            const float xl = in_x - (float)lx, xl1 = 1.0f - xl;
            for (int z = 0; z < cd; ++z) {
                const float in_z = axis_coord(z1, z2, D, cd, z, ds);
                if (in_z < 0 || in_z > (float)(D - 1)) continue;
                const int fz = (int)floorf(in_z), kz = (int)ceilf(in_z);
                const float zl = in_z - (float)fz, zl1 = 1.0f - zl;
                const float* gr = grads + ((((size_t)n * ch + y) * cw + x) * cd + z) * C;
                for (int c0 = 0; c0 < C; c0 += 64) {
                    const int c = c0 + lane;
                    float igy = 0.0f, igx = 0.0f, igz = 0.0f, tg = 0.0f;
                    if (c < C) {
                        const float tlf = img[ty * rowW + lx * rowD + (size_t)fz * C + c];
                        const float tlk = img[ty * rowW + lx * rowD + (size_t)kz * C + c];
                        const float trf = img[ty * rowW + rx * rowD + (size_t)fz * C + c];
                        const float trk = img[ty * rowW + rx * rowD + (size_t)kz * C + c];
                        const float blf = img[by * rowW + lx * rowD + (size_t)fz * C + c];
                        const float blk = img[by * rowW + lx * rowD + (size_t)kz * C + c];
                        const float brf = img[by * rowW + rx * rowD + (size_t)fz * C + c];
                        const float brk = img[by * rowW + rx * rowD + (size_t)kz * C + c];
                        igy = ((blf - tlf) * xl1 + (brf - trf) * xl) * zl1 + ((blk - tlk) * xl1 + (brk - trk) * xl) * zl;
                        igx = ((trf - tlf) * yl1 + (brf - blf) * yl) * zl1 + ((trk - tlk) * yl1 + (brk - blk) * yl) * zl;
                        igz = ((tlk - tlf) * yl1 + (blk - blf) * yl) * xl1 + ((trk - trf) * yl1 + (brk - brf) * yl) * xl;
                        tg = gr[c];
                    }
                    const GbTerm ty_ = gb_term(ch, y, igy * tg, hr, H);
                    const GbTerm tx_ = gb_term(cw, x, igx * tg, wr, W);
                    const GbTerm tz_ = gb_term(cd, z, igz * tg, dr, D);
                    const int cnt = C - c0 < 64 ? C - c0 : 64;
                    for (int l = 0; l < cnt; ++l) {       // channel order, one term at a time
                        gb_acc(ch, ty_, l, a0, a3);
                        gb_acc(cw, tx_, l, a1, a4);
                        gb_acc(cd, tz_, l, a2, a5);
                    }
                }
            }
        }
    }
    if (lane == 0) {
        float* o = gboxes + (size_t)n * 6;
        o[0] = a0; o[1] = a1; o[2] = a2; o[3] = a3; o[4] = a4; o[5] = a5;
    }
}

// ---- PyramidROIAlign ----------------------------------------------------------

// Box preparation + level assignment (core/models.py:611-649), one thread per (b,n).
__global__ void pyramid_prep_kernel(const float* __restrict__ boxes,
                                    const float* __restrict__ meta, int64_t meta_stride,
                                    int64_t B, int64_t N, float* __restrict__ boxes_adj,
                                    int32_t* __restrict__ levels) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B * N) return;
    const int64_t b = i / N;
    const float* bx = boxes + i * 6;
    float v[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) v[q] = smax(smin(bx[q], 1.0f), 0.0f);   // tf.clip_by_value
    const float eps = 1e-6f;
    v[3] = smax(v[3], v[0] + eps);
    v[4] = smax(v[4], v[1] + eps);
    const float* m = meta + b * meta_stride;
    const float H = m[5], W = m[6], D = m[7];
    const float min_dz = 1.0f / smax(D, 1.0f);
    v[5] = smax(v[5], v[2] + min_dz);
#pragma unroll
    for (int q = 0; q < 6; ++q) boxes_adj[i * 6 + q] = v[q];
    const float h = v[3] - v[0], w = v[4] - v[1], d = v[5] - v[2];
    const float image_area = (H * W) * D;
    const float vol = (h * w) * d;
    const float third = 0.333333343267440796f;          // (float)(1.0/3.0)
    const float r = powf(vol, third) / (224.0f / powf(image_area, third));
    const float ln2 = 0.693147182464599609375f;         // logf(2.0f)
    const float lvl = rintf(logf(r) / ln2);              // tf.round: half to even
    int li;
    if (!isfinite(lvl)) li = 2;                          // (int)NaN/inf -> INT_MIN -> clamp 2
    else {
        int64_t l64 = 4 + (int64_t)lvl;
        li = (int)(l64 < 2 ? 2 : (l64 > 5 ? 5 : l64));
    }
    levels[i] = li;
}

__global__ __launch_bounds__(256) void pyramid_fwd_kernel(Pyr P, int C,
                                                          const float* __restrict__ boxes_adj,
                                                          const int32_t* __restrict__ levels,
                                                          int64_t N, int64_t total, int ph,
                                                          int pw, int pd,
                                                          float* __restrict__ out) {
    const int64_t sidx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sidx >= total) return;
    int64_t t = sidx;
    const int z = (int)(t % pd); t /= pd;
    const int x = (int)(t % pw); t /= pw;
    const int y = (int)(t % ph);
    const int64_t bn = t / ph;
    const int64_t b = bn / N;
    const int l = levels[bn] - 2;
    const int H = P.H[l], W = P.W[l], D = P.D[l];
    const Sample s = make_sample(boxes_adj + bn * 6, H, W, D, ph, pw, pd, y, x, z);
    const float* img = P.fmaps[l] + (size_t)b * H * W * D * C;
    emit_sample<true>(img, W, D, C, s, 0, 0.0f, out + sidx * C, lane);
}

__global__ __launch_bounds__(256) void pyramid_bwd_kernel(Pyr P, int C,
                                                          const float* __restrict__ boxes_adj,
                                                          const int32_t* __restrict__ levels,
                                                          int64_t N, int64_t total, int ph,
                                                          int pw, int pd,
                                                          const float* __restrict__ gout) {
    const int64_t sidx = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (sidx >= total) return;
    int64_t t = sidx;
    const int z = (int)(t % pd); t /= pd;
    const int x = (int)(t % pw); t /= pw;
    const int y = (int)(t % ph);
    const int64_t bn = t / ph;
    const int64_t b = bn / N;
    const int l = levels[bn] - 2;
    const int H = P.H[l], W = P.W[l], D = P.D[l];
    const Sample s = make_sample(boxes_adj + bn * 6, H, W, D, ph, pw, pd, y, x, z);
    float* img = P.gmaps[l] + (size_t)b * H * W * D * C;
    scatter_sample(img, W, D, C, s, 0, gout + sidx * C, lane);
}


// DetectionTargetLayer GT-mask targets (core/models.py:972-996): for each
// positive ROI p, crop channel assign[p] of the boolean instance masks
// [H,W,D,G] (read in place -- the reference materialises a [P,H,W,D,1]
// gather first) to (mh,mw,md) with trilinear CropAndResize3D semantics
// (A.1), then tf.round (half to even).  One thread per output voxel.
__global__ void mask_targets_kernel(const uint8_t* __restrict__ masks, int H, int W, int D, int G,
                                    const float* __restrict__ boxes,
                                    const int32_t* __restrict__ assign, int64_t total, int mh,
                                    int mw, int md, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int64_t t = i;
    const int z = (int)(t % md); t /= md;
    const int x = (int)(t % mw); t /= mw;
    const int y = (int)(t % mh);
    const int64_t p = t / mh;
    const int g = assign[p];
    if (g < 0) {      // not a positive ROI (DetectionTargetLayer padding rows)
        out[i] = 0.0f;
        return;
    }
    const Sample s = make_sample(boxes + p * 6, H, W, D, mh, mw, md, y, x, z);
    float v = 0.0f;   // extrapolation_value 0
    if (!s.oob) {
        auto M = [&](int yy, int xx, int zz) {
            return (float)masks[(((int64_t)yy * W + xx) * D + zz) * G + g];
        };
        v = tri(M(s.ty, s.lx, s.fz), M(s.ty, s.lx, s.kz), M(s.ty, s.rx, s.fz), M(s.ty, s.rx, s.kz),
                M(s.by, s.lx, s.fz), M(s.by, s.lx, s.kz), M(s.by, s.rx, s.fz), M(s.by, s.rx, s.kz),
                s.yl, s.xl, s.zl);
    }
    out[i] = rintf(v);
}

}  // namespace m3d

using namespace m3d;

static int check_crop_args(int64_t B, int64_t H, int64_t W, int64_t D, int64_t C, int32_t ch,
                           int32_t cw, int32_t cd, int32_t method) {
    if (B < 0 || H <= 0 || W <= 0 || D <= 0 || C <= 0)
        return einval("image dimensions must be positive");
    if (ch <= 0 || cw <= 0 || cd <= 0) return einval("crop dimensions must be positive");
    if (method != 0 && method != 1) return einval("method must be 'trilinear' or 'nearest'");
    return M3D_OK;
}

extern "C" int m3d_crop_and_resize3d_fwd(const float* image, int64_t B, int64_t H, int64_t W,
                                         int64_t D, int64_t C, const float* boxes,
                                         const int32_t* box_ind, int64_t N, int32_t ch,
                                         int32_t cw, int32_t cd, int32_t method,
                                         float extrapolation, float* crops, m3d_stream_t s) {
    int rc = check_crop_args(B, H, W, D, C, ch, cw, cd, method);
    if (rc) return rc;
    const int64_t total = N * ch * cw * cd;
    if (total == 0) return M3D_OK;
    if (method == 0 && (C & 3) == 0) {
        LineArgs a{image, box_ind, boxes, nullptr, 0, N * ch * cw, (int)H, (int)W, (int)D, (int)C,
                   ch, cw, cd, extrapolation, crops};
        hipLaunchKernelGGL(line_fwd_kernel<false>, dim3(grid_for(a.lines, 4)), dim3(256), 0, st(s), a,
                           Pyr{});
        return check_launch("line_fwd_kernel");
    }
    hipLaunchKernelGGL(crop_fwd_kernel, dim3(grid_for(total, 4)), dim3(256), 0, st(s), image,
                       (int)B, (int)H, (int)W, (int)D, (int)C, boxes, box_ind, total, ch, cw, cd,
                       method, extrapolation, crops);
    return check_launch("crop_fwd_kernel");
}

extern "C" int m3d_crop_and_resize3d_bwd_image(const float* grads, const float* boxes,
                                               const int32_t* box_ind, int64_t N, int32_t ch,
                                               int32_t cw, int32_t cd, int64_t B, int64_t H,
                                               int64_t W, int64_t D, int64_t C, int32_t method,
                                               int32_t deterministic, float* grad_image,
                                               m3d_stream_t s) {
    int rc = check_crop_args(B, H, W, D, C, ch, cw, cd, method);
    if (rc) return rc;
    if (deterministic < 0 || deterministic > 2) return einval("deterministic must be 0, 1 or 2");
    const int64_t total = N * ch * cw * cd;
    if (deterministic == 1 && B > 0 && ch <= 64 && cw <= 64 && cd <= 64) {
        // destination-owned sums in the replay order: writes every voxel (no zero fill)
        launch_det_bwd(grads, boxes, box_ind, N, ch, cw, cd, B, H, W, D, C, method, grad_image, st(s));
        return check_launch("crop_bwd_det_kernel");
    }
    if (hipMemsetAsync(grad_image, 0, sizeof(float) * (size_t)(B * H * W * D * C), st(s)) !=
        hipSuccess)
        return check_launch("memset grad_image");
    if (total == 0 || B == 0) return M3D_OK;
    if (deterministic) {
        hipLaunchKernelGGL(crop_bwd_serial_kernel, dim3(grid_for(B * C, 256)), dim3(256), 0,
                           st(s), grads, boxes, box_ind, N, ch, cw, cd, (int)B, (int)H, (int)W,
                           (int)D, (int)C, method, grad_image);
        return check_launch("crop_bwd_serial_kernel");
    }
    if (method == 0 && gather_bwd_ok(C, ch, cw, cd)) {
        GatherArgs a{grads, boxes, box_ind, nullptr, grad_image, N, 0, (int)H, (int)W, (int)D, ch, cw, cd};
        launch_gather_bwd<false>(a, Pyr{}, C, st(s));
        return check_launch("gather_bwd_kernel");
    }
    hipLaunchKernelGGL(crop_bwd_atomic_kernel, dim3(grid_for(total, 4)), dim3(256), 0, st(s),
                       grads, boxes, box_ind, total, ch, cw, cd, (int)H, (int)W, (int)D, (int)C,
                       method, grad_image);
    return check_launch("crop_bwd_atomic_kernel");
}

extern "C" int m3d_crop_and_resize3d_bwd_boxes(const float* grads, const float* image, int64_t B,
                                               int64_t H, int64_t W, int64_t D, int64_t C,
                                               const float* boxes, const int32_t* box_ind,
                                               int64_t N, int32_t ch, int32_t cw, int32_t cd,
                                               float* grad_boxes, m3d_stream_t s) {
    int rc = check_crop_args(B, H, W, D, C, ch, cw, cd, 0);
    if (rc) return rc;
    if (N == 0) return M3D_OK;
    hipLaunchKernelGGL(crop_bwd_boxes_kernel, dim3((unsigned)N), dim3(64), 0, st(s), grads,
                       image, (int)B, (int)H, (int)W, (int)D, (int)C, boxes, box_ind, ch, cw, cd,
                       grad_boxes);
    return check_launch("crop_bwd_boxes_kernel");
}

static int make_pyr(Pyr& P, const float* const fmaps[4], float* const gmaps[4],
                    const int64_t fshape[4][3]) {
    for (int l = 0; l < 4; ++l) {
        P.fmaps[l] = fmaps ? fmaps[l] : nullptr;
        P.gmaps[l] = gmaps ? gmaps[l] : nullptr;
        P.H[l] = (int)fshape[l][0];
        P.W[l] = (int)fshape[l][1];
        P.D[l] = (int)fshape[l][2];
        if (P.H[l] <= 0 || P.W[l] <= 0 || P.D[l] <= 0)
            return einval("feature map dimensions must be positive");
    }
    return M3D_OK;
}

// workspace of the spatially sorted line order (m3d_pyramid_roi_align3d_fwd_ws)
static size_t pyr_sort_layout(const int64_t fshape[4][3], int64_t B, int64_t N, int32_t ph, int32_t pw,
                              int64_t* nbuckets, int64_t* lines) {
    int64_t nb = 0;
    for (int l = 0; l < 4; ++l) nb += B * fshape[l][0] * fshape[l][1];
    const int64_t nl = B * N * ph * pw;
    if (nbuckets) *nbuckets = nb;
    if (lines) *lines = nl;
    return sizeof(int32_t) * (size_t)(2 * nb + 2 * nl) + 256;
}

extern "C" size_t m3d_pyramid_roi_align3d_fwd_workspace_bytes(const int64_t fshape[4][3], int64_t B, int64_t N,
                                                              int32_t ph, int32_t pw) {
    return pyr_sort_layout(fshape, B, N, ph, pw, nullptr, nullptr);
}

static int pyramid_fwd_impl(const float* const fmaps[4], const int64_t fshape[4][3], int64_t C,
                            const float* boxes, const float* image_meta, int64_t meta_stride, int64_t B,
                            int64_t N, int32_t ph, int32_t pw, int32_t pd, float* out, float* boxes_adj,
                            int32_t* levels, void* workspace, size_t ws_bytes, hipStream_t s) {
    Pyr P{};
    int rc = make_pyr(P, fmaps, nullptr, fshape);
    if (rc) return rc;
    if (ph <= 0 || pw <= 0 || pd <= 0) return einval("crop dimensions must be positive");
    if (meta_stride < 8) return einval("image_meta must have at least 8 columns");
    if (B * N == 0) return M3D_OK;
    hipLaunchKernelGGL(pyramid_prep_kernel, dim3(grid_for(B * N, 256)), dim3(256), 0, s,
                       boxes, image_meta, meta_stride, B, N, boxes_adj, levels);
    rc = check_launch("pyramid_prep_kernel");
    if (rc) return rc;
    const int64_t total = B * N * ph * pw * pd;
    if ((C & 3) == 0) {
        LineArgs a{nullptr, nullptr, boxes_adj, levels, N, B * N * ph * pw, 0, 0, 0, (int)C, ph, pw, pd,
                   0.0f, out};
        const int sl = roi_slices();
        if (C == 256 && (sl == 2 || sl == 4 || sl == 8 || sl == 16)) {
            const int32_t* perm = nullptr;
            const int32_t* wperm = nullptr;
            int64_t nb = 0, nl = 0;
            const size_t need = pyr_sort_layout(fshape, B, N, ph, pw, &nb, &nl);
            // waves sorted by their feature-map column for the 14^3 mask pool -- PMC
            // fabric reads at 256^3 / 512 ROIs 3.41 -> 1.89 GB, 128^3 / 128 ROIs 0.167
            // -> 0.140 ms -- and for the 7^3 pool once the launch is large (512 ROIs at
            // 256^3: PMC traffic 1.34 -> 1.09 GB); launch order for small 7^3 launches
            // (their lines are short: at 128^3 the sort costs 4 us of 58)
            const bool wave_sort = pd >= 14 || a.lines >= 16384;
            if (wave_sort && workspace && ws_bytes >= need && nb < INT32_MAX && nl < INT32_MAX) {
                const int64_t nw = (nl + sl - 1) / sl;
                int32_t* counts = (int32_t*)workspace;
                int32_t* offs = counts + nb;
                int32_t* keys = offs + nb;
                int32_t* pm = keys + nl;
                RegionBase rb{};
                int64_t acc = 0;
                for (int l = 0; l < 4; ++l) {
                    rb.base[l] = acc;
                    acc += B * fshape[l][0] * fshape[l][1];
                }
                if (hipMemsetAsync(counts, 0, sizeof(int32_t) * (size_t)nb, s) != hipSuccess)
                    return check_launch("memset wave buckets");
                hipLaunchKernelGGL(wave_key_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, s, a, P, rb, sl, nw,
                                   keys, counts);
                hipLaunchKernelGGL(excl_scan_kernel, dim3(1), dim3(1024), 0, s, counts, nb, offs);
                hipLaunchKernelGGL(line_scatter_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, s, keys, nw, offs, pm);
                rc = check_launch("wave sort");
                if (rc) return rc;
                wperm = pm;
            }
            const int zs = 1;
            const int64_t bs8 = (((a.lines * zs + sl - 1) / sl + 3) / 4 + 7) / 8 * 8;
            const unsigned grid = (unsigned)(bs8 * sl);
            if constexpr (M3D_TUNE_ROI_SLICES == 2)
                hipLaunchKernelGGL(line_fwd_sl_kernel<2>, dim3(grid), dim3(256), 0, s, a, P, perm, zs, wperm);
            else if constexpr (M3D_TUNE_ROI_SLICES == 4)
                hipLaunchKernelGGL(line_fwd_sl_kernel<4>, dim3(grid), dim3(256), 0, s, a, P, perm, zs, wperm);
            else if constexpr (M3D_TUNE_ROI_SLICES == 16)
                hipLaunchKernelGGL(line_fwd_sl_kernel<16>, dim3(grid), dim3(256), 0, s, a, P, perm, zs, wperm);
            else
                hipLaunchKernelGGL(line_fwd_sl_kernel<8>, dim3(grid), dim3(256), 0, s, a, P, perm, zs, wperm);
            return check_launch("line_fwd_sl_kernel");
        }
        hipLaunchKernelGGL(line_fwd_kernel<true>, dim3(grid_for(a.lines, 4)), dim3(256), 0, s, a, P);
        return check_launch("line_fwd_kernel");
    }
    hipLaunchKernelGGL(pyramid_fwd_kernel, dim3(grid_for(total, 4)), dim3(256), 0, s, P,
                       (int)C, boxes_adj, levels, N, total, ph, pw, pd, out);
    return check_launch("pyramid_fwd_kernel");
}

extern "C" int m3d_pyramid_roi_align3d_fwd(const float* const fmaps[4],
                                           const int64_t fshape[4][3], int64_t C,
                                           const float* boxes, const float* image_meta,
                                           int64_t meta_stride, int64_t B, int64_t N, int32_t ph,
                                           int32_t pw, int32_t pd, float* out, float* boxes_adj,
                                           int32_t* levels, m3d_stream_t s) {
    return pyramid_fwd_impl(fmaps, fshape, C, boxes, image_meta, meta_stride, B, N, ph, pw, pd, out,
                            boxes_adj, levels, nullptr, 0, st(s));
}

extern "C" int m3d_pyramid_roi_align3d_fwd_ws(const float* const fmaps[4], const int64_t fshape[4][3],
                                              int64_t C, const float* boxes, const float* image_meta,
                                              int64_t meta_stride, int64_t B, int64_t N, int32_t ph,
                                              int32_t pw, int32_t pd, float* out, float* boxes_adj,
                                              int32_t* levels, void* workspace, size_t ws_bytes,
                                              m3d_stream_t s) {
    return pyramid_fwd_impl(fmaps, fshape, C, boxes, image_meta, meta_stride, B, N, ph, pw, pd, out,
                            boxes_adj, levels, workspace, ws_bytes, st(s));
}

extern "C" int m3d_pyramid_roi_align3d_bwd(const float* grad_out, const float* boxes_adj,
                                           const int32_t* levels, int64_t B, int64_t N,
                                           int32_t ph, int32_t pw, int32_t pd,
                                           float* const gmaps[4], const int64_t fshape[4][3],
                                           int64_t C, m3d_stream_t s) {
    Pyr P{};
    int rc = make_pyr(P, nullptr, gmaps, fshape);
    if (rc) return rc;
    if (ph <= 0 || pw <= 0 || pd <= 0) return einval("crop dimensions must be positive");
    if (B < 0 || N < 0 || C <= 0) return einval("pyramid_roi_align3d_bwd: invalid B, N or C");
    for (int l = 0; l < 4; ++l)
        if (hipMemsetAsync(gmaps[l], 0,
                           sizeof(float) * (size_t)(B * P.H[l] * P.W[l] * P.D[l] * C),
                           st(s)) != hipSuccess)
            return check_launch("memset gmaps");
    const int64_t total = B * N * ph * pw * pd;
    if (total == 0) return M3D_OK;
    if (gather_bwd_ok(C, ph, pw, pd)) {
        GatherArgs a{grad_out, boxes_adj, nullptr, levels, nullptr, B * N, N, 0, 0, 0, ph, pw, pd};
        launch_gather_bwd<true>(a, P, C, st(s));
        return check_launch("gather_bwd_kernel<pyr>");
    }
    hipLaunchKernelGGL(pyramid_bwd_kernel, dim3(grid_for(total, 4)), dim3(256), 0, st(s), P,
                       (int)C, boxes_adj, levels, N, total, ph, pw, pd, grad_out);
    return check_launch("pyramid_bwd_kernel");
}

// Deterministic PyramidROIAlign backward (the gradient of core/models.py:597-687
// through custom_op.py:28-65): per level, CropAndResize3DGradImage over that
// level's ROIs in ascending order -- the reference's tf.where gather order --
// as crop_bwd_det_kernel (destination-owned sums in the sequential replay
// order, bit-identical to it; every voxel written, no zero fill).  box_ind_ws:
// [4][B*N] int32 device scratch; ROIs of other levels get -1 (never match).
__global__ void pyr_level_bi_kernel(const int32_t* __restrict__ levels, int64_t BN, int64_t N,
                                    int32_t* __restrict__ bi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= BN) return;
    const int l = levels[i] - 2;
    for (int k = 0; k < 4; ++k) bi[k * BN + i] = l == k ? (int32_t)(i / N) : -1;
}

extern "C" int m3d_pyramid_roi_align3d_bwd_det(const float* grad_out, const float* boxes_adj,
                                               const int32_t* levels, int64_t B, int64_t N,
                                               int32_t ph, int32_t pw, int32_t pd,
                                               float* const gmaps[4], const int64_t fshape[4][3],
                                               int64_t C, int32_t* box_ind_ws, m3d_stream_t s) {
    Pyr P{};
    int rc = make_pyr(P, nullptr, gmaps, fshape);
    if (rc) return rc;
    if (ph <= 0 || pw <= 0 || pd <= 0) return einval("crop dimensions must be positive");
    if (ph > 64 || pw > 64 || pd > 64) return einval("pyramid_roi_align3d_bwd_det: crop sizes up to 64");
    if (B < 0 || N < 0 || C <= 0) return einval("pyramid_roi_align3d_bwd: invalid B, N or C");
    if (B * N > 0 && !box_ind_ws) return einval("pyramid_roi_align3d_bwd_det: box_ind workspace missing");
    const int64_t BN = B * N;
    if (BN > 0) hipLaunchKernelGGL(pyr_level_bi_kernel, dim3(grid_for(BN, 256)), dim3(256), 0, st(s), levels, BN,
                                   N, box_ind_ws);
    for (int l = 0; l < 4; ++l) {
        const int64_t H = P.H[l], W = P.W[l], D = P.D[l];
        if (BN == 0) {
            if (hipMemsetAsync(gmaps[l], 0, sizeof(float) * (size_t)(B * H * W * D * C), st(s)) != hipSuccess)
                return check_launch("memset gmaps");
            continue;
        }
        launch_det_bwd(grad_out, boxes_adj, box_ind_ws + l * BN, BN, ph, pw, pd, B, H, W, D, C, 0, gmaps[l],
                       st(s));
    }
    return check_launch("crop_bwd_det_kernel<pyr>");
}

extern "C" int m3d_mask_targets3d(const uint8_t* gt_masks, int64_t H, int64_t W, int64_t D,
                                  int64_t G, const float* rois, const int32_t* assign, int64_t P,
                                  int32_t mh, int32_t mw, int32_t md, float* out, m3d_stream_t s) {
    if (H <= 0 || W <= 0 || D <= 0 || G < 0) return einval("gt_masks must be [H,W,D,G]");
    if (mh <= 0 || mw <= 0 || md <= 0) return einval("crop dimensions must be positive");
    const int64_t total = P * mh * mw * md;
    if (total == 0) return M3D_OK;
    if (G == 0) return einval("no GT masks to crop");
    hipLaunchKernelGGL(mask_targets_kernel, dim3(grid_for(total, 256)), dim3(256), 0, st(s), gt_masks,
                       (int)H, (int)W, (int)D, (int)G, rois, assign, total, mh, mw, md, out);
    return check_launch("mask_targets_kernel");
}
