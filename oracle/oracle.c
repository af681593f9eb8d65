/*
 * oracle.c -- CPU restatement of the reference's native 3-D ops.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library, and only as the checker / the timed CPU baseline.
 *
 * PARITY STATUS: "parity unpinned".  The reference ops live in the vendored
 * binary wheel tensorflow_nms_car_3d==0.1.0
 * (core/custom_op/tensorflow_nms_car_3d-0.1.0-cp36-cp36m-linux_x86_64.whl),
 * whose source is absent and which may not be executed here.
 * The reference ships no tests, fixtures or golden vectors for this path
 * (SURVEY.md 4).  This file restates the op semantics recovered by static
 * disassembly in the TF-2.2 CPU kernel structure they
 * generalise, and is pinned only by hand-derived known-answer tests
 * (tests/test_oracle.py).
 *
 * Compiled with -O2 -ffp-contract=off so every float op rounds exactly as
 * written (no FMA contraction), mirroring the SSE scalar code of the wheel.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

/* std::min / std::max semantics (NaN propagation identical to TF). */
#define SMIN(a, b) (((b) < (a)) ? (b) : (a))
#define SMAX(a, b) (((a) < (b)) ? (b) : (a))

/* ------------------------------------------------------------------------ */
/* CropAndResize3D forward  (whl _crop_and_resize_3d_ops.so     */
/* CropAndResize3DOp::Compute @0x4370).  Loop order box -> y -> x -> z -> c. */
/* method 0 = trilinear, 1 = nearest.  Returns 0, or -1 on a bad box_ind.    */
/* ------------------------------------------------------------------------ */
static inline float axis_scale(float b1, float b2, int S, int n) {
    /* @0x499a-0x4a62: ((b2-b1)*(float)(S-1)) / (float)(n-1) in f32 */
    return n > 1 ? ((b2 - b1) * (float)(S - 1)) / (float)(n - 1) : 0.0f;
}
static inline float axis_coord(float b1, float b2, int S, int n, int i, float sc) {
    if (n > 1) return b1 * (float)(S - 1) + (float)i * sc;            /* @0x4abd */
    return (float)(0.5 * (double)(b1 + b2) * (double)(S - 1));        /* @0x5287 */
}

int oracle_crop_and_resize3d(const float* image, int B, int H, int W, int D, int C,
                             const float* boxes, const int32_t* box_ind, int N,
                             int ch, int cw, int cd, int method, float extrap,
                             float* crops) {
    for (int n = 0; n < N; ++n)
        if (box_ind[n] < 0 || box_ind[n] >= B) return -1;
    for (int n = 0; n < N; ++n) {
        const float y1 = boxes[n * 6 + 0], x1 = boxes[n * 6 + 1], z1 = boxes[n * 6 + 2];
        const float y2 = boxes[n * 6 + 3], x2 = boxes[n * 6 + 4], z2 = boxes[n * 6 + 5];
        const int b = box_ind[n];
        const float hs = axis_scale(y1, y2, H, ch);
        const float ws = axis_scale(x1, x2, W, cw);
        const float ds = axis_scale(z1, z2, D, cd);
        const float* img = image + (size_t)b * H * W * D * C;
        for (int y = 0; y < ch; ++y) {
            const float in_y = axis_coord(y1, y2, H, ch, y, hs);
            float* orow = crops + ((((size_t)n * ch + y) * cw) * cd) * C;
            if (in_y < 0 || in_y > (float)(H - 1)) {
                for (size_t i = 0; i < (size_t)cw * cd * C; ++i) orow[i] = extrap;
                continue;
            }
            const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
            const float yl = in_y - (float)ty;
            for (int x = 0; x < cw; ++x) {
                const float in_x = axis_coord(x1, x2, W, cw, x, ws);
                float* ocol = orow + (size_t)x * cd * C;
                if (in_x < 0 || in_x > (float)(W - 1)) {
                    for (size_t i = 0; i < (size_t)cd * C; ++i) ocol[i] = extrap;
                    continue;
                }
                const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
                const float xl = in_x - (float)lx;
                for (int z = 0; z < cd; ++z) {
                    const float in_z = axis_coord(z1, z2, D, cd, z, ds);
                    float* o = ocol + (size_t)z * C;
                    if (in_z < 0 || in_z > (float)(D - 1)) {
                        for (int c = 0; c < C; ++c) o[c] = extrap;
                        continue;
                    }
                    if (method == 1) {  /* nearest: roundf (half away from zero) @0x54c2 */
                        const int cy = (int)roundf(in_y), cx = (int)roundf(in_x), cz = (int)roundf(in_z);
                        const float* v = img + (((size_t)cy * W + cx) * D + cz) * C;
                        for (int c = 0; c < C; ++c) o[c] = v[c];
                        continue;
                    }
                    const int fz = (int)floorf(in_z), kz = (int)ceilf(in_z);
                    const float zl = in_z - (float)fz;
#define V(yy, xx, zz) (img + (((size_t)(yy) * W + (xx)) * D + (zz)) * C)
                    const float *tlf = V(ty, lx, fz), *tlk = V(ty, lx, kz);
                    const float *trf = V(ty, rx, fz), *trk = V(ty, rx, kz);
                    const float *blf = V(by, lx, fz), *blk = V(by, lx, kz);
                    const float *brf = V(by, rx, fz), *brk = V(by, rx, kz);
#undef V
                    for (int c = 0; c < C; ++c) {   /* lerp order @0x4f88-0x5011 */
                        const float tl = tlf[c] + (tlk[c] - tlf[c]) * zl;
                        const float bl = blf[c] + (blk[c] - blf[c]) * zl;
                        const float tr = trf[c] + (trk[c] - trf[c]) * zl;
                        const float br = brf[c] + (brk[c] - brf[c]) * zl;
                        const float top = tl + (tr - tl) * xl;
                        const float bot = bl + (br - bl) * xl;
                        o[c] = top + (bot - top) * yl;
                    }
                }
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CropAndResize3DGradImage (Compute @0x3a80).  Zero-fill, then  */
/* sequential scatter of g*w_k into the 8 corners, box->y->x->z->c order.    */
/* ------------------------------------------------------------------------ */
int oracle_crop_and_resize3d_grad_image(const float* grads, const float* boxes,
                                        const int32_t* box_ind, int N, int ch, int cw, int cd,
                                        int B, int H, int W, int D, int C, int method,
                                        float* out) {
    for (int n = 0; n < N; ++n)
        if (box_ind[n] < 0 || box_ind[n] >= B) return -1;
    memset(out, 0, sizeof(float) * (size_t)B * H * W * D * C);
    for (int n = 0; n < N; ++n) {
        const float y1 = boxes[n * 6 + 0], x1 = boxes[n * 6 + 1], z1 = boxes[n * 6 + 2];
        const float y2 = boxes[n * 6 + 3], x2 = boxes[n * 6 + 4], z2 = boxes[n * 6 + 5];
        float* img = out + (size_t)box_ind[n] * H * W * D * C;
        const float hs = axis_scale(y1, y2, H, ch);
        const float ws = axis_scale(x1, x2, W, cw);
        const float ds = axis_scale(z1, z2, D, cd);
        for (int y = 0; y < ch; ++y) {
            const float in_y = axis_coord(y1, y2, H, ch, y, hs);
            if (in_y < 0 || in_y > (float)(H - 1)) continue;
            const int ty = (int)floorf(in_y), by = (int)ceilf(in_y);
            const float yl = in_y - (float)ty;
            for (int x = 0; x < cw; ++x) {
                const float in_x = axis_coord(x1, x2, W, cw, x, ws);
                if (in_x < 0 || in_x > (float)(W - 1)) continue;
                const int lx = (int)floorf(in_x), rx = (int)ceilf(in_x);
                const float xl = in_x - (float)lx;
                for (int z = 0; z < cd; ++z) {
                    const float in_z = axis_coord(z1, z2, D, cd, z, ds);
                    if (in_z < 0 || in_z > (float)(D - 1)) continue;
                    const float* g = grads + ((((size_t)n * ch + y) * cw + x) * cd + z) * C;
                    if (method == 1) {
                        const int cy = (int)roundf(in_y), cx = (int)roundf(in_x), cz = (int)roundf(in_z);
                        float* v = img + (((size_t)cy * W + cx) * D + cz) * C;
                        for (int c = 0; c < C; ++c) v[c] += g[c];
                        continue;
                    }
                    const int fz = (int)floorf(in_z), kz = (int)ceilf(in_z);
                    const float zl = in_z - (float)fz;
                    /* per-sample corner weights, computed once (@0x4628-0x470c) */
                    const float wy[2] = {1.0f - yl, yl}, wx[2] = {1.0f - xl, xl}, wz[2] = {1.0f - zl, zl};
                    const int iy[2] = {ty, by}, ix[2] = {lx, rx}, iz[2] = {fz, kz};
                    float w[8];
                    float* dst[8];
                    for (int a = 0; a < 2; ++a)
                        for (int bb = 0; bb < 2; ++bb)
                            for (int cc = 0; cc < 2; ++cc) {
                                const int k = a * 4 + bb * 2 + cc;
                                w[k] = (wy[a] * wx[bb]) * wz[cc];
                                dst[k] = img + (((size_t)iy[a] * W + ix[bb]) * D + iz[cc]) * C;
                            }
                    for (int c = 0; c < C; ++c)
                        for (int k = 0; k < 8; ++k) dst[k][c] += g[c] * w[k];
                }
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* CropAndResize3DGradBoxes, out[n] = (dy1, dx1, dz1, dy2, dx2, dz2),         */
/* restated from the wheel's compiled code (SURVEY.md
 * style appendix A.4 in DESIGN.md; whl _crop_and_resize_3d_grad_boxes_ops.so,
 * CropAndResize3DGradBoxesOp::Compute @0x3980):
 *  - ratios r = (S-1)/(n-1) per axis (0 when n == 1), @0x3f4a-0x3fdb;
 *  - scales hs = (y2-y1)*rh, ws = (x2-x1)*rw and, as compiled, the DEPTH
 *    scale ds = (z2 - y1)*rh (y1 and the height ratio, @0x4059-0x4071);
 *  - loops box -> y -> x -> z -> c, a sample out of bounds on an axis is
 *    skipped (@0x40f4, 0x4250, 0x43c2); in = b1*(S-1) + i*scale, or
 *    (float)((double)(b1+b2)*0.5*(double)(S-1)) when n == 1 (@0x4a50...);
 *  - image gradients per channel in the compiled association (@0x46a4-0x47c6):
 *      igy = ((blf-tlf)(1-xl) + (brf-trf)xl)(1-zl) + ((blk-tlk)(1-xl) + (brk-trk)xl)zl
 *      igx = ((trf-tlf)(1-yl) + (brf-blf)yl)(1-zl) + ((trk-tlk)(1-yl) + (brk-blk)yl)zl
 *      igz = ((tlk-tlf)(1-yl) + (blk-blf)yl)(1-xl) + ((trk-trf)(1-yl) + (brk-brf)yl)xl
 *    times the incoming gradient;
 *  - accumulation into the zero-filled float output, sequentially
 *    (@0x4590-0x469e): out[a] += ((S-1) - r*i) * g_a and out[a+3] += (g_a*i)*r
 *    for n > 1; for n == 1 both get (float)((double)out + (double)g_a*0.5*(double)(S-1))
 *    (@0x47d0-0x48e3).
 * Not reachable from the reference graph. */
static void gb_add(float* o, int n, int i, float g, float r, int S) {
    if (n > 1) {
        o[0] += ((float)(S - 1) - r * (float)i) * g;
        o[3] += (g * (float)i) * r;
    } else {
        const double d = (double)g * 0.5 * (double)(S - 1);
        o[0] = (float)((double)o[0] + d);
        o[3] = (float)(d + (double)o[3]);
    }
}

int oracle_crop_and_resize3d_grad_boxes(const float* grads, const float* image,
                                        int B, int H, int W, int D, int C,
                                        const float* boxes, const int32_t* box_ind, int N,
                                        int ch, int cw, int cd, float* out) {
    for (int n = 0; n < N; ++n)
        if (box_ind[n] < 0 || box_ind[n] >= B) return -1;
    memset(out, 0, sizeof(float) * (size_t)N * 6);
    for (int n = 0; n < N; ++n) {
        const float y1 = boxes[n * 6 + 0], x1 = boxes[n * 6 + 1], z1 = boxes[n * 6 + 2];
        const float y2 = boxes[n * 6 + 3], x2 = boxes[n * 6 + 4], z2 = boxes[n * 6 + 5];
        const float* img = image + (size_t)box_ind[n] * H * W * D * C;
        const float hr = ch > 1 ? (float)(H - 1) / (float)(ch - 1) : 0.0f;
        const float wr = cw > 1 ? (float)(W - 1) / (float)(cw - 1) : 0.0f;
        const float dr = cd > 1 ? (float)(D - 1) / (float)(cd - 1) : 0.0f;
        const float hs = ch > 1 ? (y2 - y1) * hr : 0.0f;
        const float ws = cw > 1 ? (x2 - x1) * wr : 0.0f;
        const float ds = cd > 1 ? (z2 - y1) * hr : 0.0f;      /* sic: the compiled depth scale */
        float* gb = out + (size_t)n * 6;
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
                    const float* g = grads + ((((size_t)n * ch + y) * cw + x) * cd + z) * C;
#define V(yy, xx, zz) (img + (((size_t)(yy) * W + (xx)) * D + (zz)) * C)
                    const float *ptlf = V(ty, lx, fz), *ptlk = V(ty, lx, kz);
                    const float *ptrf = V(ty, rx, fz), *ptrk = V(ty, rx, kz);
                    const float *pblf = V(by, lx, fz), *pblk = V(by, lx, kz);
                    const float *pbrf = V(by, rx, fz), *pbrk = V(by, rx, kz);
#undef V
                    for (int c = 0; c < C; ++c) {
                        const float tlf = ptlf[c], tlk = ptlk[c], trf = ptrf[c], trk = ptrk[c];
                        const float blf = pblf[c], blk = pblk[c], brf = pbrf[c], brk = pbrk[c];
                        const float igy = ((blf - tlf) * xl1 + (brf - trf) * xl) * zl1 +
                                          ((blk - tlk) * xl1 + (brk - trk) * xl) * zl;
                        const float igx = ((trf - tlf) * yl1 + (brf - blf) * yl) * zl1 +
                                          ((trk - tlk) * yl1 + (brk - blk) * yl) * zl;
                        const float igz = ((tlk - tlf) * yl1 + (blk - blf) * yl) * xl1 +
                                          ((trk - trf) * yl1 + (brk - brf) * yl) * xl;
                        const float tg = g[c];
                        float o[4];
                        o[0] = gb[0]; o[3] = gb[3];
                        gb_add(o, ch, y, igy * tg, hr, H);
                        gb[0] = o[0]; gb[3] = o[3];
                        o[0] = gb[1]; o[3] = gb[4];
                        gb_add(o, cw, x, igx * tg, wr, W);
                        gb[1] = o[0]; gb[4] = o[3];
                        o[0] = gb[2]; o[3] = gb[5];
                        gb_add(o, cd, z, igz * tg, dr, D);
                        gb[2] = o[0]; gb[5] = o[3];
                    }
                }
            }
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* IOU<float> 3-D  (whl _non_max_suppression_3d_ops.so @0xb500) */
/* mode 0: boxes (y1,x1,z1,y2,x2,z2); mode 1: 2-D (y1,x1,y2,x2) rows of 4.   */
/* ------------------------------------------------------------------------ */
float oracle_iou3d(const float* bi, const float* bj) {
    const float ymin_i = SMIN(bi[0], bi[3]), ymax_i = SMAX(bi[0], bi[3]);
    const float xmin_i = SMIN(bi[1], bi[4]), xmax_i = SMAX(bi[1], bi[4]);
    const float zmin_i = SMIN(bi[2], bi[5]), zmax_i = SMAX(bi[2], bi[5]);
    const float ymin_j = SMIN(bj[0], bj[3]), ymax_j = SMAX(bj[0], bj[3]);
    const float xmin_j = SMIN(bj[1], bj[4]), xmax_j = SMAX(bj[1], bj[4]);
    const float zmin_j = SMIN(bj[2], bj[5]), zmax_j = SMAX(bj[2], bj[5]);
    const float area_i = ((ymax_i - ymin_i) * (xmax_i - xmin_i)) * (zmax_i - zmin_i);
    const float area_j = ((ymax_j - ymin_j) * (xmax_j - xmin_j)) * (zmax_j - zmin_j);
    if (area_i <= 0 || area_j <= 0) return 0.0f;
    const float iymin = SMAX(ymin_i, ymin_j), iymax = SMIN(ymax_i, ymax_j);
    const float ixmin = SMAX(xmin_i, xmin_j), ixmax = SMIN(xmax_i, xmax_j);
    const float izmin = SMAX(zmin_i, zmin_j), izmax = SMIN(zmax_i, zmax_j);
    const float inter = (SMAX(iymax - iymin, 0.0f) * SMAX(ixmax - ixmin, 0.0f)) * SMAX(izmax - izmin, 0.0f);
    return inter / ((area_i + area_j) - inter);
}

float oracle_iou2d(const float* bi, const float* bj) {   /* TF 2.2 IOU<float> */
    const float ymin_i = SMIN(bi[0], bi[2]), ymax_i = SMAX(bi[0], bi[2]);
    const float xmin_i = SMIN(bi[1], bi[3]), xmax_i = SMAX(bi[1], bi[3]);
    const float ymin_j = SMIN(bj[0], bj[2]), ymax_j = SMAX(bj[0], bj[2]);
    const float xmin_j = SMIN(bj[1], bj[3]), xmax_j = SMAX(bj[1], bj[3]);
    const float area_i = (ymax_i - ymin_i) * (xmax_i - xmin_i);
    const float area_j = (ymax_j - ymin_j) * (xmax_j - xmin_j);
    if (area_i <= 0 || area_j <= 0) return 0.0f;
    const float iymin = SMAX(ymin_i, ymin_j), iymax = SMIN(ymax_i, ymax_j);
    const float ixmin = SMAX(xmin_i, xmin_j), ixmax = SMIN(xmax_i, xmax_j);
    const float inter = SMAX(iymax - iymin, 0.0f) * SMAX(ixmax - ixmin, 0.0f);
    return inter / ((area_i + area_j) - inter);
}

/* ------------------------------------------------------------------------ */
/* NonMaxSuppression3D (DoNonMaxSuppressionOp<float> @0xd0c0).   */
/* Priority queue with cmp(a,b) = (a.s==b.s && a.i>b.i) || a.s<b.s: pops the */
/* highest score, ties to the LOWER index.  Hard NMS (sigma = 0) never        */
/* re-enqueues, so the pop order is exactly the (score desc, index asc) sort  */
/* of the candidates with score > -FLT_MAX.  Suppress when IoU > thr.        */
/* ------------------------------------------------------------------------ */
typedef struct { float s; int i; } cand_t;
static int cand_cmp(const void* pa, const void* pb) {
    const cand_t* a = (const cand_t*)pa;
    const cand_t* b = (const cand_t*)pb;
    if (a->s > b->s) return -1;
    if (a->s < b->s) return 1;
    return (a->i > b->i) - (a->i < b->i);
}

int oracle_nms3d(const float* boxes, const float* scores, int N, int max_out,
                 float iou_thr, int mode, int32_t* keep) {
    if (N <= 0 || max_out <= 0) return 0;
    cand_t* c = (cand_t*)malloc(sizeof(cand_t) * (size_t)N);
    int nc = 0;
    for (int i = 0; i < N; ++i)
        if (scores[i] > -FLT_MAX) { c[nc].s = scores[i]; c[nc].i = i; ++nc; }
    qsort(c, (size_t)nc, sizeof(cand_t), cand_cmp);
    const int stride = mode == 1 ? 4 : 6;
    int nsel = 0;
    for (int q = 0; q < nc && nsel < max_out; ++q) {
        const float* bc = boxes + (size_t)c[q].i * stride;
        int suppressed = 0;
        for (int j = nsel - 1; j >= 0; --j) {   /* backwards, as @0xda47 */
            const float* bs = boxes + (size_t)keep[j] * stride;
            const float sim = mode == 1 ? oracle_iou2d(bc, bs) : oracle_iou3d(bc, bs);
            if (sim > iou_thr) { suppressed = 1; break; }
        }
        if (!suppressed) keep[nsel++] = c[q].i;
    }
    free(c);
    return nsel;
}
