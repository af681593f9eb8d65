// The RPN training losses of core/models.py on gfx950, value and gradient in
// one pass:
//   rpn_class_loss_graph (core/models.py:1589-1625): focal-weighted softmax CE
//     alpha_t * (1 - p_t)^gamma * CE over the anchors with rpn_match != 0,
//     K.mean over them;
//   rpn_bbox_loss_graph (core/models.py:1629-1673): pred clipped to [-5, 5],
//     diff = gt - pred clipped to [-2, 2], Huber (threshold 1 on y/x, 0.5 with
//     half weight on z) over the positives, K.mean over their 6 * n values;
//   weighted sum LOSS_WEIGHTS (core/models.py:3366-3376).
// In the eager step these were ~100 tiny framework launches between the
// forward and the backward (the GPU idles while the host issues them); here:
//   K1 rpn_loss_terms_kernel   per anchor: both loss terms and their
//                              unnormalised gradients (d term / d logits,
//                              d term / d pred), per-workgroup partial sums
//   K2 rpn_loss_final_kernel   one workgroup: partials in a fixed order ->
//                              total / class / bbox loss and the two gradient
//                              scales (weight / denominator)
//   backward: rpn_loss_scale_kernel multiplies the kept gradients by
//                              dL/dtotal * scale, in place.
// Every sum runs in a fixed order: results are run-to-run identical.
#include <math.h>

#include "common.h"

namespace m3d {

constexpr int RL_BLOCK = 256;

struct RLPart { float cls, box; int n_valid, n_pos; };

__device__ __forceinline__ float rl_clamp(float v, float lo, float hi) { return smin(smax(v, lo), hi); }

__global__ __launch_bounds__(RL_BLOCK) void rpn_loss_terms_kernel(
        const float* __restrict__ logits, const float* __restrict__ pred,
        const int8_t* __restrict__ match, const int32_t* __restrict__ row,
        const float* __restrict__ gt, int64_t n_gt, int64_t A, float alpha, float gamma,
        float* __restrict__ g_logits, float* __restrict__ g_pred, RLPart* __restrict__ part) {
    const int64_t a = (int64_t)blockIdx.x * RL_BLOCK + threadIdx.x;
    float t_cls = 0.0f, t_box = 0.0f;
    int valid = 0, pos = 0;
    if (a < A) {
        const int m = match[a];
        float g0 = 0.0f, g1 = 0.0f;
        if (m != 0) {
            valid = 1;
            const int y = m == 1;
            const float z0 = logits[2 * a], z1 = logits[2 * a + 1];
            const float mx = smax(z0, z1);
            const float e0 = expf(z0 - mx), e1 = expf(z1 - mx);
            const float s = e0 + e1;
            const float zy = y ? z1 : z0;
            const float ce = logf(s) - (zy - mx);                 // sparse softmax CE
            const float pt = (y ? e1 : e0) / s;                    // softmax gathered at the label
            const float po = (y ? e0 : e1) / s;
            const float q = 1.0f - pt;
            const float fw = powf(q, gamma);
            const float at = y ? alpha : 1.0f - alpha;
            t_cls = at * (fw * ce);
            // d/dz_k [at * q^g * ce] = at * (p_k - [k == y]) * (g q^(g-1) p_t ce + q^g)
            const float dq = q > 0.0f ? gamma * powf(q, gamma - 1.0f) : 0.0f;
            const float b = at * (dq * pt * ce + fw);
            const float gy = -q * b, go = po * b;
            g0 = y ? go : gy;
            g1 = y ? gy : go;
        }
        g_logits[2 * a] = g0;
        g_logits[2 * a + 1] = g1;
        float gp[6] = {0, 0, 0, 0, 0, 0};
        if (m == 1) {
            pos = 1;
            int64_t r = row[a];
            r = r < 0 ? 0 : (r >= n_gt ? n_gt - 1 : r);
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                const float p = pred[a * 6 + c];
                const float pc = rl_clamp(p, -5.0f, 5.0f);
                const float d = gt[r * 6 + c] - pc;
                const float dc = rl_clamp(d, -2.0f, 2.0f);
                const float ad = fabsf(dc);
                const float sg = dc > 0.0f ? 1.0f : (dc < 0.0f ? -1.0f : 0.0f);
                float h, dh;
                if (c == 2 || c == 5) {                            // z: threshold 0.5, half slope
                    h = ad < 0.5f ? 0.5f * dc * dc : 0.5f * ad - 0.25f;
                    dh = ad < 0.5f ? dc : 0.5f * sg;
                } else {
                    h = ad < 1.0f ? 0.5f * dc * dc : ad - 0.5f;
                    dh = ad < 1.0f ? dc : sg;
                }
                t_box += h;
                // clip_by_value passes the gradient on [lo, hi] (ends included)
                const bool pass = (p >= -5.0f && p <= 5.0f) && (d >= -2.0f && d <= 2.0f);
                gp[c] = pass ? -dh : 0.0f;
            }
        }
#pragma unroll
        for (int c = 0; c < 6; ++c) g_pred[a * 6 + c] = gp[c];
    }
    // fixed-order workgroup reduction: wave butterflies, then the 4 waves in order
    for (int o = 32; o > 0; o >>= 1) {
        t_cls += __shfl_xor(t_cls, o);
        t_box += __shfl_xor(t_box, o);
        valid += __shfl_xor(valid, o);
        pos += __shfl_xor(pos, o);
    }
    __shared__ RLPart wp[RL_BLOCK / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) wp[wave] = RLPart{t_cls, t_box, valid, pos};
    __syncthreads();
    if (threadIdx.x == 0) {
        RLPart r = wp[0];
        for (int w = 1; w < RL_BLOCK / 64; ++w) {
            r.cls += wp[w].cls; r.box += wp[w].box;
            r.n_valid += wp[w].n_valid; r.n_pos += wp[w].n_pos;
        }
        part[blockIdx.x] = r;
    }
}

// total / class / bbox loss, scales[0..1] = the two gradient scales.
// den_cls / den_pos > 0: the K.mean denominators given by the host (global
// counts for a depth slab); <= 0: the counts found here (clamped to 1).
__global__ __launch_bounds__(1024) void rpn_loss_final_kernel(const RLPart* __restrict__ part, int nb,
                                                              int64_t den_cls, int64_t den_pos,
                                                              float w_cls, float w_box,
                                                              float* __restrict__ total,
                                                              float* __restrict__ cls_loss,
                                                              float* __restrict__ box_loss,
                                                              float* __restrict__ scales) {
    __shared__ double sc[1024], sb[1024];
    __shared__ long long nv[1024], np_[1024];
    const int t = threadIdx.x;
    double c = 0.0, b = 0.0;
    long long v = 0, p = 0;
    for (int i = t; i < nb; i += 1024) {
        c += part[i].cls; b += part[i].box;
        v += part[i].n_valid; p += part[i].n_pos;
    }
    sc[t] = c; sb[t] = b; nv[t] = v; np_[t] = p;
    __syncthreads();
    for (int s = 512; s > 0; s >>= 1) {
        if (t < s) {
            sc[t] += sc[t + s]; sb[t] += sb[t + s];
            nv[t] += nv[t + s]; np_[t] += np_[t + s];
        }
        __syncthreads();
    }
    if (t == 0) {
        const double dc = den_cls > 0 ? (double)den_cls : (double)(nv[0] > 0 ? nv[0] : 1);
        const double dp = den_pos > 0 ? (double)den_pos : (double)(np_[0] > 0 ? np_[0] : 1);
        const float lc = (float)(sc[0] / dc);
        const float lb = (float)(sb[0] / (6.0 * dp));
        *total = lc * w_cls + lb * w_box;
        *cls_loss = lc;
        *box_loss = lb;
        scales[0] = (float)(w_cls / dc);
        scales[1] = (float)(w_box / (6.0 * dp));
    }
}

__global__ void rpn_loss_scale_kernel(float* __restrict__ g_logits, float* __restrict__ g_pred, int64_t A,
                                      const float* __restrict__ g_total, const float* __restrict__ scales) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 8 * A) return;
    const float g = *g_total;
    if (i < 2 * A) g_logits[i] = g_logits[i] * (g * scales[0]);
    else g_pred[i - 2 * A] = g_pred[i - 2 * A] * (g * scales[1]);
}

}  // namespace m3d

using namespace m3d;

extern "C" size_t m3d_rpn_loss_workspace_bytes(int64_t A) {
    const int64_t nb = A > 0 ? (A + RL_BLOCK - 1) / RL_BLOCK : 1;
    return sizeof(RLPart) * (size_t)nb;
}

extern "C" int m3d_rpn_loss_fwd(const float* logits, const float* pred, const int8_t* match,
                                const int32_t* row, const float* gt_bbox, int64_t n_gt, int64_t A,
                                float alpha, float gamma, int64_t den_cls, int64_t den_pos,
                                float w_cls, float w_box, float* g_logits, float* g_pred, float* total,
                                float* cls_loss, float* box_loss, float* scales, void* workspace, size_t ws_bytes, m3d_stream_t s) {
    if (A < 0) return einval("rpn_loss: negative anchor count");
    if (n_gt < 1) return einval("rpn_loss: gt_bbox needs at least one row");
    if (!(gamma >= 1.0f)) return einval("rpn_loss: gamma must be >= 1");
    if (ws_bytes < m3d_rpn_loss_workspace_bytes(A)) return einval("rpn_loss: workspace too small");
    const int64_t nb = A > 0 ? (A + RL_BLOCK - 1) / RL_BLOCK : 0;
    if (nb > 0x7FFFFFFF) return einval("rpn_loss: too many anchors");
    RLPart* part = (RLPart*)workspace;
    if (nb > 0) {
        hipLaunchKernelGGL(rpn_loss_terms_kernel, dim3((unsigned)nb), dim3(RL_BLOCK), 0, st(s), logits, pred,
                           match, row, gt_bbox, n_gt, A, alpha, gamma, g_logits, g_pred, part);
        int rc = check_launch("rpn_loss_terms_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(rpn_loss_final_kernel, dim3(1), dim3(1024), 0, st(s), part, (int)nb, den_cls,
                       den_pos, w_cls, w_box, total, cls_loss, box_loss, scales);
    return check_launch("rpn_loss_final_kernel");
}

extern "C" int m3d_rpn_loss_bwd(float* g_logits, float* g_pred, int64_t A, const float* g_total,
                                const float* scales, m3d_stream_t s) {
    if (A < 0) return einval("rpn_loss: negative anchor count");
    if (A == 0) return M3D_OK;
    hipLaunchKernelGGL(rpn_loss_scale_kernel, dim3(grid_for(8 * A, 256)), dim3(256), 0, st(s), g_logits,
                       g_pred, A, g_total, scales);
    return check_launch("rpn_loss_scale_kernel");
}
