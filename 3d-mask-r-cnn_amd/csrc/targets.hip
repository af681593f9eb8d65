// Training-target builders on gfx950.
//
// detection_targets_kernel -- DetectionTargetLayer / detection_targets_graph
// (core/models.py:736-1040) for one image, in ONE workgroup (no host round
// trip, fixed-size padded outputs):
//   trim zero proposals / GT rows; overlaps_graph IoU (core/models.py:695-733,
//   op order kept); iou_max and first-max GT; positive (>= pos_thr) /
//   negative (< neg_thr) sets; tf.random.shuffle of each set replaced by a
//   seeded 30-bit hash key per proposal (same distribution: a uniformly random
//   order; reproducible, so the oracle can follow it); positive_count =
//   min(int(f32(T) * ratio), #pos), negative_count = min(T - pos, #neg);
//   rows: positives, negatives, zero padding; box_refinement_graph
//   (core/utils.py:616-650, the module's final definition) / BBOX_STD_DEV;
//   mini-mask box normalisation (core/models.py:977-988).  The GT-mask crop
//   is m3d_mask_targets3d on the returned (mask_boxes, mask_assign).
// Compiled with -ffp-contract=off (exact TF float32 op order).
#include <float.h>

#include "common.h"

namespace m3d {

__device__ __forceinline__ uint32_t mix32(uint32_t x) {      // lowbias32 finaliser
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ float iou_graph(const float* a, const float* b) {
    const float y1 = smax(a[0], b[0]), x1 = smax(a[1], b[1]), z1 = smax(a[2], b[2]);
    const float y2 = smin(a[3], b[3]), x2 = smin(a[4], b[4]), z2 = smin(a[5], b[5]);
    const float inter = smax(y2 - y1, 0.0f) * smax(x2 - x1, 0.0f) * smax(z2 - z1, 0.0f);
    const float va = (a[3] - a[0]) * (a[4] - a[1]) * (a[5] - a[2]);
    const float vb = (b[3] - b[0]) * (b[4] - b[1]) * (b[5] - b[2]);
    const float uni = va + vb - inter;
    return inter / smax(uni, 1e-10f);
}

constexpr int DT_MAX_N = 16384, DT_MAX_G = 256, DT_THREADS = 1024;

struct DTArgs {
    const float* proposals;   // [N,6]
    const int32_t* gt_class_ids;
    const float* gt_boxes;    // [G,6]
    int N, G, T;
    float pos_thr, neg_thr, ratio;
    float std_[6];
    int mini_mask;
    uint32_t seed;
    float* rois;              // [T,6]
    float* roi_gt_boxes;      // [T,6]
    int32_t* class_ids;       // [T]
    float* deltas;            // [T,6]
    float* mask_boxes;        // [T,6]
    int32_t* mask_assign;     // [T] original GT index or -1
    int32_t* counts;          // [2] positives, negatives (optional)
    int32_t* assign_ws;       // [N] scratch
};

__global__ __launch_bounds__(DT_THREADS) void detection_targets_kernel(DTArgs a) {
    __shared__ uint64_t keys[DT_MAX_N];
    __shared__ float gt[DT_MAX_G][6];
    __shared__ int gt_orig[DT_MAX_G];
    __shared__ int s_ng, s_npos, s_nneg, s_nvalid;
    const int tid = threadIdx.x;
    if (tid == 0) { s_ng = 0; s_npos = 0; s_nneg = 0; s_nvalid = 0; }
    __syncthreads();
    if (tid == 0) {                       // trim_zeros_graph on the GT rows, order kept
        int ng = 0;
        for (int g = 0; g < a.G; ++g) {
            const float* b = a.gt_boxes + g * 6;
            float sa = 0.0f;
            for (int q = 0; q < 6; ++q) sa += fabsf(b[q]);
            if (sa != 0.0f) {
                for (int q = 0; q < 6; ++q) gt[ng][q] = b[q];
                gt_orig[ng++] = g;
            }
        }
        s_ng = ng;
    }
    __syncthreads();
    const int ng = s_ng;
    int npow = 1;
    while (npow < a.N) npow <<= 1;
    for (int i = tid; i < npow; i += DT_THREADS) {
        uint64_t cls = 3;                               // 3: padding / trimmed
        if (i < a.N) {
            const float* p = a.proposals + (int64_t)i * 6;
            float sa = 0.0f;
            for (int q = 0; q < 6; ++q) sa += fabsf(p[q]);
            if (sa != 0.0f) {
                atomicAdd(&s_nvalid, 1);
                float best = -FLT_MAX;
                int arg = -1;
                for (int g = 0; g < ng; ++g) {
                    const float v = iou_graph(p, gt[g]);
                    if (arg < 0 || v > best) { best = v; arg = g; }   // tf.argmax: first max
                }
                a.assign_ws[i] = arg >= 0 ? gt_orig[arg] : -1;
                if (ng > 0) {
                    if (best >= a.pos_thr) { cls = 0; atomicAdd(&s_npos, 1); }
                    else if (best < a.neg_thr) { cls = 1; atomicAdd(&s_nneg, 1); }
                    else cls = 2;
                }
            }
        }
        const uint64_t h = (uint64_t)(mix32((uint32_t)i * 0x9E3779B9u ^ a.seed) >> 2);
        keys[i] = (cls << 62) | (h << 14) | (uint64_t)(i < a.N ? i : 0);
    }
    __syncthreads();
    // bitonic sort (ascending) of npow keys
    for (int k = 2; k <= npow; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = tid; i < npow; i += DT_THREADS) {
                const int l = i ^ j;
                if (l > i) {
                    const uint64_t x = keys[i], y = keys[l];
                    const bool up = (i & k) == 0;
                    if ((x > y) == up) { keys[i] = y; keys[l] = x; }
                }
            }
            __syncthreads();
        }
    }
    const bool empty = ng == 0 || s_nvalid == 0;
    const int npos = empty ? 0 : s_npos, nneg = empty ? 0 : s_nneg;
    int pc = (int)((float)a.T * a.ratio);
    pc = pc < npos ? pc : npos;
    pc = pc > 0 ? pc : 0;
    int nc = a.T - pc;
    nc = nc < nneg ? nc : nneg;
    nc = nc > 0 ? nc : 0;
    if (tid == 0 && a.counts) { a.counts[0] = pc; a.counts[1] = nc; }
    for (int r = tid; r < a.T; r += DT_THREADS) {
        float roi[6] = {0, 0, 0, 0, 0, 0}, gtb[6] = {0, 0, 0, 0, 0, 0}, dl[6] = {0, 0, 0, 0, 0, 0};
        float mb[6] = {0, 0, 0, 0, 0, 0};
        int cid = 0, massign = -1;
        if (r < pc + nc) {
            const int i = (int)(keys[r < pc ? r : npos + (r - pc)] & 0x3FFF);
            for (int q = 0; q < 6; ++q) roi[q] = a.proposals[(int64_t)i * 6 + q];
            if (r < pc) {
                const int g = a.assign_ws[i];
                massign = g;
                cid = a.gt_class_ids[g];
                for (int q = 0; q < 6; ++q) gtb[q] = a.gt_boxes[g * 6 + q];
                const float eps = 1e-6f;
                const float h = roi[3] - roi[0], w = roi[4] - roi[1], d = roi[5] - roi[2];
                const float cy = roi[0] + 0.5f * h, cx = roi[1] + 0.5f * w, cz = roi[2] + 0.5f * d;
                const float gh = gtb[3] - gtb[0], gw = gtb[4] - gtb[1], gd = gtb[5] - gtb[2];
                const float gcy = gtb[0] + 0.5f * gh, gcx = gtb[1] + 0.5f * gw, gcz = gtb[2] + 0.5f * gd;
                dl[0] = (gcy - cy) / smax(h, eps);
                dl[1] = (gcx - cx) / smax(w, eps);
                dl[2] = (gcz - cz) / smax(d, eps);
                dl[3] = logf(smax(gh, eps) / smax(h, eps));
                dl[4] = logf(smax(gw, eps) / smax(w, eps));
                dl[5] = logf(smax(gd, eps) / smax(d, eps));
                for (int q = 0; q < 6; ++q) dl[q] = dl[q] / a.std_[q];
                if (a.mini_mask) {
                    const float ext[3] = {gh, gw, gd};
                    for (int q = 0; q < 6; ++q) mb[q] = (roi[q] - gtb[q % 3]) / ext[q % 3];
                } else {
                    for (int q = 0; q < 6; ++q) mb[q] = roi[q];
                }
            }
        }
        for (int q = 0; q < 6; ++q) {
            a.rois[r * 6 + q] = roi[q];
            a.roi_gt_boxes[r * 6 + q] = gtb[q];
            a.deltas[r * 6 + q] = dl[q];
            a.mask_boxes[r * 6 + q] = mb[q];
        }
        a.class_ids[r] = cid;
        a.mask_assign[r] = massign;
    }
}

}  // namespace m3d

using namespace m3d;

extern "C" size_t m3d_detection_targets_workspace_bytes(int64_t N) {
    return sizeof(int32_t) * (size_t)(N > 0 ? N : 1);
}

extern "C" int m3d_detection_targets(const float* proposals, int64_t N, const int32_t* gt_class_ids,
                                     const float* gt_boxes, int64_t G, int32_t train_rois_per_image,
                                     float roi_positive_ratio, float positive_iou_threshold,
                                     float negative_iou_threshold, const float bbox_std_dev[6],
                                     int32_t use_mini_mask, uint32_t seed, float* rois,
                                     float* roi_gt_boxes, int32_t* class_ids, float* deltas,
                                     float* mask_boxes, int32_t* mask_assign, int32_t* counts,
                                     void* workspace, size_t ws_bytes, m3d_stream_t s) {
    if (N < 0 || N > DT_MAX_N) return einval("detection_targets: at most 16384 proposals");
    if (G < 0 || G > DT_MAX_G) return einval("detection_targets: at most 256 GT instances");
    if (train_rois_per_image <= 0) return einval("detection_targets: TRAIN_ROIS_PER_IMAGE must be positive");
    if (ws_bytes < m3d_detection_targets_workspace_bytes(N))
        return einval("detection_targets: workspace too small");
    DTArgs a{};
    a.proposals = proposals; a.gt_class_ids = gt_class_ids; a.gt_boxes = gt_boxes;
    a.N = (int)N; a.G = (int)G; a.T = train_rois_per_image;
    a.pos_thr = positive_iou_threshold; a.neg_thr = negative_iou_threshold; a.ratio = roi_positive_ratio;
    for (int q = 0; q < 6; ++q) a.std_[q] = bbox_std_dev[q];
    a.mini_mask = use_mini_mask; a.seed = seed;
    a.rois = rois; a.roi_gt_boxes = roi_gt_boxes; a.class_ids = class_ids; a.deltas = deltas;
    a.mask_boxes = mask_boxes; a.mask_assign = mask_assign; a.counts = counts;
    a.assign_ws = (int32_t*)workspace;
    hipLaunchKernelGGL(detection_targets_kernel, dim3(1), dim3(DT_THREADS), 0, st(s), a);
    return check_launch("detection_targets_kernel");
}
