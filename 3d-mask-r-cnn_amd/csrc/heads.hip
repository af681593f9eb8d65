// Mask R-CNN head glue for gfx950: the small per-ROI ops between the head
// GEMMs/convs (which run on conv3d.hip's MFMA kernels) and the 2-D NMS
// (nms3d.hip, mode 1).
//
//   head_outputs_kernel   fpn_classifier_graph tail (core/models.py:1146-1186):
//                         clip(logits, -10, 10), softmax, bbox reshape
//   refine_kernel         refine_detections_graph per-ROI part
//                         (core/models.py:1415-1500): confidence filter, class-1
//                         deltas, denorm, apply_box_deltas_3d_graph
//                         (core/utils.py:412-458), clip, min size
//   detections_kernel     NMS gather, re-normalise, [max_inst, 8] rows, zero pad
//                         (core/models.py:1503-1524)
// Compiled with -ffp-contract=off like the other exact-order kernels.
#include <float.h>

#include "common.h"

namespace m3d {

__global__ void head_outputs_kernel(const float* __restrict__ raw, int64_t N, int ldr, int C,
                                    float* __restrict__ logits, float* __restrict__ probs,
                                    float* __restrict__ bbox) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float* r = raw + i * ldr;
    float mx = -FLT_MAX;
    for (int c = 0; c < C; ++c) {
        const float v = smin(smax(r[c], -10.0f), 10.0f);     // tf.clip_by_value
        logits[i * C + c] = v;
        mx = smax(mx, v);
    }
    float sum = 0.0f;
    for (int c = 0; c < C; ++c) sum += expf(logits[i * C + c] - mx);
    for (int c = 0; c < C; ++c) probs[i * C + c] = expf(logits[i * C + c] - mx) / sum;
    for (int q = 0; q < 6 * C; ++q) bbox[i * 6 * C + q] = r[C + q];
}

struct F6 { float v[6]; };

// boxes_px [N,6] refined pixel boxes; nms_boxes [N,4] = (y1,x1,y2,x2) of the
// (y,x) footprint; scores [N] = fg prob if the ROI survives the confidence and
// min-size filters, else -FLT_MAX (skipped by m3d_nms3d), so NMS indices are
// the original ROI indices and the survivors keep their order.
__global__ void refine_kernel(const float* __restrict__ rois, const float* __restrict__ probs,
                              const float* __restrict__ deltas, int64_t N, int C,
                              const float* __restrict__ meta, F6 sd, float min_conf,
                              float* __restrict__ boxes_px, float* __restrict__ nms_boxes,
                              float* __restrict__ scores) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float H = meta[5], W = meta[6], D = meta[7];
    const float fg = probs[i * C + 1];
    const float* dl = deltas + (i * C + 1) * 6;                // class id 1
    const float* r = rois + i * 6;
    const float y1 = r[0] * H, x1 = r[1] * W, z1 = r[2] * D;
    const float y2 = r[3] * H, x2 = r[4] * W, z2 = r[5] * D;
    const float dy = dl[0] * sd.v[0], dx = dl[1] * sd.v[1], dz = dl[2] * sd.v[2];
    float dh = dl[3] * sd.v[3], dw = dl[4] * sd.v[4], dd = dl[5] * sd.v[5];
    const float h = y2 - y1, w = x2 - x1, d = z2 - z1;
    const float cy = y1 + 0.5f * h, cx = x1 + 0.5f * w, cz = z1 + 0.5f * d;
    const float lim = (float)log(1000.0 / 16.0);                // LOG_SCALE_LIMIT (float64 log, as the oracle)
    dh = smin(smax(dh, -lim), lim);
    dw = smin(smax(dw, -lim), lim);
    dd = smin(smax(dd, -lim), lim);
    const float cy2 = cy + dy * h, cx2 = cx + dx * w, cz2 = cz + dz * d;
    // exp through float64 (the oracle's form, oracle/heads_ref.py): bit-identical boxes
    const float h2 = h * (float)exp((double)dh), w2 = w * (float)exp((double)dw), d2 = d * (float)exp((double)dd);
    const float ny1 = cy2 - 0.5f * h2, nx1 = cx2 - 0.5f * w2, nz1 = cz2 - 0.5f * d2;
    float b[6] = {ny1, nx1, nz1, ny1 + h2, nx1 + w2, nz1 + d2};
    const float lo[6] = {H, W, D, H, W, D};
#pragma unroll
    for (int q = 0; q < 6; ++q) b[q] = smin(smax(b[q], 0.0f), lo[q]);
    const bool ok = fg >= min_conf && (b[3] - b[0]) >= 1.0f && (b[4] - b[1]) >= 1.0f &&
                    (b[5] - b[2]) >= 0.5f;
#pragma unroll
    for (int q = 0; q < 6; ++q) boxes_px[i * 6 + q] = b[q];
    nms_boxes[i * 4 + 0] = b[0];
    nms_boxes[i * 4 + 1] = b[1];
    nms_boxes[i * 4 + 2] = b[3];
    nms_boxes[i * 4 + 3] = b[4];
    scores[i] = ok ? fg : -FLT_MAX;
}

__global__ void detections_kernel(const float* __restrict__ boxes_px,
                                  const float* __restrict__ scores,
                                  const int32_t* __restrict__ keep,
                                  const int32_t* __restrict__ num_keep, int max_inst,
                                  const float* __restrict__ meta, float* __restrict__ det) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= max_inst) return;
    float* o = det + (int64_t)j * 8;
    if (j >= *num_keep) {
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = 0.0f;
        return;
    }
    const int i = keep[j];
    const float s[6] = {meta[5], meta[6], meta[7], meta[5], meta[6], meta[7]};
#pragma unroll
    for (int q = 0; q < 6; ++q) o[q] = smin(smax(boxes_px[(int64_t)i * 6 + q] / s[q], 0.0f), 1.0f);
    o[6] = 1.0f;
    o[7] = scores[i];
}

}  // namespace m3d

using namespace m3d;

extern "C" int m3d_head_outputs(const float* raw, int64_t N, int64_t ldr, int32_t num_classes,
                                float* logits, float* probs, float* bbox, m3d_stream_t s) {
    if (N < 0 || num_classes <= 0 || ldr < 7 * (int64_t)num_classes)
        return einval("head_outputs: raw rows must hold num_classes logits + 6*num_classes deltas");
    if (N == 0) return M3D_OK;
    hipLaunchKernelGGL(head_outputs_kernel, dim3(grid_for(N, 256)), dim3(256), 0, st(s), raw, N,
                       (int)ldr, (int)num_classes, logits, probs, bbox);
    return check_launch("head_outputs_kernel");
}

extern "C" int m3d_refine_detections(const float* rois, const float* probs, const float* deltas,
                                     int64_t N, int32_t num_classes, const float* image_meta,
                                     const float bbox_std_dev[6], float min_conf,
                                     float* boxes_px, float* nms_boxes, float* scores,
                                     m3d_stream_t s) {
    if (N < 0 || num_classes < 2) return einval("refine_detections: need num_classes >= 2");
    if (N == 0) return M3D_OK;
    F6 sd{};
    for (int q = 0; q < 6; ++q) sd.v[q] = bbox_std_dev[q];
    hipLaunchKernelGGL(refine_kernel, dim3(grid_for(N, 256)), dim3(256), 0, st(s), rois, probs, deltas,
                       N, (int)num_classes, image_meta, sd, min_conf, boxes_px, nms_boxes, scores);
    return check_launch("refine_kernel");
}

extern "C" int m3d_detections_gather(const float* boxes_px, const float* scores,
                                     const int32_t* keep, const int32_t* num_keep,
                                     int32_t max_inst, const float* image_meta, float* det,
                                     m3d_stream_t s) {
    if (max_inst < 0) return einval("detections_gather: negative DETECTION_MAX_INSTANCES");
    if (max_inst == 0) return M3D_OK;
    hipLaunchKernelGGL(detections_kernel, dim3(grid_for(max_inst, 256)), dim3(256), 0, st(s), boxes_px,
                       scores, keep, num_keep, max_inst, image_meta, det);
    return check_launch("detections_kernel");
}
