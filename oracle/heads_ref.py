"""CPU restatement (oracle) of the Mask R-CNN inference heads.

TEST INFRASTRUCTURE ONLY (see oracle/ops_ref.py header); the product never
imports it.  Restated from the reference's source text:

* fpn_classifier_graph (core/models.py:1121-1186): TimeDistributed
  Conv3D(fc, pool^3, 'valid') -> BN -> ReLU -> Conv3D(fc, 1^3) -> BN -> ReLU
  -> Dense(C) -> clip [-10, 10] -> softmax; Dense(6C) -> reshape [N, C, 6]
* build_fpn_mask_graph (core/models.py:1190-1234): 3x(Conv3D 3^3 same + BN +
  ReLU), res = conv3, x = res + ReLU(BN(Conv3D 3^3 dilation 2 (res))),
  conv4, Conv3DTranspose(2^3, stride 2) + ReLU, Conv3D(C, 1^3) + sigmoid
* refine_detections_graph (core/models.py:1415-1524) with
  apply_box_deltas_3d_graph (core/utils.py:412-458, the module's final
  definition), float32 op for op; tf.image.non_max_suppression as the 2-D
  mode of oracle.c's NMS.
BN in inference form x*inv + (beta - mean*inv), inv = rsqrt(var+1e-3)*gamma.
Parity status: "parity unpinned" (TF/Keras absent; reference not executable).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from . import ops_ref as R
from .model_ref import batchnorm, conv3d


def _exp32(x):
    """(float)exp((double)x): float64 exp rounded to float32, the kernels' form."""
    return np.exp(np.asarray(x, np.float64)).astype(np.float32)


def _t(p, k, dtype):
    return torch.as_tensor(np.asarray(p[k])).to(dtype)


def _bn(p, name, x, dtype):
    return batchnorm(x, _t(p, f"{name}/gamma:0", dtype), _t(p, f"{name}/beta:0", dtype),
                     _t(p, f"{name}/moving_mean:0", dtype), _t(p, f"{name}/moving_variance:0", dtype))


def classifier_head(p, pooled, num_classes, dtype=torch.float64):
    """pooled [B,N,s,s,s,C] -> logits [B,N,C], probs [B,N,C], bbox [B,N,C,6]."""
    x = torch.as_tensor(np.asarray(pooled)).to(dtype)
    B, N = x.shape[:2]
    x = x.reshape(B * N, *x.shape[2:])
    x = conv3d(x, _t(p, "mrcnn_class_conv1/kernel:0", dtype), _t(p, "mrcnn_class_conv1/bias:0", dtype),
               padding="valid")
    x = torch.relu(_bn(p, "mrcnn_class_bn1", x, dtype))
    x = conv3d(x, _t(p, "mrcnn_class_conv2/kernel:0", dtype), _t(p, "mrcnn_class_conv2/bias:0", dtype),
               padding="valid")
    x = torch.relu(_bn(p, "mrcnn_class_bn2", x, dtype))
    shared = x.reshape(B * N, -1)
    logits = shared @ _t(p, "mrcnn_class_logits/kernel:0", dtype) + _t(p, "mrcnn_class_logits/bias:0", dtype)
    logits = logits.clamp(-10.0, 10.0)
    probs = torch.softmax(logits, -1)
    bbox = shared @ _t(p, "mrcnn_bbox_fc/kernel:0", dtype) + _t(p, "mrcnn_bbox_fc/bias:0", dtype)
    C = num_classes
    return logits.reshape(B, N, C), probs.reshape(B, N, C), bbox.reshape(B, N, C, 6)


def _conv_same(p, name, x, dtype, dilation=1):
    w = _t(p, f"{name}/kernel:0", dtype)
    xt = x.permute(0, 4, 1, 2, 3)
    y = F.conv3d(xt, w.permute(4, 3, 0, 1, 2), None, padding=dilation, dilation=dilation)
    return y.permute(0, 2, 3, 4, 1) + _t(p, f"{name}/bias:0", dtype)


def deconv_k2s2(x, w, b):
    """Conv3DTranspose((2,2,2), strides 2, 'valid'): x [M,H,W,D,Ci], Keras w [2,2,2,Co,Ci]."""
    M, H, W, D, _ = x.shape
    Co = w.shape[3]
    y = torch.einsum("nhwdi,abcoi->nhawbdco", x, w)
    return y.reshape(M, 2 * H, 2 * W, 2 * D, Co) + b


def mask_head(p, pooled, num_classes, dtype=torch.float64):
    """pooled [B,N,s,s,s,C] -> masks [B,N,2s,2s,2s,num_classes] (sigmoid)."""
    x = torch.as_tensor(np.asarray(pooled)).to(dtype)
    B, N = x.shape[:2]
    x = x.reshape(B * N, *x.shape[2:])
    x = torch.relu(_bn(p, "mrcnn_mask_bn1", _conv_same(p, "mrcnn_mask_conv1", x, dtype), dtype))
    x = torch.relu(_bn(p, "mrcnn_mask_bn2", _conv_same(p, "mrcnn_mask_conv2", x, dtype), dtype))
    res = torch.relu(_bn(p, "mrcnn_mask_bn3", _conv_same(p, "mrcnn_mask_conv3", x, dtype), dtype))
    xd = torch.relu(_bn(p, "mrcnn_mask_bn3b", _conv_same(p, "mrcnn_mask_conv3b", res, dtype, 2), dtype))
    x = res + xd
    x = torch.relu(_bn(p, "mrcnn_mask_bn4", _conv_same(p, "mrcnn_mask_conv4", x, dtype), dtype))
    x = torch.relu(deconv_k2s2(x, _t(p, "mrcnn_mask_deconv/kernel:0", dtype),
                               _t(p, "mrcnn_mask_deconv/bias:0", dtype)))
    x = conv3d(x, _t(p, "mrcnn_mask/kernel:0", dtype), _t(p, "mrcnn_mask/bias:0", dtype), padding="valid")
    x = torch.sigmoid(x)
    return x.reshape(B, N, *x.shape[1:])


def refine_detections(rois, probs, deltas, image_meta, bbox_std_dev, min_conf, nms_thr, max_inst):
    """One image: rois [N,6], probs [N,C], deltas [N,C,6], image_meta [>=8]
    -> (detections [max_inst, 8] float32, kept ROI indices)."""
    f = np.float32
    rois = np.asarray(rois, f)
    probs = np.asarray(probs, f)
    deltas = np.asarray(deltas, f)
    H, W, D = (f(v) for v in np.asarray(image_meta, f)[5:8])
    fg = probs[:, 1]
    conf = np.nonzero(fg >= f(min_conf))[0]
    det = np.zeros((max_inst, 8), f)
    if conf.size == 0:
        return det, np.zeros(0, np.int64)
    scale = np.array([H, W, D, H, W, D], f)
    bx = rois[conf] * scale
    d = deltas[conf, 1] * np.asarray(bbox_std_dev, f)
    y1, x1, z1, y2, x2, z2 = (bx[:, q] for q in range(6))
    dy, dx, dz, dh, dw, dd = (d[:, q] for q in range(6))
    h, w, dep = y2 - y1, x2 - x1, z2 - z1
    cy, cx, cz = y1 + f(0.5) * h, x1 + f(0.5) * w, z1 + f(0.5) * dep
    lim = f(np.log(1000.0 / 16.0))          # float64 log rounded to float32 (= the kernel's)
    dh, dw, dd = (np.minimum(np.maximum(v, -lim), lim) for v in (dh, dw, dd))
    cy2, cx2, cz2 = cy + dy * h, cx + dx * w, cz + dz * dep
    h2, w2, d2 = (v * _exp32(e) for v, e in ((h, dh), (w, dw), (dep, dd)))
    ny1, nx1, nz1 = cy2 - f(0.5) * h2, cx2 - f(0.5) * w2, cz2 - f(0.5) * d2
    b = np.stack([ny1, nx1, nz1, ny1 + h2, nx1 + w2, nz1 + d2], 1).astype(f)
    hi = np.array([H, W, D, H, W, D], f)
    b = np.minimum(np.maximum(b, f(0)), hi)
    ok = np.nonzero(((b[:, 3] - b[:, 0]) >= f(1)) & ((b[:, 4] - b[:, 1]) >= f(1)) &
                    ((b[:, 5] - b[:, 2]) >= f(0.5)))[0]
    if ok.size == 0:
        return det, np.zeros(0, np.int64)
    b2, s2 = b[ok], fg[conf][ok]
    sel = R.non_max_suppression_3d(np.ascontiguousarray(b2[:, [0, 1, 3, 4]]), s2, max_inst, nms_thr,
                                   mode="2d")
    k = len(sel)
    det[:k, :6] = np.minimum(np.maximum(b2[sel] / scale, f(0)), f(1))
    det[:k, 6] = 1.0
    det[:k, 7] = s2[sel]
    return det, conf[ok][sel]


# ---------------------------------------------------------------------------
# DetectionTargetLayer (core/models.py:736-1040)
# ---------------------------------------------------------------------------
def _mix32(x):
    x = np.uint32(x)
    x ^= x >> np.uint32(16)
    x = np.uint32((int(x) * 0x7feb352d) & 0xFFFFFFFF)
    x ^= x >> np.uint32(15)
    x = np.uint32((int(x) * 0x846ca68b) & 0xFFFFFFFF)
    x ^= x >> np.uint32(16)
    return x


def shuffle_keys(n, seed):
    """The seeded random order that replaces tf.random.shuffle (30-bit keys, index tie-break)."""
    return [int(_mix32((i * 0x9E3779B9 & 0xFFFFFFFF) ^ seed)) >> 2 for i in range(n)]


def overlaps_graph(b1, b2):
    """core/models.py:695-733, float32."""
    f = np.float32
    b1 = np.asarray(b1, f)[:, None]
    b2 = np.asarray(b2, f)[None]
    y1 = np.maximum(b1[..., 0], b2[..., 0]); x1 = np.maximum(b1[..., 1], b2[..., 1])
    z1 = np.maximum(b1[..., 2], b2[..., 2]); y2 = np.minimum(b1[..., 3], b2[..., 3])
    x2 = np.minimum(b1[..., 4], b2[..., 4]); z2 = np.minimum(b1[..., 5], b2[..., 5])
    inter = np.maximum(y2 - y1, f(0)) * np.maximum(x2 - x1, f(0)) * np.maximum(z2 - z1, f(0))
    v1 = (b1[..., 3] - b1[..., 0]) * (b1[..., 4] - b1[..., 1]) * (b1[..., 5] - b1[..., 2])
    v2 = (b2[..., 3] - b2[..., 0]) * (b2[..., 4] - b2[..., 1]) * (b2[..., 5] - b2[..., 2])
    return (inter / np.maximum(v1 + v2 - inter, f(1e-10))).astype(f)


def box_refinement(box, gt):
    """core/utils.py:616-650 (the module's final box_refinement_graph), float32."""
    f = np.float32
    eps = f(1e-6)
    h, w, d = box[:, 3] - box[:, 0], box[:, 4] - box[:, 1], box[:, 5] - box[:, 2]
    cy, cx, cz = box[:, 0] + f(0.5) * h, box[:, 1] + f(0.5) * w, box[:, 2] + f(0.5) * d
    gh, gw, gd = gt[:, 3] - gt[:, 0], gt[:, 4] - gt[:, 1], gt[:, 5] - gt[:, 2]
    gcy, gcx, gcz = gt[:, 0] + f(0.5) * gh, gt[:, 1] + f(0.5) * gw, gt[:, 2] + f(0.5) * gd
    return np.stack([(gcy - cy) / np.maximum(h, eps), (gcx - cx) / np.maximum(w, eps),
                     (gcz - cz) / np.maximum(d, eps), np.log(np.maximum(gh, eps) / np.maximum(h, eps)),
                     np.log(np.maximum(gw, eps) / np.maximum(w, eps)),
                     np.log(np.maximum(gd, eps) / np.maximum(d, eps))], 1).astype(f)


def detection_targets(proposals, gt_class_ids, gt_boxes, T, ratio, pos_thr, neg_thr, std, use_mini_mask,
                      seed):
    """One image -> rois, roi_gt_boxes, class_ids, deltas, mask_boxes, mask_assign (all [T,...])."""
    f = np.float32
    P = np.asarray(proposals, f)
    gtb = np.asarray(gt_boxes, f)
    pv = np.nonzero(np.abs(P).sum(1) != 0)[0]
    gv = np.nonzero(np.abs(gtb).sum(1) != 0)[0]
    out = [np.zeros((T, 6), f), np.zeros((T, 6), f), np.zeros(T, np.int32), np.zeros((T, 6), f),
           np.zeros((T, 6), f), np.full(T, -1, np.int32)]
    if len(pv) == 0 or len(gv) == 0:
        return out
    ov = overlaps_graph(P[pv], gtb[gv])
    iou_max = ov.max(1)
    arg = gv[ov.argmax(1)]
    keys = shuffle_keys(len(P), seed)
    pos = [i for i, m in zip(pv, iou_max) if m >= f(pos_thr)]
    neg = [i for i, m in zip(pv, iou_max) if m < f(neg_thr)]
    pos.sort(key=lambda i: (keys[i], i))
    neg.sort(key=lambda i: (keys[i], i))
    pc = min(int(f(T) * f(ratio)), len(pos))
    nc = max(min(T - pc, len(neg)), 0)
    amap = dict(zip(pv, arg))
    sel_p = np.array(pos[:pc], np.int64)
    sel_n = np.array(neg[:nc], np.int64)
    out[0][:pc] = P[sel_p]
    out[0][pc:pc + nc] = P[sel_n]
    if pc:
        g = np.array([amap[i] for i in sel_p])
        out[1][:pc] = gtb[g]
        out[2][:pc] = np.asarray(gt_class_ids)[g]
        out[3][:pc] = box_refinement(P[sel_p], gtb[g]) / np.asarray(std, f)
        if use_mini_mask:
            ext = np.stack([gtb[g, 3] - gtb[g, 0], gtb[g, 4] - gtb[g, 1], gtb[g, 5] - gtb[g, 2]], 1)
            out[4][:pc] = (P[sel_p] - np.concatenate([gtb[g, :3], gtb[g, :3]], 1)) / np.concatenate([ext, ext], 1)
        else:
            out[4][:pc] = P[sel_p]
        out[5][:pc] = g
    return out


# ---------------------------------------------------------------------------
# build_rpn_targets (core/data_generators.py:2031-2178)
# ---------------------------------------------------------------------------
def compute_overlaps_3d(b1, b2):
    """core/utils.py:78-143, float32."""
    f = np.float32
    b1 = np.asarray(b1, f)
    b2 = np.asarray(b2, f)

    def norm(b):
        out = b.copy()
        out[:, :3] = np.minimum(b[:, :3], b[:, 3:])
        out[:, 3:] = np.maximum(b[:, :3], b[:, 3:])
        return out
    b1, b2 = norm(b1), norm(b2)
    e1, e2 = b1[:, None], b2[None]
    h = np.maximum(np.minimum(e1[..., 3], e2[..., 3]) - np.maximum(e1[..., 0], e2[..., 0]), f(0))
    w = np.maximum(np.minimum(e1[..., 4], e2[..., 4]) - np.maximum(e1[..., 1], e2[..., 1]), f(0))
    d = np.maximum(np.minimum(e1[..., 5], e2[..., 5]) - np.maximum(e1[..., 2], e2[..., 2]), f(0))
    inter = h * w * d
    v1 = ((b1[:, 3] - b1[:, 0]) * (b1[:, 4] - b1[:, 1]) * (b1[:, 5] - b1[:, 2]))[:, None]
    v2 = ((b2[:, 3] - b2[:, 0]) * (b2[:, 4] - b2[:, 1]) * (b2[:, 5] - b2[:, 2]))[None]
    union = np.maximum(v1 + v2 - inter, f(1e-10))
    return np.clip(inter / union, f(0), f(1)).astype(f)


def neg_keys(idx, seed):
    """The seeded order that picks the kept negatives (replaces np.random.choice)."""
    return [(int(_mix32((int(i) * 0x9E3779B9 & 0xFFFFFFFF) ^ seed)), -int(i)) for i in idx]


def build_rpn_targets(anchors, gt_boxes_norm, pos_iou, neg_iou, total, ratio, atss_topk, atss_min_pos, std,
                      seed):
    """Restatement of the reference with its implementation-defined orders fixed:
    top-k / ties by (IoU desc, index asc); kept negatives = the target_neg
    smallest seeded keys.  anchors [A,6], gt [G,6] normalised."""
    f = np.float32
    A, G = len(anchors), len(gt_boxes_norm)
    match = np.zeros(A, np.int32)
    bbox = np.zeros((total, 6), f)
    if G == 0:
        match[:] = -1
        return match, bbox
    ov = compute_overlaps_3d(anchors, gt_boxes_norm)
    iou_max = ov.max(1)
    match[ov.argmax(0)] = 1
    match[iou_max < f(neg_iou)] = -1
    match[iou_max >= f(pos_iou)] = 1
    for g in range(G):
        ious = ov[:, g]
        if not np.any(ious > 0):
            continue
        k = min(atss_topk, A)
        order = np.lexsort((np.arange(A), -ious))[:k]      # IoU desc, index asc
        vals = ious[order].astype(np.float64)
        mu = float(np.float32(vals.mean()))
        sd = float(np.float32(vals.std()))
        thr = np.float32(max(pos_iou, mu + sd))
        cand = np.nonzero(ious >= thr)[0]
        if cand.size < atss_min_pos:
            cand = order[:atss_min_pos]
        match[cand] = 1
    target_pos = int(round(total * ratio))
    pos = np.nonzero(match == 1)[0]
    if pos.size > target_pos:
        keep = pos[np.lexsort((pos, -iou_max[pos]))][:target_pos]
        drop = np.setdiff1d(pos, keep)
        match[drop] = 0
    neg = np.nonzero(match == -1)[0]
    target_neg = int(min(len(neg), total - int(np.sum(match == 1))))
    if len(neg) > target_neg:
        keys = neg_keys(neg, seed)
        kept = set(int(neg[j]) for j in sorted(range(len(neg)), key=lambda j: keys[j])[:max(target_neg, 0)])
        match[[i for i in neg if int(i) not in kept]] = 0
    pos = np.nonzero(match == 1)[0]
    if pos.size:
        g = ov[pos].argmax(1)
        a = np.asarray(anchors, f)[pos]
        gb = np.asarray(gt_boxes_norm, f)[g]
        d = box_refinement(a, gb) / np.asarray(std, f)
        n = min(len(d), total)
        bbox[:n] = d[:n]
    return match, bbox
