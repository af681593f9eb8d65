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
    lim = np.log(f(1000.0 / 16.0))
    dh, dw, dd = (np.minimum(np.maximum(v, -lim), lim) for v in (dh, dw, dd))
    cy2, cx2, cz2 = cy + dy * h, cx + dx * w, cz + dz * dep
    h2, w2, d2 = h * np.exp(dh), w * np.exp(dw), dep * np.exp(dd)
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
