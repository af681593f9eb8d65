"""CPU restatement (oracle) of the reference hot-path ops and layer glue.

TEST INFRASTRUCTURE ONLY -- only tests/, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module.  The product
package (``m3d``) never imports it.

PARITY STATUS: "parity unpinned" (SURVEY.md 8c).  The reference native ops are
a prebuilt wheel without source that may not be executed here, and the
reference ships no tests or golden vectors.  These functions restate:

* ``crop_and_resize_3d*`` / ``non_max_suppression_3d``: the op semantics
  recovered from the wheel's disassembly via the C
  restatement in ``oracle/oracle.c``;
* ``proposal_layer``: ``core/models.py:369-503`` with ``apply_box_deltas_graph``
  (280-337) and ``clip_boxes_graph`` (343-366), float32 op for op;
* ``pyramid_roi_align``: ``core/models.py:597-687`` (clip, min size, level
  assignment with half-to-even rounding, per-level crop, original order,
  non-finite scrub).

They are pinned by hand-derived known-answer tests in ``tests/test_oracle.py``.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build() -> str:
    """Compile ``oracle.c`` into ``oracle/_build/liboracle.so`` (gcc)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "_build", "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        # M3D_ORACLE_LIB: an instrumented build of the same oracle.c (the
        # ASan/UBSan run of tests/test_sanitizers.py)
        path = os.environ.get("M3D_ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
        if "M3D_ORACLE_LIB" not in os.environ and (not os.path.exists(path) or os.path.getmtime(path) <
                                                   os.path.getmtime(os.path.join(_HERE, "oracle.c"))):
            build()
        L = ctypes.CDLL(path)
        fp = ctypes.POINTER(ctypes.c_float)
        ip = ctypes.POINTER(ctypes.c_int32)
        i = ctypes.c_int
        f = ctypes.c_float
        L.oracle_crop_and_resize3d.argtypes = [fp, i, i, i, i, i, fp, ip, i, i, i, i, i, f, fp]
        L.oracle_crop_and_resize3d_grad_image.argtypes = [fp, fp, ip, i, i, i, i, i, i, i, i, i, i, fp]
        L.oracle_crop_and_resize3d_grad_boxes.argtypes = [fp, fp, i, i, i, i, i, fp, ip, i, i, i, i, fp]
        L.oracle_nms3d.argtypes = [fp, fp, i, i, f, i, ip]
        L.oracle_iou3d.argtypes = [fp, fp]
        L.oracle_iou3d.restype = ctypes.c_float
        _LIB = L
    return _LIB


def _f(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _i(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))


_METHODS = {"trilinear": 0, "nearest": 1}


# --------------------------------------------------------------------------
# The four native ops (core/custom_op/custom_op.py:22-25 wrappers)
# --------------------------------------------------------------------------
def crop_and_resize_3d(image, boxes, box_ind, crop_size, method_name="trilinear",
                       extrapolation_value=0.0):
    image = np.ascontiguousarray(image, np.float32)
    boxes = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    box_ind = np.ascontiguousarray(box_ind, np.int32).reshape(-1)
    B, H, W, D, C = image.shape
    ch, cw, cd = (int(v) for v in crop_size)
    N = boxes.shape[0]
    out = np.empty((N, ch, cw, cd, C), np.float32)
    rc = lib().oracle_crop_and_resize3d(_f(image), B, H, W, D, C, _f(boxes), _i(box_ind), N,
                                        ch, cw, cd, _METHODS[method_name],
                                        float(extrapolation_value), _f(out))
    if rc != 0:
        raise ValueError("box_index has values outside [0, batch_size)")
    return out


def crop_and_resize_3d_grad_image(grads, boxes, box_ind, image_size, method_name="trilinear"):
    grads = np.ascontiguousarray(grads, np.float32)
    boxes = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    box_ind = np.ascontiguousarray(box_ind, np.int32).reshape(-1)
    B, H, W, D, C = (int(v) for v in image_size)
    N, ch, cw, cd, _ = grads.shape
    out = np.empty((B, H, W, D, C), np.float32)
    rc = lib().oracle_crop_and_resize3d_grad_image(_f(grads), _f(boxes), _i(box_ind), N, ch, cw, cd,
                                                   B, H, W, D, C, _METHODS[method_name], _f(out))
    if rc != 0:
        raise ValueError("box_index has values outside [0, batch_size)")
    return out


def crop_and_resize_3d_grad_boxes(grads, image, boxes, box_ind):
    grads = np.ascontiguousarray(grads, np.float32)
    image = np.ascontiguousarray(image, np.float32)
    boxes = np.ascontiguousarray(boxes, np.float32).reshape(-1, 6)
    box_ind = np.ascontiguousarray(box_ind, np.int32).reshape(-1)
    B, H, W, D, C = image.shape
    N, ch, cw, cd, _ = grads.shape
    out = np.empty((N, 6), np.float32)
    rc = lib().oracle_crop_and_resize3d_grad_boxes(_f(grads), _f(image), B, H, W, D, C, _f(boxes),
                                                   _i(box_ind), N, ch, cw, cd, _f(out))
    if rc != 0:
        raise ValueError("box_index has values outside [0, batch_size)")
    return out


def non_max_suppression_3d(boxes, scores, max_output_size, iou_threshold=0.5, mode="3d"):
    if not 0.0 <= iou_threshold <= 1.0:
        raise ValueError("iou_threshold must be in [0, 1]")
    cols = 4 if mode == "2d" else 6
    boxes = np.ascontiguousarray(boxes, np.float32).reshape(-1, cols)
    scores = np.ascontiguousarray(scores, np.float32).reshape(-1)
    N = boxes.shape[0]
    keep = np.zeros(max(int(max_output_size), 1), np.int32)
    n = lib().oracle_nms3d(_f(boxes), _f(scores), N, int(max_output_size), float(iou_threshold),
                           1 if mode == "2d" else 0, _i(keep))
    return keep[:n].copy()


def iou3d(bi, bj):
    bi = np.ascontiguousarray(bi, np.float32)
    bj = np.ascontiguousarray(bj, np.float32)
    return float(lib().oracle_iou3d(_f(bi), _f(bj)))


# --------------------------------------------------------------------------
# ProposalLayer (core/models.py:369-503)
# --------------------------------------------------------------------------
def stable_topk_indices(scores, k):
    """tf.nn.top_k(sorted=True): descending, equal values -> lower index first."""
    order = np.argsort(-scores.astype(np.float64), kind="stable")
    return order[:k]


def apply_box_deltas(boxes, deltas):
    """core/models.py:280-337, float32 op for op."""
    f = np.float32
    boxes = boxes.astype(f)
    deltas = np.clip(deltas.astype(f), f(-3.0), f(3.0))
    height = boxes[:, 3] - boxes[:, 0]
    width = boxes[:, 4] - boxes[:, 1]
    depth = boxes[:, 5] - boxes[:, 2]
    cy = boxes[:, 0] + f(0.5) * height
    cx = boxes[:, 1] + f(0.5) * width
    cz = boxes[:, 2] + f(0.5) * depth
    cy = cy + deltas[:, 0] * height
    cx = cx + deltas[:, 1] * width
    cz = cz + deltas[:, 2] * depth
    # exp in float64 rounded to float32: csrc/nms3d.hip computes (float)exp((double)d)
    height = height * np.exp(deltas[:, 3].astype(np.float64)).astype(f)
    width = width * np.exp(deltas[:, 4].astype(np.float64)).astype(f)
    depth = depth * np.exp(deltas[:, 5].astype(np.float64)).astype(f)
    y1 = cy - f(0.5) * height
    x1 = cx - f(0.5) * width
    z1 = cz - f(0.5) * depth
    y2 = y1 + height
    x2 = x1 + width
    z2 = z1 + depth
    res = np.stack([y1, x1, z1, y2, x2, z2], axis=1)
    return np.clip(res, f(0.0), f(1.0)).astype(f)


def clip_boxes(boxes, window):
    """core/models.py:343-366."""
    w = np.asarray(window, np.float32)
    lo = np.concatenate([w[:3], w[:3]])
    hi = np.concatenate([w[3:], w[3:]])
    return np.maximum(np.minimum(boxes, hi), lo).astype(np.float32)


def proposal_decode(probs, bbox, anchors, pre_nms_limit, rpn_bbox_std_dev, image_depth):
    """Everything in ProposalLayer.call before NMS, for one image.

    Returns (boxes [k,6], scores [k]) in top-k order (core/models.py:391-447).
    """
    f = np.float32
    scores = probs[:, 1].astype(f)
    deltas = bbox.astype(f) * np.asarray(rpn_bbox_std_dev, f).reshape(1, 6)
    deltas = np.clip(deltas, f(-3.0), f(3.0))
    k = min(int(pre_nms_limit), anchors.shape[0])
    idx = stable_topk_indices(scores, k)
    s = scores[idx]
    d = deltas[idx]
    a = anchors[idx].astype(f)
    boxes = apply_box_deltas(a, d)
    boxes = clip_boxes(boxes, [0, 0, 0, 1, 1, 1])
    eps = f(1e-6)
    img_depth = max(f(image_depth), f(1.0))
    min_d = max(f(1.0) / img_depth, f(1e-4))
    y1, x1, z1, y2, x2, z2 = (boxes[:, i] for i in range(6))
    y2 = np.maximum(y2, y1 + eps)
    x2 = np.maximum(x2, x1 + eps)
    z2 = np.maximum(z2, z1 + f(min_d))
    boxes = np.stack([y1, x1, z1, y2, x2, z2], axis=1).astype(f)
    return boxes, s, idx


def proposal_layer(probs, bbox, anchors, proposal_count, nms_threshold, pre_nms_limit,
                   rpn_bbox_std_dev, image_depth):
    """ProposalLayer.call for a batch: [B,A,2],[B,A,6],[B,A,6] -> [B,P,6]."""
    out = np.zeros((probs.shape[0], proposal_count, 6), np.float32)
    for b in range(probs.shape[0]):
        boxes, s, _ = proposal_decode(probs[b], bbox[b], anchors[b], pre_nms_limit,
                                      rpn_bbox_std_dev, image_depth)
        keep = non_max_suppression_3d(boxes, s, proposal_count, nms_threshold)
        out[b, :len(keep)] = boxes[keep]
    return out


# --------------------------------------------------------------------------
# PyramidROIAlign (core/models.py:597-687)
# --------------------------------------------------------------------------
def roi_prepare(boxes, image_shape_hwd):
    """Clip + min sizes + level (core/models.py:611-649) for one image.

    boxes [N,6] float32, image_shape_hwd (H,W,D).  Returns (boxes', level int32).
    """
    f = np.float32
    b = np.clip(boxes.astype(f), f(0.0), f(1.0))
    y1, x1, z1, y2, x2, z2 = (b[:, i].copy() for i in range(6))
    eps = f(1e-6)
    y2 = np.maximum(y2, y1 + eps)
    x2 = np.maximum(x2, x1 + eps)
    H, W, D = (f(v) for v in image_shape_hwd)
    min_dz = f(1.0) / max(D, f(1.0))
    z2 = np.maximum(z2, z1 + min_dz)
    out = np.stack([y1, x1, z1, y2, x2, z2], axis=1).astype(f)
    h = y2 - y1
    w = x2 - x1
    d = z2 - z1
    image_area = (H * W) * D
    vol = (h * w) * d
    third = f(1.0 / 3.0)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.power(vol, third) / (f(224.0) / np.power(f(image_area), third))
        lvl = np.log(r) / np.log(f(2.0))
    lvl = np.rint(lvl.astype(f))  # tf.round: half to even
    with np.errstate(invalid="ignore"):
        lvl_i = np.where(np.isfinite(lvl), lvl, -(2 ** 31)).astype(np.int64)
    lvl_i = np.minimum(5, np.maximum(2, 4 + lvl_i)).astype(np.int32)
    return out, lvl_i


def pyramid_roi_align(boxes, image_meta, feature_maps, pool_shape):
    """boxes [B,N,6], image_meta [B,M], feature_maps P2..P5 [B,H,W,D,C] -> [B,N,p,p,p,C]."""
    boxes = np.asarray(boxes, np.float32)
    Bn, N = boxes.shape[:2]
    C = feature_maps[0].shape[-1]
    ph, pw, pd = pool_shape
    out = np.zeros((Bn, N, ph, pw, pd, C), np.float32)
    for b in range(Bn):
        hwd = np.asarray(image_meta[b, 5:8], np.float32)  # core/models.py:7511-7532
        bx, lvl = roi_prepare(boxes[b], hwd)
        for li, level in enumerate(range(2, 6)):
            sel = np.nonzero(lvl == level)[0]
            if sel.size == 0:
                continue
            crops = crop_and_resize_3d(feature_maps[li], bx[sel], np.full(sel.size, b, np.int32),
                                       pool_shape)
            out[b, sel] = crops
    out[~np.isfinite(out)] = 0.0
    return out
