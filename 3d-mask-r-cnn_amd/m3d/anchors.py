"""Anchor pyramid (host constant).

Restates core/utils.py:1026-1142 (generate_anchors / generate_pyramid_anchors)
and RPN.get_anchors (core/models.py:3475-3528): one scale group per level,
anchors ordered (y, x, z, anchor) to match the RPN head's reshape, clipped,
min-sized and normalised by (H, W, D).  Also compute_backbone_shapes
(core/models.py:127-147).
"""
from __future__ import annotations

import math

import numpy as np


def compute_backbone_shapes(config, image_shape):
    shapes = []
    for stride in config.BACKBONE_STRIDES:
        if isinstance(stride, (int, np.integer)):
            sy = sx = sz = int(stride)
        else:
            sy, sx, sz = stride
        shapes.append([int(math.ceil(image_shape[0] / sy)), int(math.ceil(image_shape[1] / sx)),
                       int(math.ceil(image_shape[2] / sz))])
    return np.array(shapes)


def generate_anchors(scales, ratios, shape, feature_stride, anchor_stride, max_depth=None):
    if isinstance(feature_stride, (list, tuple)):
        if len(feature_stride) == 3:
            sy, sx, sz = feature_stride
        elif len(feature_stride) == 2:
            sy = sx = feature_stride[0]
            sz = feature_stride[1]
        else:
            sy = sx = sz = int(feature_stride[0])
    else:
        sy = sx = sz = int(feature_stride)
    shifts_y = np.arange(0, shape[0], anchor_stride) * sy
    shifts_x = np.arange(0, shape[1], anchor_stride) * sx
    shifts_z = np.arange(0, shape[2], anchor_stride) * sz
    shifts_y, shifts_x, shifts_z = np.meshgrid(shifts_y, shifts_x, shifts_z, indexing="ij")
    if isinstance(scales, (int, float)):
        scales = [scales]
    if isinstance(ratios, (int, float)):
        ratios = [ratios]
    base = []
    for scale in scales:
        for ratio in ratios:
            h = w = scale
            d = scale * ratio
            d = np.clip(d, 0.5, max_depth) if max_depth is not None else max(0.5, d)
            base.append([-h / 2, -w / 2, -d / 2, h / 2, w / 2, d / 2])
    base = np.array(base, dtype=np.float32)
    sy_, sx_, sz_ = shifts_y.ravel(), shifts_x.ravel(), shifts_z.ravel()
    shifts = np.stack([sy_, sx_, sz_, sy_, sx_, sz_], axis=1)
    anchors = base[np.newaxis, :, :] + shifts[:, np.newaxis, :]
    return anchors.reshape(-1, 6).astype(np.float32)


def generate_pyramid_anchors(scales, ratios, feature_shapes, feature_strides, anchor_stride,
                             config=None):
    L = len(feature_shapes)
    scales = sorted(list(scales))
    n = len(scales)
    max_depth = None
    if config is not None:
        max_depth = getattr(config, "IMAGE_DEPTH", None)
        if max_depth is None:
            max_depth = getattr(config, "IMAGE_SHAPE", (0, 0, 16))[2]
    if n >= L:
        per, extra = n // L, n % L
        level_scales, start = [], 0
        for i in range(L):
            end = start + per + (1 if i < extra else 0)
            level_scales.append(scales[start:end])
            start = end
    else:
        level_scales = [[scales[min(i, n - 1)]] for i in range(L)]
    out = []
    for li in range(L):
        stride = feature_strides[li]
        if isinstance(stride, (list, tuple)):
            if len(stride) == 3:
                s3 = [stride[0], stride[1], stride[2]]
            elif len(stride) == 2:
                s3 = [stride[0], stride[0], stride[1]]
            else:
                s3 = [stride[0]] * 3
        else:
            s3 = [stride] * 3
        for scale in level_scales[li]:
            out.append(generate_anchors(scale, ratios, feature_shapes[li], s3, anchor_stride,
                                        max_depth))
    return np.concatenate(out, axis=0)


def get_anchors(config, image_shape=None):
    """RPN.get_anchors: normalised float32 anchors [A,6] (core/models.py:3475-3528)."""
    image_shape = config.IMAGE_SHAPE if image_shape is None else image_shape
    shapes = compute_backbone_shapes(config, image_shape)
    a = generate_pyramid_anchors(config.RPN_ANCHOR_SCALES, config.RPN_ANCHOR_RATIOS, shapes,
                                 config.BACKBONE_STRIDES, config.RPN_ANCHOR_STRIDE, config=config)
    H, W, D = int(image_shape[0]), int(image_shape[1]), int(image_shape[2])
    a[:, 0] = np.clip(a[:, 0], 0, H - 1)
    a[:, 1] = np.clip(a[:, 1], 0, W - 1)
    a[:, 2] = np.clip(a[:, 2], 0, D - 1)
    a[:, 3] = np.clip(a[:, 3], 1, H)
    a[:, 4] = np.clip(a[:, 4], 1, W)
    a[:, 5] = np.clip(a[:, 5], 1, D)
    a[:, 3] = np.maximum(a[:, 3], a[:, 0] + 1)
    a[:, 4] = np.maximum(a[:, 4], a[:, 1] + 1)
    a[:, 5] = np.maximum(a[:, 5], a[:, 2] + 0.5)
    scale = np.array([H, W, D, H, W, D], dtype=np.float32)
    return np.clip(a / scale, 0.0, 1.0).astype(np.float32)
