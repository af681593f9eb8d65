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


FEATURE_STRIDES_YX = (4, 8, 16, 32, 64)   # P2..P6 of resnet_graph + FPN (strides (2,2,1), P6 subsample)


def patch_backbone_strides(config):
    """RPN.train's stride patch (core/models.py:3408-3419): every
    BACKBONE_STRIDES entry becomes (sy, sx, 1), because the network never
    strides depth (resnet_graph strides (2,2,1), core/models.py:242-267; FPN
    upsample (2,2,1), 3193; P6 = subsample (2,2,1), 3211).  The reference
    applies it only in RPN.train, after build() made the anchors (3225), so a
    preset with z-strides != 1 (core/config.py:40, configs/rpn/scp_rpn_hela.json)
    builds anchors that disagree with its own RPN head rows (SURVEY.md App.
    B.2).  Here it is applied before the anchors are made; returns True when
    the config changed (ANCHOR_NB is re-derived, core/config.py:235-241)."""
    fixed = []
    for s in config.BACKBONE_STRIDES:
        if isinstance(s, (tuple, list, np.ndarray)):
            fixed.append((int(s[0]), int(s[1]), 1))
        else:
            fixed.append((int(s), int(s), 1))
    old = [tuple(int(v) for v in s) if isinstance(s, (tuple, list, np.ndarray)) else (int(s),) * 3
           for s in config.BACKBONE_STRIDES]
    config.BACKBONE_STRIDES = fixed
    if hasattr(config, "IMAGE_SHAPE") and hasattr(config, "ANCHOR_NB"):
        H, W, D = (int(v) for v in config.IMAGE_SHAPE[:3])
        config.ANCHOR_NB = int(sum((H / sy) * (W / sx) * (D / sz) for sy, sx, sz in fixed[:5]))
    return fixed != old


def rpn_row_count(config, image_shape=None):
    """Rows of the shared RPN head's concatenated outputs (core/models.py:
    3250-3263): P2..P6 are (ceil(H/s), ceil(W/s), D) for s = 4..64 and the head
    emits len(RPN_ANCHOR_RATIOS) anchors per location (build_rpn_model,
    core/models.py:3244-3248)."""
    image_shape = config.IMAGE_SHAPE if image_shape is None else image_shape
    H, W, D = (int(v) for v in image_shape[:3])
    apl = len(config.RPN_ANCHOR_RATIOS)
    return int(sum(-(-H // s) * -(-W // s) * D * apl for s in FEATURE_STRIDES_YX))


def model_anchors(config, image_shape=None, inplace=True):
    """The anchors a model built from ``config`` uses: the z-stride patch
    (patch_backbone_strides), then RPN.get_anchors, checked against the RPN
    head's row count.  Raises ValueError when the preset cannot give one anchor
    per RPN row (y/x strides other than 4..64, several scales per level), where
    the reference would gather past its anchor constant.

    ``inplace``: patch the caller's config, as RPN.train does to its own
    (core/models.py:3408-3419; m3d.model.RPN).  MaskRCNN (inference,
    m3d.heads) passes False: the reference never patches there, so a z-stride-2
    preset leaves its anchors short of the head's rows and its tf.gather fails;
    here the anchors are built from a patched copy (one anchor per head row)
    and the caller's config is left as it was (a documented deviation,
    INTEGRATION.md)."""
    import copy
    import warnings
    if not inplace:
        config = copy.copy(config)
        config.BACKBONE_STRIDES = list(config.BACKBONE_STRIDES)
    if patch_backbone_strides(config):
        warnings.warn("BACKBONE_STRIDES z-components set to 1 as RPN.train does "
                      "(core/models.py:3408-3419): the network never strides depth", stacklevel=3)
    a = get_anchors(config, image_shape)
    rows = rpn_row_count(config, image_shape)
    if a.shape[0] != rows:
        raise ValueError(
            f"anchor count {a.shape[0]} != RPN head rows {rows}: BACKBONE_STRIDES {config.BACKBONE_STRIDES} "
            f"and {len(config.RPN_ANCHOR_SCALES)} RPN_ANCHOR_SCALES x {len(config.RPN_ANCHOR_RATIOS)} ratios "
            f"do not give one anchor per (y, x, z, ratio) of P2..P6 (y/x strides must be {FEATURE_STRIDES_YX}, "
            f"one scale per level; SURVEY.md App. B.2)")
    return a


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
