"""Pin the CPU restatement (oracle/) with hand-derived known-answer tests.

The reference has no tests / golden vectors for this path and may not be
executed here, so these analytic cases -- derived from the
op semantics recovered from the wheel -- are what the
oracle is pinned by ("parity unpinned" w.r.t. the reference binary).
"""
import math

import numpy as np
import pytest

from oracle import ops_ref as R

F32_MAX = np.finfo(np.float32).max


def ramp(B, H, W, D, C, a=1.0, b=0.0, c=0.0):
    y, x, z = np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij")
    base = (a * y + b * x + c * z).astype(np.float32)
    img = np.repeat(base[None, ..., None], B, 0)
    return np.repeat(img, C, -1) + np.arange(C, dtype=np.float32) * 100.0


# ---------------------------------------------------------------- crop fwd
def test_crop_grid_aligned_is_exact_gather():
    img = np.random.default_rng(0).normal(size=(2, 9, 9, 5, 3)).astype(np.float32)
    # y: [0,1] over H=9 with 5 samples -> rows 0,2,4,6,8; x: [0.25,0.75] -> 2..6 step 1
    boxes = np.array([[0.0, 0.25, 0.0, 1.0, 0.75, 1.0]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [1], (5, 5, 5))
    np.testing.assert_array_equal(out[0], img[1][0:9:2][:, 2:7][:, :, 0:5])


def test_crop_half_grid_ramp_exact():
    img = ramp(1, 5, 5, 5, 2, a=1.0, b=3.0, c=7.0)
    boxes = np.array([[0.0, 0.0, 0.0, 1.0, 1.0, 1.0]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [0], (9, 9, 9))
    t = np.arange(9) * 0.5
    want = (t[:, None, None] + 3 * t[None, :, None] + 7 * t[None, None, :]).astype(np.float32)
    np.testing.assert_array_equal(out[0, ..., 0], want)
    np.testing.assert_array_equal(out[0, ..., 1], want + 100.0)


def test_crop_affine_field_reproduced():
    img = ramp(1, 17, 13, 11, 1, a=0.5, b=-1.25, c=2.0)
    rng = np.random.default_rng(1)
    y1, x1, z1 = rng.uniform(0, 0.5, 3)
    boxes = np.array([[y1, x1, z1, y1 + 0.4, x1 + 0.45, z1 + 0.3]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [0], (6, 7, 5))[0, ..., 0]
    b = boxes[0].astype(np.float64)
    iy = b[0] * 16 + np.arange(6) * (b[3] - b[0]) * 16 / 5
    ix = b[1] * 12 + np.arange(7) * (b[4] - b[1]) * 12 / 6
    iz = b[2] * 10 + np.arange(5) * (b[5] - b[2]) * 10 / 4
    want = 0.5 * iy[:, None, None] - 1.25 * ix[None, :, None] + 2.0 * iz[None, None, :]
    np.testing.assert_allclose(out, want, rtol=1e-5, atol=1e-4)


def test_crop_size_one_uses_centre_rule_in_double():
    img = ramp(1, 11, 11, 11, 1, a=1.0)
    y1, y2 = np.float32(0.2), np.float32(0.6)
    boxes = np.array([[y1, 0.0, 0.0, y2, 1.0, 1.0]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [0], (1, 2, 2))
    want = np.float32(0.5 * float(np.float32(y1 + y2)) * 10.0)
    assert out[0, 0, 0, 0, 0] == want


def test_crop_extrapolation_rows_planes_columns():
    img = ramp(1, 5, 5, 5, 2)
    boxes = np.array([[-0.5, 0.0, 0.0, 0.5, 1.5, 1.0]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [0], (5, 5, 3), extrapolation_value=-7.0)
    in_y = -0.5 * 4 + np.arange(5) * (1.0 * 4 / 4)
    in_x = 0.0 + np.arange(5) * (1.5 * 4 / 4)
    for yi, vy in enumerate(in_y):
        for xi, vx in enumerate(in_x):
            oob = vy < 0 or vy > 4 or vx < 0 or vx > 4
            if oob:
                assert np.all(out[0, yi, xi] == -7.0)
            else:
                assert np.all(out[0, yi, xi, :, 0] == np.float32(vy))


def test_crop_nearest_rounds_half_away_from_zero():
    img = ramp(1, 5, 5, 5, 1, a=10.0)
    boxes = np.array([[0.0, 0.0, 0.0, 1.0, 1.0, 1.0]], np.float32)
    out = R.crop_and_resize_3d(img, boxes, [0], (9, 2, 2), method_name="nearest")
    in_y = np.arange(9) * 0.5
    want = 10.0 * np.floor(in_y + 0.5)            # 0.5 -> 1, 1.5 -> 2, 2.5 -> 3 ...
    np.testing.assert_array_equal(out[0, :, 0, 0, 0], want.astype(np.float32))


def test_crop_bad_box_index_rejected():
    with pytest.raises(ValueError, match="box_index"):
        R.crop_and_resize_3d(np.zeros((1, 3, 3, 3, 1), np.float32),
                             np.zeros((1, 6), np.float32), [1], (2, 2, 2))


# ---------------------------------------------------------------- grads
def test_grad_image_is_adjoint_of_forward():
    rng = np.random.default_rng(3)
    img = rng.normal(size=(2, 8, 7, 6, 4)).astype(np.float32)
    boxes = rng.uniform(-0.1, 1.1, size=(5, 6)).astype(np.float32)
    bi = rng.integers(0, 2, size=5).astype(np.int32)
    for method in ("trilinear", "nearest"):
        crops = R.crop_and_resize_3d(img, boxes, bi, (3, 4, 5), method_name=method)
        g = rng.normal(size=crops.shape).astype(np.float32)
        gi = R.crop_and_resize_3d_grad_image(g, boxes, bi, img.shape, method_name=method)
        lhs = np.sum(crops.astype(np.float64) * g)
        rhs = np.sum(img.astype(np.float64) * gi)
        assert abs(lhs - rhs) <= 1e-4 * (abs(lhs) + 1.0)


def _fd_box_grad(img, boxes, g, crop, j, eps=1e-3):
    bp, bm = boxes.copy(), boxes.copy()
    bp[0, j] += eps
    bm[0, j] -= eps
    fp = np.sum(R.crop_and_resize_3d(img, bp, [0], crop).astype(np.float64) * g)
    fm = np.sum(R.crop_and_resize_3d(img, bm, [0], crop).astype(np.float64) * g)
    return (fp - fm) / (2 * eps)


def _grad_boxes_f64(g, img, box, crop):
    """Independent float64 numpy evaluation of A.4 (the wheel's sampling, incl.
    its depth scale (z2 - y1)(H-1)/(ch-1), and its analytic box gradient)."""
    _, H, W, D, _ = img.shape
    ch, cw, cd = crop
    y1, x1, z1, y2, x2, z2 = (float(v) for v in box)
    r = [(S - 1) / (n - 1) if n > 1 else 0.0 for S, n in ((H, ch), (W, cw), (D, cd))]
    scale = [(y2 - y1) * r[0], (x2 - x1) * r[1], (z2 - y1) * r[0]]
    lo, hi = [y1, x1, z1], [y2, x2, z2]
    out = np.zeros(6)
    im = img[0].astype(np.float64)
    for iy in range(ch):
        for ix in range(cw):
            for iz in range(cd):
                p = [lo[a] * (S - 1) + i * scale[a] if n > 1 else 0.5 * (lo[a] + hi[a]) * (S - 1)
                     for a, (S, i, n) in enumerate(((H, iy, ch), (W, ix, cw), (D, iz, cd)))]
                if any(v < 0 or v > S - 1 for v, S in zip(p, (H, W, D))):
                    continue
                t = [int(np.floor(v)) for v in p]
                b = [int(np.ceil(v)) for v in p]
                l = [v - tt for v, tt in zip(p, t)]
                c = {(a, bb, cc): im[(t, b)[a][0], (t, b)[bb][1], (t, b)[cc][2]]
                     for a in (0, 1) for bb in (0, 1) for cc in (0, 1)}
                wy, wx, wz = ((1 - l[0], l[0]), (1 - l[1], l[1]), (1 - l[2], l[2]))
                gy = sum(wx[bb] * wz[cc] * (c[1, bb, cc] - c[0, bb, cc]) for bb in (0, 1) for cc in (0, 1))
                gx = sum(wy[a] * wz[cc] * (c[a, 1, cc] - c[a, 0, cc]) for a in (0, 1) for cc in (0, 1))
                gz = sum(wy[a] * wx[bb] * (c[a, bb, 1] - c[a, bb, 0]) for a in (0, 1) for bb in (0, 1))
                gg = g[0, iy, ix, iz].astype(np.float64)
                for a, (n, i, S, ga) in enumerate(((ch, iy, H, gy), (cw, ix, W, gx), (cd, iz, D, gz))):
                    d = np.sum(ga * gg)
                    out[a] += d * ((S - 1) - i * r[a]) if n > 1 else d * 0.5 * (S - 1)
                    out[a + 3] += d * i * r[a] if n > 1 else d * 0.5 * (S - 1)
    return out


def test_grad_boxes_compiled_formulas():
    """CropAndResize3DGradBoxes (restated from the wheel's
    compiled code): (1) against an independent float64 evaluation of the same
    formulas on boxes where the wheel's depth scale (z2 - y1)(H-1)/(ch-1)
    differs from the forward's; (2) where the two coincide (y1 == z1,
    (H-1)/(ch-1) == (D-1)/(cd-1)) it is the finite-difference derivative of
    CropAndResize3D for all six coordinates; (3) single-sample axes (n == 1)."""
    rng = np.random.default_rng(4)
    y, x, z = np.meshgrid(np.linspace(0, 1, 9), np.linspace(0, 1, 8), np.linspace(0, 1, 9), indexing="ij")
    img = np.stack([np.sin(3 * y + x) * np.cos(2 * z), y * x + z * z], -1)[None].astype(np.float32)
    g = rng.normal(size=(1, 4, 3, 4, 2)).astype(np.float32)
    for box in ([0.11, 0.21, 0.19, 0.71, 0.79, 0.63], [0.3, 0.05, 0.02, 0.9, 0.6, 0.95]):
        boxes = np.array([box], np.float32)
        gb = R.crop_and_resize_3d_grad_boxes(g, img, boxes, [0])[0]
        ref = _grad_boxes_f64(g, img, boxes[0], (4, 3, 4))
        assert np.allclose(gb, ref, rtol=1e-5, atol=1e-5), (gb, ref)
    aligned = np.array([[0.16, 0.21, 0.16, 0.71, 0.79, 0.61]], np.float32)
    gb = R.crop_and_resize_3d_grad_boxes(g, img, aligned, [0])
    for j in range(6):
        fd = _fd_box_grad(img, aligned, g, (4, 3, 4), j)
        assert abs(gb[0, j] - fd) <= 2e-2 * (abs(fd) + 0.1), (j, gb[0, j], fd)
    g1 = rng.normal(size=(1, 1, 3, 1, 2)).astype(np.float32)
    gb1 = R.crop_and_resize_3d_grad_boxes(g1, img, aligned, [0])[0]
    assert np.allclose(gb1, _grad_boxes_f64(g1, img, aligned[0], (1, 3, 1)), rtol=1e-5, atol=1e-5)


# ---------------------------------------------------------------- NMS
def nms(boxes, scores, k, thr):
    return R.non_max_suppression_3d(np.asarray(boxes, np.float32), np.asarray(scores, np.float32), k, thr)


def test_iou_equal_to_threshold_is_kept():
    a = [0, 0, 0, 1, 1, 1]
    b = [0, 0, 0, 1, 1, 0.5]            # IoU = 0.5 / (1 + 0.5 - 0.5) = 0.5 exactly
    assert R.iou3d(np.array(a, np.float32), np.array(b, np.float32)) == 0.5
    assert list(nms([a, b], [0.9, 0.8], 10, 0.5)) == [0, 1]
    assert list(nms([a, b], [0.9, 0.8], 10, 0.49)) == [0]


def test_equal_scores_lower_index_first():
    box = [0.1, 0.1, 0.1, 0.5, 0.5, 0.5]
    assert list(nms([box, box, box], [0.5, 0.9, 0.9], 10, 0.5)) == [1]
    assert list(nms([box, box, [0.6, 0.6, 0.6, 0.9, 0.9, 0.9]], [0.7, 0.7, 0.7], 10, 0.5)) == [0, 2]


def test_zero_volume_boxes_never_suppress_or_get_suppressed():
    a = [0, 0, 0, 1, 1, 1]
    flat = [0, 0, 0.5, 1, 1, 0.5]
    assert list(nms([a, flat, a], [0.9, 0.8, 0.7], 10, 0.1)) == [0, 1]


def test_flipped_corners_use_min_max():
    a = [1, 1, 1, 0, 0, 0]
    b = [0, 0, 0, 1, 1, 1]
    assert R.iou3d(np.array(a, np.float32), np.array(b, np.float32)) == 1.0


def test_max_output_size_and_empty():
    rng = np.random.default_rng(5)
    lo = rng.uniform(0, 0.5, (50, 3))
    boxes = np.concatenate([lo, lo + 0.01], 1)
    keep = nms(boxes, rng.uniform(size=50), 7, 0.5)
    assert len(keep) == 7
    assert len(nms(np.zeros((0, 6)), np.zeros(0), 5, 0.5)) == 0


def test_invalid_scores_are_not_candidates():
    box = [[0.1 * i, 0, 0, 0.1 * i + 0.05, 1, 1] for i in range(5)]
    s = [np.nan, -np.inf, -F32_MAX, -F32_MAX / 2, 0.0]
    assert list(nms(box, s, 10, 0.5)) == [4, 3]


def test_nms_matches_bruteforce_greedy():
    rng = np.random.default_rng(6)
    lo = rng.uniform(0, 0.8, (300, 3)).astype(np.float32)
    sz = rng.uniform(0.02, 0.3, (300, 3)).astype(np.float32)
    boxes = np.concatenate([lo, lo + sz], 1)
    scores = np.round(rng.uniform(size=300), 2).astype(np.float32)   # many ties
    order = sorted(range(300), key=lambda i: (-scores[i], i))
    keep = []
    for i in order:
        if all(R.iou3d(boxes[i], boxes[j]) <= 0.3 for j in keep):
            keep.append(i)
    assert list(nms(boxes, scores, 1000, 0.3)) == keep


# ---------------------------------------------------------------- layer glue
def test_level_assignment_at_reference_sizes():
    # 256^3 image: pixel side s -> level clamp(4 + round(log2(s / 224)), 2, 5)
    S = 256
    sides = np.array([30, 60, 100, 150, 200, 256])
    b = np.zeros((len(sides), 6), np.float32)
    b[:, 3:] = (sides / S)[:, None]
    _, lvl = R.roi_prepare(b, (S, S, S))
    want = np.clip(4 + np.rint(np.log2(sides / 224.0)), 2, 5)
    np.testing.assert_array_equal(lvl, want)


def test_level_rounding_is_half_to_even():
    # roi_prepare uses np.rint (banker's) exactly like tf.round
    assert np.rint(np.float32(-0.5)) == 0 and np.rint(np.float32(-1.5)) == -2
    assert np.rint(np.float32(0.5)) == 0 and np.rint(np.float32(1.5)) == 2


def test_roi_prepare_min_sizes_and_clip():
    b = np.array([[-0.2, 0.3, 0.5, 1.4, 0.3, 0.5]], np.float32)
    out, _ = R.roi_prepare(b, (64, 64, 16))
    assert out[0, 0] == 0 and out[0, 3] == 1
    assert out[0, 4] == np.float32(0.3) + np.float32(1e-6)
    assert out[0, 5] == np.float32(0.5) + np.float32(1.0 / 16)


def test_pyramid_roi_align_routes_levels_in_original_order():
    rng = np.random.default_rng(7)
    S, C = 64, 4
    maps = [rng.normal(size=(1, S // s, S // s, S, C)).astype(np.float32) for s in (4, 8, 16, 32)]
    boxes = np.array([[[0.0, 0.0, 0.0, 0.2, 0.2, 0.2], [0.1, 0.1, 0.1, 0.9, 0.9, 0.9]]], np.float32)
    meta = np.zeros((1, 18), np.float32)
    meta[0, 5:8] = S
    out = R.pyramid_roi_align(boxes, meta, maps, (3, 3, 3))
    for n in range(2):
        bx, lvl = R.roi_prepare(boxes[0, n:n + 1], (S, S, S))
        want = R.crop_and_resize_3d(maps[lvl[0] - 2], bx, [0], (3, 3, 3))
        np.testing.assert_array_equal(out[0, n], want[0])


def test_apply_box_deltas_identity_and_scale():
    a = np.array([[0.2, 0.2, 0.2, 0.6, 0.4, 0.5]], np.float32)
    out = R.apply_box_deltas(a, np.zeros((1, 6), np.float32))
    np.testing.assert_allclose(out, a, atol=1e-7)
    d = np.array([[0, 0, 0, math.log(2.0), 0, 0]], np.float32)
    out = R.apply_box_deltas(a, d)
    np.testing.assert_allclose(out[0, [0, 3]], [0.0, 0.8], atol=1e-6)


def test_heads_ref_deconv_matches_torch_conv_transpose():
    """oracle/heads_ref.py's Conv3DTranspose restatement vs torch's transposed conv."""
    import torch
    from oracle import heads_ref as HR
    g = torch.Generator().manual_seed(0)
    x = torch.randn((2, 3, 2, 4, 5), generator=g, dtype=torch.float64)
    w = torch.randn((2, 2, 2, 6, 5), generator=g, dtype=torch.float64)
    b = torch.randn((6,), generator=g, dtype=torch.float64)
    pt = torch.nn.functional.conv_transpose3d(x.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2), b, stride=2)
    assert torch.allclose(pt.permute(0, 2, 3, 4, 1), HR.deconv_k2s2(x, w, b), atol=1e-12)


def test_heads_ref_refine_detections_known_answer():
    """Zero deltas keep the ROI; confidence / min-size filters; 2-D NMS over the
    (y,x) footprint suppresses a z-shifted duplicate; padding rows are zero."""
    from oracle import heads_ref as HR
    rois = np.array([[0.1, 0.1, 0.1, 0.3, 0.3, 0.3],      # kept (score .9)
                     [0.1, 0.1, 0.6, 0.3, 0.3, 0.9],      # same y/x footprint: suppressed
                     [0.5, 0.5, 0.1, 0.7, 0.7, 0.2],      # kept (score .8)
                     [0.5, 0.5, 0.5, 0.5, 0.5, 0.5],      # zero size: dropped
                     [0.8, 0.1, 0.1, 0.9, 0.2, 0.2]],     # below confidence
                    np.float32)
    fg = np.array([0.9, 0.85, 0.8, 0.95, 0.1], np.float32)
    probs = np.stack([1 - fg, fg], 1)
    deltas = np.zeros((5, 2, 6), np.float32)
    meta = np.zeros(18, np.float32)
    meta[5:8] = [100, 100, 10]
    det, kept = HR.refine_detections(rois, probs, deltas, meta, [0.1] * 6, 0.5, 0.3, 4)
    assert list(kept) == [0, 2]
    np.testing.assert_allclose(det[0, :6], rois[0], atol=1e-6)
    np.testing.assert_allclose(det[1, :6], rois[2], atol=1e-6)
    assert det[0, 7] == np.float32(0.9) and det[1, 7] == np.float32(0.8)
    assert np.all(det[2:] == 0)
