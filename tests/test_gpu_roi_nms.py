"""GPU parity: CropAndResize3D family, PyramidROIAlign, NMS3D, ProposalLayer
against the committed golden fixtures and the CPU oracle (tests/golden/)."""
import os

import numpy as np
import pytest
import torch

from oracle import ops_ref as R

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def T(a, dev, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t if dtype is None else t.to(dtype)


def test_crop_forward_bit_exact(cuda):
    from m3d import ops
    f = load("crop.npz")
    img, boxes, bi = T(f["image"], cuda), T(f["boxes"], cuda), T(f["box_ind"], cuda)
    tri = ops.crop_and_resize_3d(img, boxes, bi, (5, 4, 3), "trilinear", -1.5)
    near = ops.crop_and_resize_3d(img, boxes, bi, (5, 4, 3), "nearest", -1.5)
    one = ops.crop_and_resize_3d(img, boxes, bi, (1, 3, 1))
    np.testing.assert_array_equal(tri.cpu().numpy(), f["crops_trilinear"])
    np.testing.assert_array_equal(near.cpu().numpy(), f["crops_nearest"])
    np.testing.assert_array_equal(one.cpu().numpy(), f["crops_one"])


def test_crop_grad_image(cuda):
    from m3d import ops
    f = load("crop.npz")
    g, boxes, bi = T(f["grads"], cuda), T(f["boxes"], cuda), T(f["box_ind"], cuda)
    shape = f["image"].shape
    det = ops.crop_and_resize_3d_grad_image(g, boxes, bi, shape, deterministic=True)
    np.testing.assert_array_equal(det.cpu().numpy(), f["grad_image_trilinear"])   # same order
    fast = ops.crop_and_resize_3d_grad_image(g, boxes, bi, shape)
    np.testing.assert_allclose(fast.cpu().numpy(), f["grad_image_trilinear"], rtol=1e-5, atol=1e-5)
    near = ops.crop_and_resize_3d_grad_image(g, boxes, bi, shape, method_name="nearest",
                                             deterministic=True)
    np.testing.assert_array_equal(near.cpu().numpy(), f["grad_image_nearest"])


def test_crop_grad_boxes_and_autograd(cuda):
    from m3d import ops
    f = load("crop.npz")
    img = T(f["image"], cuda).requires_grad_(True)
    boxes = T(f["boxes"], cuda).requires_grad_(True)
    out = ops.crop_and_resize_3d(img, boxes, T(f["box_ind"], cuda), (5, 4, 3), "trilinear", -1.5)
    out.backward(T(f["grads"], cuda))
    np.testing.assert_allclose(img.grad.cpu().numpy(), f["grad_image_trilinear"], rtol=1e-5, atol=1e-5)
    # CropAndResize3DGradBoxes follows the wheel's compiled formulas and its
    # sequential summation order: bit-identical to the oracle
    np.testing.assert_array_equal(boxes.grad.cpu().numpy(), f["grad_boxes"])


def test_crop_validation_messages(cuda):
    from m3d import ops
    img = torch.zeros((1, 4, 4, 4, 2), device=cuda)
    with pytest.raises(ValueError, match="boxes must have 6 columns"):
        ops.crop_and_resize_3d(img, torch.zeros((2, 4), device=cuda),
                               torch.zeros(2, dtype=torch.int32, device=cuda), (2, 2, 2))
    with pytest.raises(ValueError, match="box_index has values outside"):
        ops.crop_and_resize_3d(img, torch.zeros((1, 6), device=cuda),
                               torch.ones(1, dtype=torch.int32, device=cuda), (2, 2, 2))
    with pytest.raises(ValueError, match="crop_size must have three elements"):
        ops.crop_and_resize_3d(img, torch.zeros((1, 6), device=cuda),
                               torch.zeros(1, dtype=torch.int32, device=cuda), (2, 2))


def test_pyramid_roi_align_bit_exact_and_grad(cuda):
    from m3d import layers
    f = load("pyramid.npz")
    maps = [T(f[k], cuda).requires_grad_(True) for k in ("p2", "p3", "p4", "p5")]
    boxes, meta = T(f["boxes"], cuda), T(f["meta"], cuda)
    out7 = layers.PyramidROIAlign((7, 7, 7), name="roi_align_classifier")([boxes, meta] + maps)
    out3 = layers.PyramidROIAlign((3, 3, 3))([boxes, meta] + maps)
    np.testing.assert_array_equal(out7.detach().cpu().numpy(), f["out7"])
    np.testing.assert_array_equal(out3.detach().cpu().numpy(), f["out3"])
    # gradient = adjoint: <out, g> == sum_l <P_l, dP_l>
    g = torch.randn_like(out7)
    out7.backward(g)
    lhs = float((out7.double() * g.double()).sum())
    rhs = sum(float((m.double() * m.grad.double()).sum()) for m in maps)
    assert abs(lhs - rhs) <= 1e-4 * (abs(lhs) + 1)


def test_nms_bit_exact(cuda):
    from m3d import ops
    f = load("nms.npz")
    keep = ops.non_max_suppression_3d(T(f["boxes"], cuda), T(f["scores"], cuda), int(f["max_out"]),
                                      float(f["thr"]))
    assert keep.dtype == torch.int32
    np.testing.assert_array_equal(keep.cpu().numpy(), f["keep"])
    tk = ops.non_max_suppression_3d(T(f["tie_boxes"], cuda), T(f["tie_scores"], cuda), 200, 0.5)
    np.testing.assert_array_equal(tk.cpu().numpy(), f["tie_keep"])
    k2, n2 = ops.non_max_suppression_3d_padded(T(f["boxes2d"], cuda), T(f["scores"], cuda), 800, 0.45,
                                               mode="2d")
    np.testing.assert_array_equal(k2[: int(n2.item())].cpu().numpy(), f["keep2d"])


@pytest.mark.parametrize("n,thr,max_out", [(0, 0.5, 10), (1, 0.5, 10), (64, 0.5, 64), (65, 0.1, 3),
                                           (15000, 0.7, 6000), (20000, 0.5, 20000),
                                           # the prefetching reduction (cb <= 256): G = 64, 15, 6, 4 row groups
                                           (1000, 0.3, 1000), (4097, 0.05, 4097), (10000, 0.9, 3000),
                                           (16384, 0.5, 16384)])
def test_nms_sizes_vs_oracle(cuda, n, thr, max_out):
    from m3d import ops
    rng = np.random.default_rng(n)
    lo = rng.uniform(0, 0.9, (n, 3)).astype(np.float32)
    sz = rng.uniform(0.005, 0.2, (n, 3)).astype(np.float32)
    boxes = np.concatenate([lo, lo + sz], 1).astype(np.float32)
    scores = np.round(rng.uniform(size=n), 3).astype(np.float32)
    want = R.non_max_suppression_3d(boxes, scores, max_out, thr)
    got = ops.non_max_suppression_3d(T(boxes, cuda), T(scores, cuda), max_out, thr)
    np.testing.assert_array_equal(got.cpu().numpy(), want)


def test_nms_repeatable(cuda):
    from m3d import ops
    f = load("nms.npz")
    b, s = T(f["boxes"], cuda), T(f["scores"], cuda)
    runs = [ops.non_max_suppression_3d(b, s, 1500, 0.3).cpu().numpy() for _ in range(5)]
    for r in runs[1:]:
        np.testing.assert_array_equal(r, runs[0])


def test_proposal_layer(cuda):
    from m3d import layers, ops
    f = load("proposal.npz")
    probs, deltas, anchors = T(f["probs"], cuda), T(f["deltas"], cuda), T(f["anchors"], cuda)
    # stage 1: top-k order identical to tf.nn.top_k (ties -> lower index)
    order = ops.topk_order(probs, 1500)
    np.testing.assert_array_equal(order.cpu().numpy(), f["order"])
    # stage 2: decode within fp32 rounding of expf
    boxes, scores = ops.proposal_decode(probs, deltas, anchors, order, f["std"], 32)
    np.testing.assert_allclose(boxes.cpu().numpy(), f["boxes"], rtol=0, atol=2e-6)
    np.testing.assert_array_equal(scores.cpu().numpy(), f["scores"])
    # stage 3: NMS on the GPU-decoded boxes is bit-exact vs the oracle on the same boxes
    want = R.non_max_suppression_3d(boxes.cpu().numpy(), scores.cpu().numpy(), 300, 0.7)
    got = ops.non_max_suppression_3d(boxes, scores, 300, 0.7)
    np.testing.assert_array_equal(got.cpu().numpy(), want)
    # whole layer
    layer = layers.ProposalLayer(300, 0.7, 1500, 1, f["std"], 32, name="ROI")
    props = layer([probs[None], deltas[None], anchors[None]])
    np.testing.assert_allclose(props[0].cpu().numpy(), f["proposals"], rtol=0, atol=2e-6)


def test_detection_mask_targets_bit_exact(cuda):
    """a12: GT-mask crop of DetectionTargetLayer, read in place + tf.round."""
    from m3d import ops
    rng = np.random.default_rng(21)
    H, W, D, G = 24, 20, 12, 5
    masks = np.zeros((H, W, D, G), bool)
    for g in range(G):
        c = rng.uniform(4, [H - 4, W - 4, D - 4])
        r = rng.uniform(2, 5, 3)
        yy, xx, zz = np.meshgrid(np.arange(H), np.arange(W), np.arange(D), indexing="ij")
        masks[..., g] = ((yy - c[0]) / r[0]) ** 2 + ((xx - c[1]) / r[1]) ** 2 + ((zz - c[2]) / r[2]) ** 2 < 1
    P = 9
    lo = rng.uniform(0, 0.6, (P, 3))
    rois = np.concatenate([lo, lo + rng.uniform(0.1, 0.4, (P, 3))], 1).astype(np.float32)
    assign = rng.integers(0, G, P).astype(np.int32)
    got = ops.detection_mask_targets(T(masks, cuda), T(rois, cuda), T(assign, cuda), (28, 28, 28))
    roi_masks = np.transpose(masks, (3, 0, 1, 2))[..., None][assign].astype(np.float32)
    want = np.rint(R.crop_and_resize_3d(roi_masks, rois, np.arange(P), (28, 28, 28))[..., 0])
    np.testing.assert_array_equal(got.cpu().numpy(), want)


@pytest.mark.parametrize("C,crop", [(64, (7, 7, 7)), (256, (14, 14, 14)), (128, (5, 9, 3)), (64, (28, 2, 1))])
def test_crop_grad_image_gather_form(cuda, C, crop):
    """CropAndResize3DGradImage's fast mode (the gather-form backward for
    C in {64..512}, crops <= 32 per axis) against the deterministic replay of
    the reference's scatter order (bit-exact to the oracle): boxes smaller than
    a voxel (all samples share corners), upsampled and downsampled boxes,
    integer-aligned coordinates (floor == ceil), boxes partly outside the image
    and flipped boxes (y2 < y1)."""
    from m3d import ops
    rng = np.random.default_rng(7)
    B, H, W, D = 2, 12, 10, 20
    lo = rng.uniform(-0.2, 0.9, (40, 3))
    hi = lo + rng.choice([0.01, 0.1, 0.4, 0.9], size=(40, 3))
    boxes = np.concatenate([lo, hi], 1)
    boxes[:4] = [[0.0, 0.0, 0.0, 1.0, 1.0, 1.0], [2 / 11, 3 / 9, 5 / 19, 6 / 11, 6 / 9, 17 / 19],
                 [0.5, 0.5, 0.5, 0.5, 0.5, 0.5], [0.9, 0.8, 0.7, 0.1, 0.2, 0.3]]
    boxes = boxes.astype(np.float32)
    bi = rng.integers(0, B, 40).astype(np.int32)
    g = rng.normal(size=(40,) + crop + (C,)).astype(np.float32)
    args = (T(g, cuda), T(boxes, cuda), T(bi, cuda), (B, H, W, D, C))
    det = ops.crop_and_resize_3d_grad_image(*args, deterministic=True).cpu().numpy()
    fast = ops.crop_and_resize_3d_grad_image(*args).cpu().numpy()
    scale = np.abs(det).max()
    assert scale > 0
    np.testing.assert_allclose(fast, det, rtol=0, atol=2e-6 * scale)
    assert np.array_equal(fast == 0, det == 0)        # the same voxels touched


@pytest.mark.parametrize("C,crop", [(256, (14, 14, 14)), (70, (7, 1, 5)), (8, (1, 1, 1))])
def test_crop_grad_boxes_bit_exact(cuda, C, crop):
    """CropAndResize3DGradBoxes (A.4: the wheel's depth scale, association and
    sequential channel order) bit-identical to the oracle, incl. single-sample
    axes (double-precision update) and C not a multiple of 64."""
    from m3d import ops
    from oracle import ops_ref as R
    rng = np.random.default_rng(17)
    img = rng.normal(size=(2, 9, 11, 13, C)).astype(np.float32)
    lo = rng.uniform(-0.1, 0.7, (6, 3))
    boxes = np.concatenate([lo, lo + rng.uniform(0.05, 0.5, (6, 3))], 1).astype(np.float32)
    bi = np.array([0, 1, 1, 0, 1, 0], np.int32)
    g = rng.normal(size=(6,) + crop + (C,)).astype(np.float32)
    got = ops.crop_and_resize_3d_grad_boxes(T(g, cuda), T(img, cuda), T(boxes, cuda), T(bi, cuda)).cpu().numpy()
    want = R.crop_and_resize_3d_grad_boxes(g, img, boxes, bi)
    np.testing.assert_array_equal(got, want)


def _det_case(rng, kind, B=2, H=9, W=7, D=11, N=23, crop=(5, 4, 3)):
    lo = rng.uniform(-0.2, 0.9, (N, 3))
    hi = lo + rng.uniform(0.02, 0.6, (N, 3))
    boxes = np.concatenate([lo, hi], 1).astype(np.float32)
    if kind == "flipped":
        boxes[::3] = boxes[::3][:, [3, 4, 5, 0, 1, 2]]
    if kind == "aligned":        # in = integer: floor == ceil, two corners on one voxel
        q = rng.integers(0, 4, (N, 6)).astype(np.float32)
        boxes = (q / np.array([H - 1, W - 1, D - 1] * 2, np.float32)).astype(np.float32)
        boxes[:, 3:] = np.maximum(boxes[:, 3:], boxes[:, :3] + np.float32(2.0 / (H - 1)))
    if kind == "tiny":           # 14 samples over ~1-2 voxels per axis (upsampling)
        c = rng.uniform(0.1, 0.9, (N, 3))
        boxes = np.concatenate([c, c + 1.5 / np.array([H, W, D])], 1).astype(np.float32)
    bi = rng.integers(0, B, N).astype(np.int32)
    return boxes, bi, (B, H, W, D)


@pytest.mark.parametrize("kind,C,crop,method", [
    ("random", 8, (5, 4, 3), "trilinear"), ("random", 3, (5, 4, 3), "trilinear"),
    ("flipped", 8, (4, 6, 5), "trilinear"), ("aligned", 4, (7, 5, 9), "trilinear"),
    ("tiny", 8, (14, 14, 14), "trilinear"), ("random", 8, (1, 4, 1), "trilinear"),
    ("random", 8, (5, 4, 3), "nearest"), ("aligned", 5, (7, 5, 9), "nearest"),
    ("random", 4, (3, 2, 70), "trilinear")])
def test_grad_image_deterministic_parallel_bit_exact(cuda, kind, C, crop, method):
    """CropAndResize3DGradImage deterministic mode 1 (destination-owned sums,
    parallel, no atomics) is bit-identical to the sequential replay (mode 2)
    and to the oracle's sequential scatter, on boxes partly outside the image,
    flipped boxes, grid-aligned boxes (floor == ceil corners), upsampling
    crops, size-1 axes, nearest mode, C % 4 != 0, several images, a NaN
    gradient, and a crop > 64 samples (mode 1 falls back to mode 2)."""
    from m3d import ops
    rng = np.random.default_rng([ord(ch) for ch in kind] + [C, *crop, len(method)])
    boxes, bi, (B, H, W, D) = _det_case(rng, kind)
    N = len(boxes)
    g = rng.normal(size=(N, *crop, C)).astype(np.float32)
    if kind == "random" and C == 8:
        g[2, 0, 0, 0, 1] = np.nan
    shape = (B, H, W, D, C)
    args = (torch.from_numpy(g).to(cuda), torch.from_numpy(boxes).to(cuda), torch.from_numpy(bi).to(cuda), shape)
    par = ops.crop_and_resize_3d_grad_image(*args, method_name=method, deterministic=1).cpu().numpy()
    ser = ops.crop_and_resize_3d_grad_image(*args, method_name=method, deterministic=2).cpu().numpy()
    want = R.crop_and_resize_3d_grad_image(g, boxes, bi, shape, method)
    np.testing.assert_array_equal(ser, want)
    np.testing.assert_array_equal(par, want)
    assert np.abs(np.nan_to_num(want)).sum() > 0
