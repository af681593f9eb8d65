"""GPU DetectionTargetLayer (m3d/targets.py) vs the float32 restatement of
detection_targets_graph (oracle/heads_ref.py) with the same seeded sampling
order: selected ROIs, GT assignment, class ids and mask targets bit-exact,
box-refinement deltas to float32 log rounding."""
import numpy as np
import pytest
import torch

from oracle import heads_ref as HR
from oracle import ops_ref as R

pytestmark = pytest.mark.gpu


def _case(rng, N, G, H=32, W=32, D=16):
    gt = np.zeros((G, 6), np.float32)
    for g in range(G - 1):                              # last GT row = zero padding
        lo = rng.uniform(0.05, 0.6, 3)
        gt[g] = np.concatenate([lo, lo + rng.uniform(0.15, 0.35, 3)])
    props = np.zeros((N, 6), np.float32)
    for i in range(N - 7):                              # trailing zero padding rows
        g = gt[rng.integers(0, G - 1)]
        jit = rng.normal(0, 0.06, 6).astype(np.float32) if i % 3 else rng.uniform(-0.5, 0.5, 6).astype(np.float32)
        b = np.clip(g + jit, 0, 1)
        props[i] = np.concatenate([np.minimum(b[:3], b[3:]), np.maximum(b[:3], b[3:]) + 0.01])
    props = np.clip(props, 0, 1).astype(np.float32)
    props[-7:] = 0
    cls = rng.integers(1, 3, G).astype(np.int32)
    masks = rng.uniform(size=(H, W, D, G)) > 0.5
    return props, cls, gt, masks


@pytest.mark.parametrize("N,G,T,mini", [(300, 5, 64, False), (2000, 9, 128, True), (40, 3, 128, False)])
def test_detection_targets(cuda, N, G, T, mini):
    from m3d.targets import DetectionTargetLayer
    rng = np.random.default_rng(N)
    props, cls, gt, masks = _case(rng, N, G)
    std = [0.1, 0.1, 0.1, 0.213, 0.21, 0.15]
    layer = DetectionTargetLayer(None, T, 0.33, std, mini, (8, 8, 8), 1, positive_iou_threshold=0.5,
                                 negative_iou_threshold=0.3)
    seed = 12345
    outs = layer([torch.from_numpy(x[None]).to(cuda) for x in (props, cls, gt, masks)], seed=seed)
    rois, tgt, tcls, tdel, tmask = (o[0].cpu().numpy() for o in outs)
    ref = HR.detection_targets(props, cls, gt, T, 0.33, 0.5, 0.3, std, mini, (seed * 1000003) & 0xFFFFFFFF)
    assert np.array_equal(rois, ref[0])
    assert np.array_equal(tgt, ref[1])
    assert np.array_equal(tcls, ref[2])
    pc = int((ref[5] >= 0).sum())
    assert int(layer.last_counts[0, 0]) == pc
    assert pc > 0 or N < 100
    np.testing.assert_allclose(tdel, ref[3], rtol=2e-6, atol=2e-6)
    # mask targets: tf.round(CropAndResize3D(gt mask of the assigned GT, mask box))
    want = np.zeros_like(tmask)
    for r in range(pc):
        img = masks[..., ref[5][r]].astype(np.float32)[None, ..., None]
        crop = R.crop_and_resize_3d(img, ref[4][r:r + 1], np.zeros(1, np.int32), (8, 8, 8))
        want[r] = np.round(crop[0, ..., 0])
    assert np.array_equal(tmask, want)


def test_detection_targets_empty_gt(cuda):
    from m3d.targets import DetectionTargetLayer
    props = np.random.default_rng(0).uniform(0, 1, (50, 6)).astype(np.float32)
    layer = DetectionTargetLayer(None, 32, 0.5, [0.1] * 6, False, (4, 4, 4), 1)
    outs = layer([torch.from_numpy(x[None]).to(cuda) for x in
                  (props, np.zeros(3, np.int32), np.zeros((3, 6), np.float32), np.zeros((8, 8, 8, 3), bool))])
    for o in outs:
        assert float(o.abs().sum()) == 0.0


@pytest.mark.parametrize("S,D,G,topk,minpos", [(64, 16, 6, 24, 4), (64, 32, 12, 64, 20), (64, 16, 1, 24, 4)])
def test_build_rpn_targets(cuda, S, D, G, topk, minpos):
    """ATSS RPN targets on the GPU vs the numpy restatement (same tie rules and
    seeded negative subset): rpn_match identical, rpn_bbox to log rounding."""
    from m3d.anchors import get_anchors
    from m3d.config import synthetic_rpn_config
    from m3d.targets import build_rpn_targets
    cfg = synthetic_rpn_config(S, depth=D, RPN_POSITIVE_IOU=0.3, RPN_NEGATIVE_IOU=0.1,
                               RPN_TRAIN_ANCHORS_PER_IMAGE=512, ATSS_TOPK=topk, ATSS_MIN_POS_PER_GT=minpos)
    anchors = get_anchors(cfg)
    rng = np.random.default_rng(S + G)
    lo = rng.uniform(0, [S - 24, S - 24, D - 6], (G, 3))
    gt_px = np.concatenate([lo, lo + rng.uniform([8, 8, 2], [24, 24, 6], (G, 3))], 1).astype(np.float32)
    m, b = build_rpn_targets(torch.from_numpy(anchors).to(cuda), np.ones(G, np.int32), gt_px, cfg, seed=9)
    gt_n = np.clip(gt_px / np.array([S, S, D, S, S, D], np.float32), 0, 1).astype(np.float32)
    rm, rb = HR.build_rpn_targets(anchors, gt_n, 0.3, 0.1, 512, 0.5, topk, minpos, cfg.RPN_BBOX_STD_DEV, 9)
    m = m.cpu().numpy()
    assert np.array_equal(m, rm), (np.sum(m != rm), np.sum(m == 1), np.sum(rm == 1))
    assert (m == 1).sum() > 0 and (m == -1).sum() > 0
    np.testing.assert_allclose(b.cpu().numpy(), rb, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("S,D,G,total", [(64, 16, 6, 512), (64, 32, 12, 256), (64, 16, 1, 64), (64, 16, 0, 128)])
def test_rpn_targets_async_in_step_form(cuda, S, D, G, total):
    """m3d_rpn_targets_async (device-side balancing, no host round trip; the
    in-step builder RPNTargetBuilder) produces exactly the synchronous
    builder's rpn_match / rpn_bbox / counts -- including the stage where the
    positives exceed RPN_TRAIN_ANCHORS_PER_IMAGE * ratio and the empty-GT case
    -- and DeviceRPNTargets' mask-form losses equal the index-set losses of
    the host-prepared RPNTargets."""
    from m3d.anchors import get_anchors
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPNTargets, rpn_bbox_loss, rpn_class_loss
    from m3d.targets import RPNTargetBuilder, build_rpn_targets
    cfg = synthetic_rpn_config(S, depth=D, RPN_POSITIVE_IOU=0.3, RPN_NEGATIVE_IOU=0.1,
                               RPN_TRAIN_ANCHORS_PER_IMAGE=total, ATSS_TOPK=24, ATSS_MIN_POS_PER_GT=4)
    anchors = torch.from_numpy(get_anchors(cfg)).to(cuda)
    rng = np.random.default_rng(S + G + total)
    lo = rng.uniform(0, [S - 24, S - 24, D - 6], (G, 3))
    gt_px = np.concatenate([lo, lo + rng.uniform([8, 8, 2], [24, 24, 6], (G, 3))], 1).astype(np.float32)
    gt_n = np.clip(gt_px / np.array([S, S, D, S, S, D], np.float32), 0, 1).astype(np.float32).reshape(-1, 6)
    m_sync, b_sync = build_rpn_targets(anchors, np.ones(G, np.int32), gt_n, cfg, seed=5)
    builder = RPNTargetBuilder(anchors, cfg, max_gt=16)
    t = builder(torch.from_numpy(gt_n).to(cuda), seed=5)
    m_async = t.match.to(torch.int32)
    assert torch.equal(m_async, m_sync)
    assert torch.equal(t.bbox, b_sync)
    cnt = builder.counts.cpu().numpy()
    ms = m_sync.cpu().numpy()
    assert cnt[0] == (ms == 1).sum() and cnt[1] == (ms == -1).sum() and cnt[2] == 0
    assert cnt[0] + cnt[1] <= total or G == 0      # empty GT: every anchor negative, no balancing
    # losses: mask form (device) vs index-set form (host-prepared)
    A = anchors.shape[0]
    g = torch.Generator(device=cuda).manual_seed(3)
    logits = torch.randn((1, A, 2), device=cuda, generator=g)
    deltas = torch.randn((1, A, 6), device=cuda, generator=g)
    host = RPNTargets(ms.reshape(1, -1, 1), b_sync.cpu().numpy()[None], cuda)
    for fn, x in ((rpn_class_loss, logits), (rpn_bbox_loss, deltas)):
        a, b = float(fn(t, x)), float(fn(host, x))
        assert abs(a - b) <= 1e-6 * max(1.0, abs(b)), (fn.__name__, a, b)


def test_rpn_targets_list_cap_overflow_raises(cuda):
    """A GT whose IoU > 0 candidate list passes list_cap: the synchronous
    builder returns M3D_EINVAL (ValueError); the in-step builder raises at its
    next call / check() instead of labelling from a truncated, atomic-order
    dependent list.  The default cap (A) cannot overflow."""
    from m3d.anchors import get_anchors
    from m3d.config import synthetic_rpn_config
    from m3d.targets import RPNTargetBuilder, build_rpn_targets
    cfg = synthetic_rpn_config(64, depth=16, RPN_POSITIVE_IOU=0.3, RPN_NEGATIVE_IOU=0.1,
                               RPN_TRAIN_ANCHORS_PER_IMAGE=256, ATSS_TOPK=24, ATSS_MIN_POS_PER_GT=4)
    anchors = torch.from_numpy(get_anchors(cfg)).to(cuda)
    gt = np.array([[0.1, 0.1, 0.1, 0.9, 0.9, 0.9]], np.float32)     # overlaps most anchors
    with pytest.raises(ValueError):
        build_rpn_targets(anchors, np.ones(1, np.int32), gt, cfg, seed=1, list_cap=64)
    small = RPNTargetBuilder(anchors, cfg, max_gt=4, list_cap=64)
    gtd = torch.from_numpy(gt).to(cuda)
    small(gtd, seed=1)
    with pytest.raises(RuntimeError, match="list_cap"):
        small.check()
    small(gtd, seed=2)
    with pytest.raises(RuntimeError, match="list_cap"):
        small(gtd, seed=3)                            # raised for the previous call's flag
    full = RPNTargetBuilder(anchors, cfg, max_gt=4)
    t = full(gtd, seed=1)
    full.check()
    assert int(full.counts[2]) == 0
    m_sync, _ = build_rpn_targets(anchors, np.ones(1, np.int32), gt, cfg, seed=1)
    assert torch.equal(t.match.to(torch.int32), m_sync)
