"""Parity at the BASELINE configs' own shapes (BASELINE.json configs[1], [2]).

configs[1]: the 128^3 backbone + FPN + RPN forward against the CPU fp32
restatement (oracle/model_ref.py) at full size, and the ProposalLayer on its
outputs at full size (top-k 15000 -> decode -> 3-D NMS -> 6000).
configs[2]: the HEAD training_head_e2e chain of core/models.py:4234-4358 at
128^3 with the RPN frozen: ProposalLayer -> DetectionTargetLayer (T = 128) ->
PyramidROIAlign 7^3 and 14^3 on P2..P5 (C = 256) -> CropAndResize3DGradImage,
each stage fed the GPU's own inputs and compared with the CPU oracle
(oracle/ops_ref.py, oracle/oracle.c, oracle/heads_ref.py):
  crops / pooled features / deterministic grad_image / NMS keep / DTL sampling: bit-exact;
  decoded boxes: bit-exact (both sides evaluate exp as (float)exp((double)x));
  atomic grad_image: 1e-5 of its scale;  forward maps / logits: 1e-4 of the scale.
Head losses and head training are out of scope."""
import numpy as np
import pytest
import torch

from gradparity import deterministic, grad_parity, ref_grads
from oracle import heads_ref as HR
from oracle import model_ref as MR
from oracle import ops_ref as R

pytestmark = pytest.mark.gpu
S = 128


def rel_err(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max()) / (float(np.abs(ref).max()) + 1e-30)


@pytest.fixture(scope="module")
def fwd128(cuda):
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    cfg = synthetic_rpn_config(S)
    model = RPN(cfg, device=cuda, seed=11)
    image = synthetic_volume(S, seed=0)
    with torch.no_grad():
        out = model.forward(image.to(cuda), proposals=True)
    torch.cuda.synchronize()
    return cfg, model, image, out


def test_config1_forward_full_size(fwd128):
    """GPU fp32 forward at 128^3 vs the CPU fp32 restatement: P2..P6, logits,
    deltas within 1e-4 of each tensor's scale (north-star tolerance)."""
    cfg, model, image, out = fwd128
    torch.set_num_threads(min(16, torch.get_num_threads()))
    with torch.no_grad():
        ref = MR.RefRPN(model.store.state_dict(), dtype=torch.float32).forward(image)
    errs = {}
    for i, (a, b) in enumerate(zip(out["feature_maps"], ref["feature_maps"])):
        errs[f"P{i + 2}"] = rel_err(a.cpu().numpy(), b.numpy())
    errs["logits"] = rel_err(out["rpn_class_logits"].cpu().numpy(), ref["rpn_class_logits"].numpy())
    errs["bbox"] = rel_err(out["rpn_bbox"].cpu().numpy(), ref["rpn_bbox"].numpy())
    errs["probs"] = rel_err(out["rpn_class"].cpu().numpy(), ref["rpn_class"].numpy())
    print("configs[1] forward rel err", errs)
    assert out["rpn_class_logits"].shape == (1, 523776, 2)
    for k, e in errs.items():
        assert e < 1e-4, (k, e)


def test_config1_proposals_full_size(fwd128):
    """ProposalLayer at the training shape (15000 -> 6000, IoU 0.7) on the GPU
    RPN outputs: top-k order identical to tf.nn.top_k's, decoded boxes
    bit-exact, NMS keep indices bit-exact, and the oracle's own end-to-end
    decode -> NMS gives the same keep set; rpn_rois = gather."""
    from m3d import ops
    cfg, model, image, out = fwd128
    probs = out["rpn_class"][0].contiguous()
    deltas = out["rpn_bbox"][0].contiguous()
    anchors = model.anchors[0]
    k = min(cfg.PRE_NMS_LIMIT, anchors.shape[0])
    order = ops.topk_order(probs, k)
    boxes, scores = ops.proposal_decode(probs, deltas, anchors, order, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)
    pn, dn, an = probs.cpu().numpy(), deltas.cpu().numpy(), anchors.cpu().numpy()
    rb, rs, ridx = R.proposal_decode(pn, dn, an, cfg.PRE_NMS_LIMIT, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)
    np.testing.assert_array_equal(order.cpu().numpy(), ridx)
    np.testing.assert_array_equal(scores.cpu().numpy(), rs)
    bg = boxes.cpu().numpy()
    np.testing.assert_array_equal(bg, rb)
    keep = ops.non_max_suppression_3d(boxes, scores, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD)
    want = R.non_max_suppression_3d(bg, rs, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD)
    np.testing.assert_array_equal(keep.cpu().numpy(), want)
    rois = out["rpn_rois"][0].cpu().numpy()
    np.testing.assert_array_equal(rois[:len(want)], bg[want])
    assert not rois[len(want):].any()
    # the layer run by the oracle end to end (its own decode): the same keep
    # indices in the same order, and the layer's rpn_rois equal the oracle's
    full = R.non_max_suppression_3d(rb, rs, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD)
    np.testing.assert_array_equal(full, want)
    ref_rois = R.proposal_layer(pn[None], dn[None], an[None], cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD,
                                cfg.PRE_NMS_LIMIT, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)[0]
    np.testing.assert_array_equal(rois, ref_rois)
    print(f"configs[1] NMS: {len(want)} kept of {k}; oracle end-to-end keep set identical")


def test_decode_ulp_sensitivity(fwd128):
    """Parity risk left by the unpinned exp: perturb every decoded coordinate
    by +-1 ulp (seeded) and count how many NMS keep indices change at the
    15000 -> 6000 shape.  Reported; the bound asserts it stays a small fraction."""
    from m3d import ops
    cfg, model, image, out = fwd128
    probs = out["rpn_class"][0].contiguous()
    order = ops.topk_order(probs, cfg.PRE_NMS_LIMIT)
    boxes, scores = ops.proposal_decode(probs, out["rpn_bbox"][0].contiguous(), model.anchors[0], order,
                                        cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)
    b = boxes.cpu().numpy()
    s = scores.cpu().numpy()
    base = R.non_max_suppression_3d(b, s, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD)
    rng = np.random.default_rng(4)
    changed = []
    for trial in range(3):
        sgn = rng.choice([-1.0, 1.0], size=b.shape).astype(np.float32)
        bp = np.nextafter(b, b + sgn * np.float32(1.0)).astype(np.float32)
        kp = R.non_max_suppression_3d(bp, s, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD)
        changed.append(int(len(np.setxor1d(kp, base))))
    print(f"decode +-1ulp sensitivity: keep={len(base)}, changed indices per trial={changed}")
    assert max(changed) <= 0.01 * len(base), changed


@pytest.fixture(scope="module")
def e2e128(fwd128, cuda):
    """ProposalLayer -> DetectionTargetLayer(T=128) on the frozen 128^3 forward;
    GT boxes are jittered copies of top proposals so positives exist at IoU 0.6."""
    from m3d.targets import DetectionTargetLayer
    cfg, model, image, out = fwd128
    rois = out["rpn_rois"][0].cpu().numpy()
    rng = np.random.default_rng(3)
    G = 8
    src = rois[rng.choice(np.nonzero(np.abs(rois).sum(1) > 0)[0][:200], G, replace=False)]
    ext = np.tile(src[:, 3:] - src[:, :3], 2)                 # jitter 3 % of each box's own extent
    gt = np.clip(src + rng.normal(0, 0.03, src.shape) * ext, 0, 1).astype(np.float32)
    gt = np.concatenate([np.minimum(gt[:, :3], gt[:, 3:]), np.maximum(gt[:, :3], gt[:, 3:])], 1)
    cls = np.ones(G, np.int32)
    masks = np.zeros((S, S, S, G), bool)
    for g in range(G):
        lo = np.floor(gt[g, :3] * S).astype(int)
        hi = np.maximum(np.ceil(gt[g, 3:] * S).astype(int), lo + 1)
        masks[lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2], g] = True
    dtl = DetectionTargetLayer(cfg, cfg.TRAIN_ROIS_PER_IMAGE, cfg.ROI_POSITIVE_RATIO, cfg.BBOX_STD_DEV,
                               cfg.USE_MINI_MASK, cfg.MASK_SHAPE, 1, cfg.RPN_POSITIVE_IOU, cfg.RPN_NEGATIVE_IOU)
    seed = 77
    outs = dtl([torch.from_numpy(x[None]).to(cuda) for x in (rois, cls, gt, masks)], seed=seed)
    return cfg, out, rois, cls, gt, masks, dtl, outs, seed


def test_config2_detection_targets(e2e128):
    cfg, out, rois, cls, gt, masks, dtl, outs, seed = e2e128
    assert cfg.TRAIN_ROIS_PER_IMAGE == 128
    r_rois, r_gt, r_cls, r_del, r_mask = (o[0].cpu().numpy() for o in outs)
    ref = HR.detection_targets(rois, cls, gt, 128, cfg.ROI_POSITIVE_RATIO, cfg.RPN_POSITIVE_IOU,
                               cfg.RPN_NEGATIVE_IOU, cfg.BBOX_STD_DEV, cfg.USE_MINI_MASK,
                               (seed * 1000003) & 0xFFFFFFFF)
    assert np.array_equal(r_rois, ref[0]) and np.array_equal(r_gt, ref[1]) and np.array_equal(r_cls, ref[2])
    np.testing.assert_allclose(r_del, ref[3], rtol=2e-6, atol=2e-6)
    pc = int((ref[5] >= 0).sum())
    print(f"configs[2] DetectionTargetLayer: {pc} positives, {int((np.abs(ref[0]).sum(1) > 0).sum())} rois")
    assert pc > 0
    for r in range(pc):
        img = masks[..., ref[5][r]].astype(np.float32)[None, ..., None]
        crop = R.crop_and_resize_3d(img, ref[4][r:r + 1], np.zeros(1, np.int32), tuple(cfg.MASK_SHAPE))
        assert np.array_equal(r_mask[r], np.round(crop[0, ..., 0])), r


@pytest.mark.parametrize("pool", [7, 14])
def test_config2_pyramid_roi_align_and_grad_image(e2e128, cuda, pool):
    """PyramidROIAlign (roi_align_classifier 7^3 / roi_align_mask 14^3,
    core/models.py:4350-4358) on the 128 sampled ROIs over P2..P5 (C = 256):
    bit-exact vs the oracle; its backward (CropAndResize3DGradImage per level,
    custom_op.py:28-65): deterministic mode bit-exact, atomic mode 1e-5."""
    from m3d import layers, ops
    cfg, out, *_rest = e2e128
    outs = _rest[-2]
    rois_t = outs[0]                                          # [1,128,6] on the GPU
    maps = [m.detach().contiguous().requires_grad_(True) for m in out["feature_maps"][:4]]
    meta = np.zeros((1, cfg.IMAGE_META_SIZE), np.float32)
    meta[0, 5:9] = [S, S, S, 1]
    meta_t = torch.from_numpy(meta).to(cuda)
    layer = layers.PyramidROIAlign((pool,) * 3, name="roi_align_classifier" if pool == 7 else "roi_align_mask")
    pooled = layer([rois_t, meta_t] + maps)
    assert pooled.shape == (1, 128, pool, pool, pool, 256)
    maps_np = [m.detach().cpu().numpy() for m in maps]
    rois_np = rois_t.cpu().numpy()
    want = R.pyramid_roi_align(rois_np, meta, maps_np, (pool,) * 3)
    np.testing.assert_array_equal(pooled.detach().cpu().numpy(), want)
    # backward: atomic pyramid bwd vs the oracle's sequential scatter per level
    g = torch.randn(pooled.shape, generator=torch.Generator().manual_seed(pool)).to(cuda)
    pooled.backward(g)
    bx, lvl = R.roi_prepare(rois_np[0], meta[0, 5:8])
    gn = g.cpu().numpy()[0]
    for li, level in enumerate(range(2, 6)):
        sel = np.nonzero(lvl == level)[0]
        want_g = R.crop_and_resize_3d_grad_image(gn[sel], bx[sel], np.zeros(sel.size, np.int32),
                                                 maps_np[li].shape) if sel.size else np.zeros_like(maps_np[li])
        got = maps[li].grad.cpu().numpy()
        scale = float(np.abs(want_g).max()) + 1e-30
        assert float(np.abs(got - want_g).max()) <= 1e-5 * scale, (level, sel.size)
        if sel.size:                                          # deterministic mode: bit-exact
            det = ops.crop_and_resize_3d_grad_image(g[0][torch.from_numpy(sel).to(cuda)],
                                                    torch.from_numpy(bx[sel]).to(cuda),
                                                    torch.zeros(sel.size, dtype=torch.int32, device=cuda),
                                                    maps_np[li].shape, deterministic=True)
            np.testing.assert_array_equal(det.cpu().numpy(), want_g)
    # the whole PyramidROIAlign backward in deterministic mode (m3d_set_deterministic):
    # every level's gradient bit-exact vs the oracle's sequential scatter
    from m3d import _lib
    maps2 = [m.detach().clone().requires_grad_(True) for m in maps]
    _lib.set_deterministic(True)
    try:
        layer([rois_t, meta_t] + maps2).backward(g)
        torch.cuda.synchronize()
    finally:
        _lib.set_deterministic(False)
    for li, level in enumerate(range(2, 6)):
        sel = np.nonzero(lvl == level)[0]
        want_g = R.crop_and_resize_3d_grad_image(gn[sel], bx[sel], np.zeros(sel.size, np.int32),
                                                 maps_np[li].shape) if sel.size else np.zeros_like(maps_np[li])
        np.testing.assert_array_equal(maps2[li].grad.cpu().numpy(), want_g)
    print(f"configs[2] pool {pool}: levels {np.bincount(lvl, minlength=6)[2:].tolist()}")


def test_config1_gradients_full_size(fwd128, cuda):
    """configs[1]'s backward at its own shape (128^3, 1536 selected anchors,
    core/models.py:3320-3387): the two losses within 1e-4 of the float64
    restatement and every weight gradient held to grad_parity's bars.  The
    float64 (and the CPU fp32 yardstick) forward takes the GPU's ReLU branches
    (m3d.nn.RELU_CAPTURE): through ~60 layers a pre-activation within fp32
    rounding of 0 flips its branch in any fp32 implementation and moves every
    gradient upstream of it by up to 1e-2 (measured: the CPU fp32 restatement
    against plain float64 has median 1.3e-4, worst 1.9e-3), which would hide
    real errors behind branch noise."""
    import time
    import m3d.nn as mnn
    from m3d.model import RPNTargets, synthetic_rpn_targets
    cfg, model, image, _ = fwd128
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=2)
    model.store.zero_grad()
    mnn.RELU_CAPTURE = {}
    with deterministic():                      # the GPU step replays bit for bit
        try:
            out = model.forward(image.to(cuda), proposals=False)
            masks = mnn.RELU_CAPTURE
        finally:
            mnn.RELU_CAPTURE = None
        lc, lb = model.losses(out, RPNTargets(match, bbox, cuda))
        (lc * 1.0 + lb * 1.5).backward()
        model.rpn.finish_backward()
    torch.cuda.synchronize()
    del out
    torch.set_num_threads(min(16, torch.get_num_threads()))
    t0 = time.time()
    rlc, rlb, g64 = ref_grads(model, image, match, bbox, torch.float64, masks)
    print(f"configs[1] fp64 reference fwd+bwd {time.time() - t0:.1f} s", flush=True)
    t0 = time.time()
    _, _, g32 = ref_grads(model, image, match, bbox, torch.float32, masks)
    print(f"configs[1] fp32 reference fwd+bwd {time.time() - t0:.1f} s", flush=True)
    assert abs(float(lc) - rlc) <= 1e-4 * abs(rlc), (float(lc), rlc)
    assert abs(float(lb) - rlb) <= 1e-4 * abs(rlb), (float(lb), rlb)
    grad_parity(model, g64, g32, "configs[1]")


@pytest.mark.timeout(900)
def test_config1_gradients_atomic_and_256_paths(fwd128, cuda, monkeypatch):
    """configs[1]'s step at full shape in the DEFAULT (atomic) mode -- the
    headline path: fused RPN loss kernel, side-stream weight gradients with
    fp32-atomic split-K epilogues -- once with the 128^3 policies and once with
    the paths only 256^3 takes forced on at 128^3 (core/models.py:3162-3387):
      M3D_SHARE_WINO_MAX_GB = 0   every level of rpn_conv_shared1 on its own workspace
      M3D_WINO_KEEP_MAX_GB tiny    the large layers re-transform x in the weight gradient
      M3D_WGRAD_THROTTLE forced    the host waits for the side stream every weight gradient
    Both held to the deterministic test's bars (grad_parity) against the float64
    restatement on the GPU's ReLU branches, and to each other within the atomics'
    summation order (1e-5 of every tensor's scale)."""
    import m3d.nn as mnn
    from m3d.model import RPNTargets, synthetic_rpn_targets
    cfg, model, image, _ = fwd128
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=2)
    targets = RPNTargets(match, bbox, cuda)
    runs = []
    for forced in (False, True):
        if forced:
            monkeypatch.setattr(mnn, "SHARE_WINO_MAX_BYTES", 0)
            monkeypatch.setattr(mnn, "WINO_KEEP_MAX_BYTES", 64 << 20)
            monkeypatch.setattr(mnn, "WGRAD_THROTTLE", 1e-12)
            monkeypatch.setattr(mnn, "WGRAD_THROTTLE_EVERY", 1)
        mnn.RELU_CAPTURE = {}
        try:
            r = model.forward_backward(image.to(cuda), targets, proposals=False)
            masks = mnn.RELU_CAPTURE
        finally:
            mnn.RELU_CAPTURE = None
        torch.cuda.synchronize()
        runs.append((float(r["rpn_class_loss"]), float(r["rpn_bbox_loss"]), masks,
                     {p.name: p.grad.detach().cpu().clone() for p in model.store.params}))
    # same forward (branches) in both runs: the forced paths change no forward value
    for k in runs[0][2]:
        for a, b in zip(runs[0][2][k], runs[1][2][k]):
            assert torch.equal(a, b), k
    torch.set_num_threads(min(16, torch.get_num_threads()))
    rlc, rlb, g64 = ref_grads(model, image, match, bbox, torch.float64, runs[0][2])
    _, _, g32 = ref_grads(model, image, match, bbox, torch.float32, runs[0][2])
    for lc, lb, _m, grads in runs:
        assert abs(lc - rlc) <= 1e-4 * abs(rlc), (lc, rlc)
        assert abs(lb - rlb) <= 1e-4 * abs(rlb), (lb, rlb)
        for p in model.store.params:
            p.grad.copy_(grads[p.name].to(p.grad.device))
        grad_parity(model, g64, g32, "configs[1] atomic" + (" + 256^3 paths" if _m is runs[1][2] else ""))
    worst = max(rel_err(runs[1][3][k].numpy(), runs[0][3][k].numpy()) for k in runs[0][3])
    print(f"atomic default vs 256^3-paths-forced: worst tensor {worst:.2e}")
    assert worst < 1e-5, worst
