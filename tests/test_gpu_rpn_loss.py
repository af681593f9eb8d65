"""Fused RPN losses (m3d_rpn_loss_fwd / _bwd, m3d.model.rpn_losses) against the
framework-op form of rpn_class_loss_graph / rpn_bbox_loss_graph
(core/models.py:1589-1673, weighted as 3366-3376) in m3d.model, and through it
against the float64 numpy restatement in oracle/model_ref.py: loss values and
the gradients w.r.t. the logits and the box deltas, for host-prepared
(index-set) targets with B = 2, depth-slab targets with global denominators,
device-resident (mask-form) targets, and the edge cases the reference's
tf.cond branches cover (no labelled anchor, no positive).  Tolerance: 2e-6
relative on the losses (different fp32 summation order), 1e-6 of the largest
gradient entry on the gradients; the fused path is run-to-run bit-identical."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _case(rng, B, A, n_lab, pos_frac, scale=3.0):
    match = np.zeros((B, A), np.int32)
    bbox = np.zeros((B, max(1, int(n_lab * pos_frac) + 1), 6), np.float32)
    for b in range(B):
        lab = rng.choice(A, n_lab, replace=False)
        npos = int(n_lab * pos_frac)
        match[b, lab[:npos]] = 1
        match[b, lab[npos:]] = -1
        bbox[b, :npos] = rng.normal(0, 1.5, (npos, 6))
    logits = (rng.normal(0, scale, (B, A, 2))).astype(np.float32)
    deltas = rng.normal(0, 3.0, (B, A, 6)).astype(np.float32)
    # exact clip boundaries: pred at +-5, gt - pred at +-2, |diff| at the Huber knees
    deltas[:, :4, 0] = [5.0, -5.0, 0.5, 1.0]
    return match, bbox, logits, deltas


def _both(t, logits, deltas, w=(1.0, 1.5)):
    from m3d.model import rpn_bbox_loss, rpn_class_loss, rpn_losses
    xl = torch.tensor(logits, device="cuda", requires_grad=True)
    xd = torch.tensor(deltas, device="cuda", requires_grad=True)
    tot, lc, lb = rpn_losses(t, xl, xd, *w)
    tot.backward()
    fused = (float(tot), float(lc), float(lb), xl.grad.clone(), xd.grad.clone())
    yl = torch.tensor(logits, device="cuda", requires_grad=True)
    yd = torch.tensor(deltas, device="cuda", requires_grad=True)
    rc, rb = rpn_class_loss(t, yl), rpn_bbox_loss(t, yd)
    (rc * w[0] + rb * w[1]).backward()
    ref = (float(rc * w[0] + rb * w[1]), float(rc), float(rb), yl.grad, yd.grad)
    return fused, ref


def _close(fused, ref):
    for a, b in zip(fused[:3], ref[:3]):
        assert abs(a - b) <= 2e-6 * max(1.0, abs(b)), (a, b)
    for ga, gb in zip(fused[3:], ref[3:]):
        tol = 1e-6 * max(float(gb.abs().max()), 1e-30)
        assert float((ga - gb).abs().max()) <= tol, float((ga - gb).abs().max())


@pytest.mark.parametrize("B,A,n_lab,pos_frac", [(1, 5000, 1024, 0.5), (2, 3000, 512, 0.3), (1, 777, 64, 0.0),
                                                (1, 100, 0, 0.0), (2, 4096, 4096, 1.0)])
def test_fused_rpn_losses_host_targets(cuda, B, A, n_lab, pos_frac):
    from m3d.model import RPNTargets
    rng = np.random.default_rng(A + n_lab)
    match, bbox, logits, deltas = _case(rng, B, A, n_lab, pos_frac)
    t = RPNTargets(match[..., None], bbox, cuda)
    fused, ref = _both(t, logits, deltas)
    _close(fused, ref)
    # run-to-run identical
    again, _ = _both(t, logits, deltas)
    assert fused[:3] == again[:3]
    assert torch.equal(fused[3], again[3]) and torch.equal(fused[4], again[4])


def test_fused_rpn_losses_against_oracle(cuda):
    """The fused values against oracle/model_ref.py (float64 numpy restatement
    of the reference's graphs)."""
    from m3d.model import RPNTargets, rpn_losses
    from oracle import model_ref as MR
    rng = np.random.default_rng(7)
    match, bbox, logits, deltas = _case(rng, 1, 6000, 1024, 0.4)
    t = RPNTargets(match[..., None], bbox, cuda)
    xl = torch.tensor(logits, device="cuda")
    xd = torch.tensor(deltas, device="cuda")
    _, lc, lb = rpn_losses(t, xl, xd, 1.0, 1.5)
    m = torch.from_numpy(match[..., None].astype(np.int64)).to(torch.float64)
    rc = float(MR.rpn_class_loss(m, torch.from_numpy(logits).to(torch.float64)))
    rb = float(MR.rpn_bbox_loss(torch.from_numpy(bbox).to(torch.float64), m, torch.from_numpy(deltas).to(torch.float64)))
    assert abs(float(lc) - rc) <= 2e-6 * max(1.0, abs(rc)), (float(lc), rc)
    assert abs(float(lb) - rb) <= 2e-6 * max(1.0, abs(rb)), (float(lb), rb)


def test_fused_rpn_losses_slab_targets(cuda):
    """Depth-slab targets (RPNTargets.for_slab): local terms, global denominators."""
    from m3d.model import RPNTargets
    rng = np.random.default_rng(11)
    A = 4000
    match, bbox, _, _ = _case(rng, 1, A, 1024, 0.5)
    local = np.arange(1500, 3100, dtype=np.int64)
    t = RPNTargets.for_slab(match[..., None], bbox, local, cuda)
    logits = rng.normal(0, 3, (1, len(local), 2)).astype(np.float32)
    deltas = rng.normal(0, 3, (1, len(local), 6)).astype(np.float32)
    fused, ref = _both(t, logits, deltas)
    _close(fused, ref)


def test_fused_rpn_losses_device_targets(cuda):
    """Device-resident mask-form targets (DeviceRPNTargets): counts found on the device."""
    from m3d.model import DeviceRPNTargets
    rng = np.random.default_rng(13)
    A = 5000
    match, bbox, logits, deltas = _case(rng, 1, A, 900, 0.4)
    npos = int((match == 1).sum())
    t = DeviceRPNTargets(torch.from_numpy(match.reshape(-1).astype(np.int8)).to(cuda),
                         torch.from_numpy(bbox[0, :npos]).to(cuda))
    fused, ref = _both(t, logits, deltas)
    _close(fused, ref)


def test_fused_rpn_losses_in_model_step(cuda):
    """RPN.loss_total (used by train_step) equals losses() + LOSS_WEIGHTS."""
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    cfg = synthetic_rpn_config(64, depth=8, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=300)
    model = RPN(cfg, device=cuda)
    image = synthetic_volume(64, 8, seed=0).to(cuda)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=2)
    t = RPNTargets(match, bbox, cuda)
    with torch.no_grad():
        out = model.forward(image, proposals=False)
        tot, lc, lb = model.loss_total(out, t)
        rc, rb = model.losses(out, t)
    want = float(rc) * model.LOSS_WEIGHTS["rpn_class_loss"] + float(rb) * model.LOSS_WEIGHTS["rpn_bbox_loss"]
    assert abs(float(tot) - want) <= 2e-6 * max(1.0, abs(want))
    assert abs(float(lc) - float(rc)) <= 2e-6 * max(1.0, abs(float(rc)))
    assert abs(float(lb) - float(rb)) <= 2e-6 * max(1.0, abs(float(rb)))
