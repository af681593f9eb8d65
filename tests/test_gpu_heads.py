"""GPU parity of the Mask R-CNN inference heads (m3d/heads.py) against the CPU
restatement (oracle/heads_ref.py): classifier head and mask head within the
north-star 1e-4 of the output scale (float64 reference), DetectionLayer with
identical kept ROIs / scores and boxes to float32 rounding, plus an end-to-end
MaskRCNN.detect at a small volume."""
import numpy as np
import pytest
import torch

from oracle import heads_ref as HR

pytestmark = pytest.mark.gpu


def rel_err(got, ref):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(ref).detach().double().cpu()
    return float((got - ref).abs().max()) / (float(ref.abs().max()) + 1e-30)


def _randomize_bn(store, seed=0):
    g = torch.Generator().manual_seed(seed)
    for bn in store.bns:
        bn.moving_mean.copy_(torch.randn(bn.c, generator=g) * 0.2)
        bn.moving_variance.copy_(torch.rand(bn.c, generator=g) + 0.5)
        bn.gamma.data.copy_(torch.rand(bn.c, generator=g) + 0.5)
        bn.beta.data.copy_(torch.randn(bn.c, generator=g) * 0.1)


def _store(cuda, build):
    from m3d.params import ParamStore
    store = ParamStore()
    head = build(store)
    store.finalize(cuda, seed=3)
    with torch.no_grad():
        _randomize_bn(store)
    return store, head


@pytest.mark.parametrize("pool,C,fc,N", [(7, 256, 512, 37), (3, 64, 128, 130)])
def test_classifier_head(cuda, pool, C, fc, N):
    from m3d.heads import ClassifierHead
    store, head = _store(cuda, lambda s: ClassifierHead(s, pool, 2, fc, C))
    g = torch.Generator().manual_seed(1)
    pooled = torch.randn((1, N, pool, pool, pool, C), generator=g)
    with torch.no_grad():
        logits, probs, bbox = head(pooled.to(cuda))
    rl, rp, rb = HR.classifier_head(store.state_dict(), pooled, 2)
    assert rel_err(logits, rl) < 1e-4
    assert rel_err(probs, rp) < 1e-4
    assert rel_err(bbox, rb) < 1e-4


def test_mask_head(cuda):
    from m3d.heads import MaskHead
    store, head = _store(cuda, lambda s: MaskHead(s, 2, 128, 128))
    g = torch.Generator().manual_seed(2)
    pooled = torch.randn((1, 3, 6, 6, 6, 128), generator=g)
    with torch.no_grad():
        m = head(pooled.to(cuda))
    ref = HR.mask_head(store.state_dict(), pooled, 2)
    assert m.shape == (1, 3, 12, 12, 12, 2)
    assert rel_err(m, ref) < 1e-4


def test_deconv_k2s2(cuda):
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(4)
    x = torch.randn((2, 3, 4, 5, 64), generator=g)
    w = torch.randn((2, 2, 2, 36, 64), generator=g) * 0.1
    b = torch.randn((36,), generator=g)
    ref = torch.relu(HR.deconv_k2s2(x.double(), w.double(), b.double()))
    # the restatement itself against torch's transposed conv (weight [Ci, Co, 2, 2, 2])
    pt = torch.nn.functional.conv_transpose3d(x.double().permute(0, 4, 1, 2, 3),
                                              w.double().permute(4, 3, 0, 1, 2), b.double(), stride=2)
    assert torch.allclose(torch.relu(pt.permute(0, 2, 3, 4, 1)), ref, atol=1e-10)
    xd, wd, bd = x.to(cuda), w.to(cuda), b.to(cuda)
    y = torch.empty((2, 6, 8, 10, 36), device=cuda)
    _lib.check(L.m3d_deconv3d_k2s2(xd.data_ptr(), 2, 3, 4, 5, 64, wd.data_ptr(), 36, bd.data_ptr(), 1,
                                   y.data_ptr(), _lib.stream()))
    assert rel_err(y, ref) < 1e-5


def test_detection_layer(cuda):
    from m3d.heads import DetectionLayer
    rng = np.random.default_rng(5)
    N, C = 300, 2
    lo = rng.uniform(0, 0.8, (N, 3))
    rois = np.concatenate([lo, lo + rng.uniform(0.02, 0.2, (N, 3))], 1).astype(np.float32)
    rois[-20:] = 0.0                                    # ProposalLayer zero padding
    p1 = rng.uniform(0, 1, N).astype(np.float32)
    probs = np.stack([1 - p1, p1], 1).astype(np.float32)
    deltas = rng.normal(0, 1.0, (N, C, 6)).astype(np.float32)
    deltas[:5, 1, 3:] = 9.0                             # LOG_SCALE_LIMIT clip
    meta = np.zeros(18, np.float32)
    meta[5:8] = [64, 64, 32]
    std = [0.1, 0.1, 0.1, 0.213, 0.21, 0.15]
    layer = DetectionLayer(std, 0.3, 40, 0.3, 1)
    det = layer([torch.from_numpy(x[None]).to(cuda) for x in (rois, probs, deltas, meta)]).cpu().numpy()[0]
    ref, kept = HR.refine_detections(rois, probs, deltas, meta, std, 0.3, 0.3, 40)
    n = len(kept)
    assert n > 5
    assert np.array_equal(det[:n, 7], ref[:n, 7]), "kept detections / order differ"
    np.testing.assert_allclose(det[:n, :6], ref[:n, :6], rtol=0, atol=2e-6)
    assert np.all(det[n:] == 0) and np.all(det[:n, 6] == 1.0)


def test_maskrcnn_detect_end_to_end(cuda):
    """Full inference graph at 64x64x16: every stage runs on the GPU and the
    head outputs match the restatement on the same pooled features."""
    from m3d.config import synthetic_mrcnn_config
    from m3d.heads import MaskRCNN
    from m3d.model import compose_image_meta, synthetic_volume
    cfg = synthetic_mrcnn_config(64, depth=16, PRE_NMS_LIMIT=3000, POST_NMS_ROIS_INFERENCE=64,
                                 DETECTION_MIN_CONFIDENCE=0.0, DETECTION_MAX_INSTANCES=8)
    model = MaskRCNN(cfg, device=cuda, seed=2)
    meta = compose_image_meta(0, [64, 64, 16, 1], [64, 64, 16, 1], [0, 0, 0, 64, 64, 16], 1.0, [0, 1])
    out = model.detect(synthetic_volume(64, 16).to(cuda), torch.from_numpy(meta[None]).to(cuda))
    torch.cuda.synchronize()
    det = out["detections"].cpu().numpy()[0]
    assert out["mrcnn_mask"].shape == (1, 8, 28, 28, 28, 2)
    assert np.isfinite(det).all() and (det[:, 7] > 0).sum() >= 1
    p = model.store.state_dict()
    rl, rp, rb = HR.classifier_head(p, out["pooled"].cpu(), 2)
    assert rel_err(out["mrcnn_class"], rp) < 1e-4
    assert rel_err(out["mrcnn_bbox"], rb) < 1e-4
    rm = HR.mask_head(p, out["mask_pooled"].cpu(), 2)
    assert rel_err(out["mrcnn_mask"], rm) < 1e-4
