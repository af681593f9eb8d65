"""Parity at BASELINE.json configs[3]'s own shape: full Mask R-CNN inference on
a 256^3 volume with 512 proposals (MaskRCNN.build, MODE "inference",
core/models.py:5473-5754), every stage checked against the CPU oracle on the
GPU's own inputs, as tests/test_gpu_configs.py does for configs[1] / [2]:

  ProposalLayer(POST_NMS_ROIS_INFERENCE=512)   core/models.py:5555-5567
      top-k order / scores / decoded boxes bit-exact, NMS keep bit-exact
      (on the GPU's and on the oracle's own decode)
  PyramidROIAlign 7^3 on P2..P5 of the 256^3 maps     5697-5700   bit-exact
  fpn_classifier_graph                        5703-5709   1e-4 of scale (fp64)
  DetectionLayer (2-D NMS)                    5712-5720   kept set + order identical
  PyramidROIAlign 14^3 on the detections      5725-5728   bit-exact
  build_fpn_mask_graph                        5730-5735   1e-4 of scale (fp64)

DETECTION_MIN_CONFIDENCE is 0 so the random-init heads still yield detections
(the 2-D NMS at 0.3 keeps a few tens of the 512; the 14^3 ROIAlign and the mask
head run on all DETECTION_MAX_INSTANCES = 40 rows, zero padding included);
every shape is configs[3]'s.  The reference's inference
anchors are a model input (core/models.py:5510); the RPN training anchor set
of m3d.anchors is used for both sides here."""
import time

import numpy as np
import pytest
import torch

from oracle import heads_ref as HR
from oracle import ops_ref as R

pytestmark = pytest.mark.gpu
S = 256


def rel_err(got, ref):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(ref).detach().double().cpu()
    return float((got - ref).abs().max()) / (float(ref.abs().max()) + 1e-30)


def _log(*a):
    print(f"[configs3 {time.strftime('%H:%M:%S')}]", *a, flush=True)


@pytest.fixture(scope="module")
def infer256(cuda):
    from m3d.config import synthetic_mrcnn_config
    from m3d.heads import MaskRCNN
    from m3d.model import compose_image_meta, synthetic_volume
    cfg = synthetic_mrcnn_config(S, DETECTION_MIN_CONFIDENCE=0.0)
    assert cfg.POST_NMS_ROIS_INFERENCE == 512 and cfg.IMAGE_SHAPE[:3].tolist() == [S, S, S]
    model = MaskRCNN(cfg, device=cuda, seed=4)
    meta = compose_image_meta(0, [S, S, S, 1], [S, S, S, 1], [0, 0, 0, S, S, S], 1.0, [0, 1])[None]
    image = synthetic_volume(S, seed=0)
    out = model.detect(image.to(cuda), torch.from_numpy(meta).to(cuda))
    torch.cuda.synchronize()
    host = {k: (v.cpu().numpy() if torch.is_tensor(v) else [m.cpu().numpy() for m in v[:4]])
            for k, v in out.items()}
    _log("256^3 detect done; rpn_rois nonzero", int((np.abs(host["rpn_rois"][0]).sum(1) > 0).sum()))
    torch.set_num_threads(min(16, max(1, torch.get_num_threads())))
    return cfg, model, meta, out, host


@pytest.mark.timeout(900)
def test_config3_forward_vs_oracle(infer256):
    """The 256^3 backbone + FPN + RPN head forward (MaskRCNN.build,
    core/models.py:5473-5553; the same graph as RPN.build 3162-3263) against
    the CPU fp32 restatement (oracle/model_ref.RefRPN) under no_grad: P2..P6,
    rpn_class and rpn_bbox within 1e-4 of each tensor's scale, as configs[1]
    at 128^3.  This covers the 256^3-only workspace paths of the forward (per-
    level Winograd workspaces past M3D_SHARE_WINO_MAX_GB, 4 GiB operand bound)."""
    from oracle import model_ref as MR
    cfg, model, meta, out, host = infer256
    from m3d.model import synthetic_volume
    image = synthetic_volume(S, seed=0)
    t0 = time.time()
    with torch.no_grad():
        ref = MR.RefRPN(model.store.state_dict(), dtype=torch.float32).forward(image)
    _log(f"CPU fp32 256^3 forward {time.time() - t0:.1f} s")
    errs = {}
    for i, b in enumerate(ref["feature_maps"]):
        a = out["feature_maps"][i]
        errs[f"P{i + 2}"] = rel_err(a, b)
    errs["probs"] = rel_err(out["rpn_class"], ref["rpn_class"])
    errs["bbox"] = rel_err(out["rpn_bbox"], ref["rpn_bbox"])
    del ref
    _log("256^3 forward rel err", errs)
    for k, e in errs.items():
        assert e < 1e-4, (k, e)


def test_config3_proposal_layer(infer256):
    from m3d import ops
    cfg, model, meta, out, host = infer256
    probs = out["rpn_class"][0].contiguous()
    deltas = out["rpn_bbox"][0].contiguous()
    anchors = model.anchors[0]
    A = anchors.shape[0]
    assert A == 4190208 and probs.shape == (A, 2)
    k = min(cfg.PRE_NMS_LIMIT, A)
    order = ops.topk_order(probs, k)
    boxes, scores = ops.proposal_decode(probs, deltas, anchors, order, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)
    rb, rs, ridx = R.proposal_decode(host["rpn_class"][0], host["rpn_bbox"][0], anchors.cpu().numpy(),
                                     cfg.PRE_NMS_LIMIT, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)
    np.testing.assert_array_equal(order.cpu().numpy(), ridx)
    np.testing.assert_array_equal(scores.cpu().numpy(), rs)
    bg = boxes.cpu().numpy()
    np.testing.assert_array_equal(bg, rb)
    want = R.non_max_suppression_3d(bg, rs, cfg.POST_NMS_ROIS_INFERENCE, cfg.RPN_NMS_THRESHOLD)
    np.testing.assert_array_equal(R.non_max_suppression_3d(rb, rs, cfg.POST_NMS_ROIS_INFERENCE,
                                                           cfg.RPN_NMS_THRESHOLD), want)
    keep = ops.non_max_suppression_3d(boxes, scores, cfg.POST_NMS_ROIS_INFERENCE, cfg.RPN_NMS_THRESHOLD)
    np.testing.assert_array_equal(keep.cpu().numpy(), want)
    rois = host["rpn_rois"][0]
    assert rois.shape == (512, 6)
    np.testing.assert_array_equal(rois[:len(want)], bg[want])
    assert not rois[len(want):].any()
    _log(f"ProposalLayer: {len(want)} kept of {k} (A = {A})")


def test_config3_roi_align_7_and_classifier(infer256):
    cfg, model, meta, out, host = infer256
    maps = host["feature_maps"]
    assert maps[0].shape == (1, S // 4, S // 4, S, 256)
    want = R.pyramid_roi_align(host["rpn_rois"], meta, maps, (7, 7, 7))
    assert host["pooled"].shape == (1, 512, 7, 7, 7, 256)
    np.testing.assert_array_equal(host["pooled"], want)
    _, lvl = R.roi_prepare(host["rpn_rois"][0], meta[0, 5:8])
    _log("ROIAlign 7^3 bit-exact; levels", np.bincount(lvl, minlength=6)[2:].tolist())
    rl, rp, rb = HR.classifier_head(model.store.state_dict(), host["pooled"], cfg.NUM_CLASSES)
    e = (rel_err(out["mrcnn_class"], rp), rel_err(out["mrcnn_bbox"], rb))
    _log("classifier rel err (probs, bbox)", e)
    assert max(e) < 1e-4, e


def test_config3_detection_layer(infer256):
    cfg, model, meta, out, host = infer256
    det = host["detections"][0]
    ref, kept = HR.refine_detections(host["rpn_rois"][0], host["mrcnn_class"][0], host["mrcnn_bbox"][0],
                                     meta[0], cfg.BBOX_STD_DEV, float(cfg.DETECTION_MIN_CONFIDENCE),
                                     float(cfg.DETECTION_NMS_THRESHOLD), int(cfg.DETECTION_MAX_INSTANCES))
    n = len(kept)
    _log(f"DetectionLayer: {n} detections")
    assert 0 < n <= int(cfg.DETECTION_MAX_INSTANCES) and int((det[:, 7] > 0).sum()) == n
    assert np.array_equal(det[:n, 7], ref[:n, 7]), "kept detections / order differ"
    np.testing.assert_allclose(det[:n, :6], ref[:n, :6], rtol=0, atol=2e-6)
    assert np.all(det[n:] == 0) and np.all(det[:n, 6] == 1.0)


def test_config3_roi_align_14_and_mask_head(infer256):
    cfg, model, meta, out, host = infer256
    boxes = np.ascontiguousarray(host["detections"][:, :, :6])
    want = R.pyramid_roi_align(boxes, meta, host["feature_maps"], (14, 14, 14))
    assert host["mask_pooled"].shape == (1, int(cfg.DETECTION_MAX_INSTANCES), 14, 14, 14, 256)
    np.testing.assert_array_equal(host["mask_pooled"], want)
    _log("ROIAlign 14^3 bit-exact")
    rm = HR.mask_head(model.store.state_dict(), host["mask_pooled"], cfg.NUM_CLASSES)
    assert out["mrcnn_mask"].shape == (1, int(cfg.DETECTION_MAX_INSTANCES), 28, 28, 28, 2)
    e = rel_err(out["mrcnn_mask"], rm)
    _log("mask head rel err", e)
    assert e < 1e-4, e
