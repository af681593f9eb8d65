"""The reference's own presets on the GPU path, and the ProposalLayer's
fail-loudly contract.

scp_rpn_hela.json strides depth by 2 in BACKBONE_STRIDES; RPN.train patches
that to 1 (core/models.py:3408-3419) but only after build() made the anchors,
so the reference's graph gathers past its anchor constant.  m3d applies the
patch before the anchors (m3d.anchors.model_anchors): the RPN built from the
preset must give one anchor per RPN row and proposals decoded from in-range
anchors.  A mismatched anchor tensor, or an out-of-range top-k index through
the C-ABI, raises instead of reading past the buffer."""
import json
import os
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fields(name):
    with open(os.path.join(os.path.dirname(__file__), "golden", "ref_presets.json")) as f:
        return json.load(f)[name]


def test_rpn_from_hela_preset_is_consistent(cuda):
    from m3d.config import Config
    from m3d.model import RPN, synthetic_volume
    from oracle import ops_ref as R
    cfg = Config(**_fields("rpn/scp_rpn_hela.json"))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        model = RPN(cfg, device=cuda, seed=3)
    assert any("RPN.train" in str(x.message) for x in w)
    H, W, D = (int(v) for v in cfg.IMAGE_SHAPE[:3])
    image = synthetic_volume(H, D, seed=1).to(cuda)
    with torch.no_grad():
        out = model.forward(image, proposals=True)
    torch.cuda.synchronize()
    A = model.anchors.shape[1]
    assert out["rpn_class"].shape[1] == A == out["rpn_bbox"].shape[1]
    rois = out["rpn_rois"][0].cpu().numpy()
    ref = R.proposal_layer(out["rpn_class"].cpu().numpy(), out["rpn_bbox"].cpu().numpy(),
                           model.anchors.cpu().numpy(), cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD,
                           cfg.PRE_NMS_LIMIT, cfg.RPN_BBOX_STD_DEV, cfg.IMAGE_DEPTH)[0]
    np.testing.assert_array_equal(rois, ref)
    assert np.isfinite(rois).all() and rois.min() >= 0 and rois.max() <= 1


def test_proposal_layer_rejects_anchor_mismatch(cuda):
    from m3d.layers import ProposalLayer
    layer = ProposalLayer(100, 0.7, 500, 1, [0.1] * 6, 16)
    probs = torch.rand((1, 1000, 2), device=cuda)
    deltas = torch.zeros((1, 1000, 6), device=cuda)
    anchors = torch.rand((1, 900, 6), device=cuda)
    with pytest.raises(ValueError, match="must be equal"):
        layer([probs, deltas, anchors])


def test_decode_out_of_range_index_raises(cuda):
    """An order index >= A through m3d_proposal_decode: never read, the row is
    written empty with score -FLT_MAX, the device flag raises ValueError."""
    from m3d import _lib, ops
    A = 512
    probs = torch.rand((A, 2), device=cuda)
    deltas = torch.zeros((A, 6), device=cuda)
    anchors = torch.rand((A, 6), device=cuda).sort(dim=1).values
    order = torch.tensor([3, 7, A + 5, 11], device=cuda, dtype=torch.int64)
    with pytest.raises(ValueError, match="not in"):
        ops.proposal_decode(probs, deltas, anchors, order, [0.1] * 6, 16)
    # the raw C-ABI: in-range rows decoded, the bad row zero with score -FLT_MAX
    L = _lib.load()
    boxes = torch.full((4, 6), 7.0, device=cuda)
    scores = torch.zeros(4, device=cuda)
    err = torch.zeros(1, device=cuda, dtype=torch.int32)
    sd = (_lib.c_f * 6)(*([0.1] * 6))
    assert L.m3d_proposal_decode(_lib.ptr(probs), _lib.ptr(deltas), _lib.ptr(anchors), A, _lib.ptr(order), 4,
                                 sd, 16.0, _lib.ptr(boxes), _lib.ptr(scores), _lib.ptr(err), _lib.stream()) == 0
    torch.cuda.synchronize()
    assert int(err.item()) == 1
    assert float(scores[2]) == -np.finfo(np.float32).max and not boxes[2].any()
    assert torch.equal(scores[[0, 1, 3]], probs[[3, 7, 11], 1])
    # more indices than anchors is an argument error (M3D_EINVAL)
    big = torch.zeros(A + 1, device=cuda, dtype=torch.int64)
    assert L.m3d_proposal_decode(_lib.ptr(probs), _lib.ptr(deltas), _lib.ptr(anchors), A, _lib.ptr(big), A + 1,
                                 sd, 16.0, _lib.ptr(boxes), _lib.ptr(scores), None, _lib.stream()) == -1
