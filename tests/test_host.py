"""Host-side logic: config surface, anchors, TF padding arithmetic."""
import json

import numpy as np
import pytest

from m3d import anchors as A
from m3d import config as C
from m3d.nn import conv_geom, same_out_pad

RATS_RPN = {  # values of configs/rpn/scp_rpn_rats.json (reference preset)
    "NUM_CLASSES": 2, "CLASS_NAMES": ["neuron"], "IMAGE_SIZE": 256, "IMAGE_DEPTH": 12,
    "IMAGE_CHANNEL_COUNT": 1, "MAX_GT_INSTANCES": 6, "USE_MINI_MASK": False,
    "RPN_ANCHOR_SCALES": [25, 57, 84, 109, 135], "RPN_ANCHOR_RATIOS": [0.05, 0.06, 0.15],
    "RPN_ANCHOR_STRIDE": 1, "RPN_BBOX_STD_DEV": [0.1, 0.1, 0.1, 0.213, 0.21, 0.15],
    "RPN_NMS_THRESHOLD": 0.7, "MODE": "training",
    "BACKBONE_STRIDES": [[4, 4, 1], [8, 8, 1], [16, 16, 1], [32, 32, 1], [64, 64, 1]],
    "BACKBONE": "resnet50", "TOP_DOWN_PYRAMID_SIZE": 256, "RPN_TRAIN_ANCHORS_PER_IMAGE": 1536,
    "PRE_NMS_LIMIT": 15000, "POST_NMS_ROIS_TRAINING": 6000, "POST_NMS_ROIS_INFERENCE": 8000,
    "IMAGES_PER_GPU": 2, "GPU_COUNT": 1, "LOSS_WEIGHTS": {"rpn_class_loss": 3, "rpn_bbox_loss": 2},
    "OPTIMIZER": {"name": "SGD", "parameters": {"learning_rate": 0.0002, "momentum": 0.9,
                                                "clipnorm": 5.0, "decay": 1e-4}},
    "WEIGHT_DECAY": 0.0005, "EPOCHS": 60,
}


def test_config_accepts_reference_keys_and_derives_fields(tmp_path):
    p = tmp_path / "c.json"
    p.write_text(json.dumps(RATS_RPN))
    cfg = C.load_config(str(p))
    assert list(cfg.IMAGE_SHAPE) == [256, 256, 12, 1]
    assert cfg.BATCH_SIZE == 2 and cfg.IMAGE_META_SIZE == 18
    assert cfg.ANCHOR_NB == 256 * 256 * 12 // 16 + 256 * 256 * 12 // 64 + 256 * 256 * 12 // 256 + \
        256 * 256 * 12 // 1024 + 256 * 256 * 12 // 4096


def test_config_rejects_unknown_keys():
    with pytest.raises(TypeError):
        C.Config(NOT_A_KEY=1)


def test_anchor_count_matches_survey():
    for S, A_expected in ((128, 523776), (256, 4190208)):
        cfg = C.synthetic_rpn_config(S)
        a = A.get_anchors(cfg)
        assert a.shape == (A_expected, 6) and a.dtype == np.float32
        assert a.min() >= 0 and a.max() <= 1


def test_anchor_order_is_y_x_z_anchor():
    cfg = C.synthetic_rpn_config(128)
    a = A.get_anchors(cfg)
    # first level P2 stride 4: anchors of cell (y=0,x=0,z=1) follow the 3 of cell (0,0,0)
    cz = (a[3:6, 2] + a[3:6, 5]) / 2 * 128
    assert np.all(cz > (a[0:3, 2] + a[0:3, 5]) / 2 * 128)
    assert np.allclose(a[0:3, 3] - a[0:3, 0], a[0, 3] - a[0, 0])


def test_tf_same_padding_is_asymmetric():
    assert same_out_pad(64, 3, 2) == (32, 0)      # total pad 1 -> all after
    assert same_out_pad(128, 3, 1) == (128, 1)
    g = conv_geom((128, 128, 128), (7, 7, 7), (2, 2, 1), 3)  # ZeroPadding3D(3) + valid
    assert g.out == (64, 64, 128) and g.pad == (3, 3, 3)


@pytest.mark.parametrize("order", ["sc_first", "a_first"])
def test_gradlink_dx2_protocol_sums_once(order):
    """GradLink 'dx2' (conv block: shortcut and conv 2a read the same x): the
    first backward parks its gradient and returns none, the second takes the
    parked buffer with accumulate=1 and returns it -- in either order."""
    import torch
    from m3d.nn import GradLink, _link_park, _link_take
    x = torch.zeros(2, 3)
    link = GradLink("dx2")
    g_first, g_second = torch.full((2, 3), 1.0), torch.full((2, 3), 2.0)
    buf, acc = _link_take(link, x)
    assert buf is None and acc == 0
    assert _link_park(link, g_first, acc) is None and link.buf is g_first
    buf, acc = _link_take(link, x)
    assert buf is g_first and acc == 1 and link.buf is None
    buf += g_second                       # what the bwd-data kernel does with accumulate=1
    out = _link_park(link, buf, acc)
    assert out is g_first and torch.equal(out, torch.full((2, 3), 3.0)) and link.buf is None


def test_gradlink_res_mode_never_parks_data_gradients():
    """GradLink 'res' (identity block): only the residual conv parks (dres);
    data gradients pass through, the input conv consumes the parked dres."""
    import torch
    from m3d.nn import GradLink, _link_park, _link_take
    x = torch.zeros(4)
    link = GradLink("res")
    dx = torch.ones(4)
    assert _link_park(link, dx, 0) is dx and link.buf is None
    link.buf = torch.full((4,), 5.0)      # conv 2c's backward parks dres
    buf, acc = _link_take(link, torch.zeros(3))
    assert buf is None and acc == 0       # shape mismatch: not this tensor's gradient
    buf, acc = _link_take(link, x)
    assert acc == 1 and torch.equal(buf, torch.full((4,), 5.0)) and link.buf is None


@pytest.mark.parametrize("shape,stride", [((1, 12, 10, 9, 1), (2, 2, 1)), ((2, 9, 8, 16, 1), (1, 1, 1))])
def test_stem_zwindow_form_is_the_same_conv(shape, stride):
    """The stem's window form (x64 = the 8x8 (x, z) windows of x as channels,
    w64 = the kw x kd taps zero-padded to 8 x 8, a (kh, 1, 1) conv) equals the
    7^3 conv (float64)."""
    import torch
    from m3d.nn import _stem_zwindow, conv_geom
    g = torch.Generator().manual_seed(0)
    x = torch.randn(shape, generator=g)
    w = torch.randn((7, 7, 7, 1, 5), generator=g)
    geo = conv_geom(shape[1:4], (7, 7, 7), stride, 3)
    x8, w8, g8 = _stem_zwindow(x, w, geo)
    assert x8.shape[-1] == 64 and g8.k == (7, 1, 1) and g8.out == geo.out

    def conv(xc, wc, gg):   # channels-last [B,H,W,D,C] with pad-before; crop to gg.out
        xt = torch.nn.functional.pad(xc.permute(0, 4, 1, 2, 3).double(),
                                     (gg.pad[2], 16, gg.pad[1], 16, gg.pad[0], 16))
        y = torch.nn.functional.conv3d(xt, wc.permute(4, 3, 0, 1, 2).double(), stride=gg.stride)
        return y[:, :, :gg.out[0], :gg.out[1], :gg.out[2]]
    torch.testing.assert_close(conv(x8, w8, g8), conv(x, w, geo), rtol=0, atol=1e-12)
