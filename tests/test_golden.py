"""The oracle reproduces the committed golden fixtures exactly (regression pin)."""
import os

import numpy as np

from oracle import ops_ref as R

G = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    return np.load(os.path.join(G, name))


def test_crop_fixture():
    f = load("crop.npz")
    np.testing.assert_array_equal(
        R.crop_and_resize_3d(f["image"], f["boxes"], f["box_ind"], (5, 4, 3), "trilinear", -1.5),
        f["crops_trilinear"])
    np.testing.assert_array_equal(
        R.crop_and_resize_3d(f["image"], f["boxes"], f["box_ind"], (5, 4, 3), "nearest", -1.5),
        f["crops_nearest"])
    np.testing.assert_array_equal(
        R.crop_and_resize_3d_grad_image(f["grads"], f["boxes"], f["box_ind"], f["image"].shape),
        f["grad_image_trilinear"])


def test_nms_fixture():
    f = load("nms.npz")
    np.testing.assert_array_equal(
        R.non_max_suppression_3d(f["boxes"], f["scores"], int(f["max_out"]), float(f["thr"])), f["keep"])
    np.testing.assert_array_equal(R.non_max_suppression_3d(f["tie_boxes"], f["tie_scores"], 200, 0.5),
                                  f["tie_keep"])
    assert list(f["tie_keep"]) == list(range(20))       # first copy of each distinct box
    np.testing.assert_array_equal(
        R.non_max_suppression_3d(f["boxes2d"], f["scores"], 800, 0.45, mode="2d"), f["keep2d"])


def test_pyramid_fixture():
    f = load("pyramid.npz")
    maps = [f[k] for k in ("p2", "p3", "p4", "p5")]
    np.testing.assert_array_equal(R.pyramid_roi_align(f["boxes"], f["meta"], maps, (7, 7, 7)), f["out7"])
    assert set(np.unique(f["levels"])) == {2, 3, 4, 5}


def test_proposal_fixture():
    f = load("proposal.npz")
    out = R.proposal_layer(f["probs"][None], f["deltas"][None], f["anchors"][None], 300, 0.7, 1500,
                           f["std"], 32)
    np.testing.assert_array_equal(out[0], f["proposals"])
