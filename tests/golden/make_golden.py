"""Generate the committed golden fixtures (tests/golden/*.npz) from the oracle.

The reference cannot be executed here (running reference code
was denied; TF 2.2 / cp36 absent) and ships no golden vectors, so these
fixtures are produced by the CPU restatement in oracle/ (itself pinned by the
known-answer tests of tests/test_oracle.py).  They freeze seeded inputs AND
outputs so the GPU parity tests and the oracle regression test compare
against data, not against code run at test time.

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import ops_ref as R  # noqa: E402


def rand_boxes(rng, n, lo=-0.15, hi=1.15, min_size=0.02, max_size=0.6):
    a = rng.uniform(lo, hi - max_size, (n, 3))
    s = rng.uniform(min_size, max_size, (n, 3))
    return np.concatenate([a, a + s], 1).astype(np.float32)


def crop():
    rng = np.random.default_rng(100)
    img = rng.normal(size=(2, 12, 10, 9, 8)).astype(np.float32)
    boxes = rand_boxes(rng, 16)
    boxes[3] = [0.0, 0.0, 0.0, 1.0, 1.0, 1.0]           # whole image
    boxes[4] = [0.25, 0.5, 0.125, 0.75, 0.5, 0.875]      # zero extent in x
    bi = rng.integers(0, 2, 16).astype(np.int32)
    tri = R.crop_and_resize_3d(img, boxes, bi, (5, 4, 3), "trilinear", -1.5)
    near = R.crop_and_resize_3d(img, boxes, bi, (5, 4, 3), "nearest", -1.5)
    one = R.crop_and_resize_3d(img, boxes, bi, (1, 3, 1), "trilinear", 0.0)
    g = rng.normal(size=tri.shape).astype(np.float32)
    gi_tri = R.crop_and_resize_3d_grad_image(g, boxes, bi, img.shape, "trilinear")
    gi_near = R.crop_and_resize_3d_grad_image(g, boxes, bi, img.shape, "nearest")
    gb = R.crop_and_resize_3d_grad_boxes(g, img, boxes, bi)
    np.savez_compressed(os.path.join(HERE, "crop.npz"), image=img, boxes=boxes, box_ind=bi,
                        crops_trilinear=tri, crops_nearest=near, crops_one=one, grads=g,
                        grad_image_trilinear=gi_tri, grad_image_nearest=gi_near, grad_boxes=gb)


def nms():
    rng = np.random.default_rng(101)
    n = 3000
    lo = rng.uniform(0, 0.9, (n, 3)).astype(np.float32)
    sz = rng.uniform(0.01, 0.25, (n, 3)).astype(np.float32)
    boxes = np.concatenate([lo, lo + sz], 1).astype(np.float32)
    scores = np.round(rng.uniform(size=n), 2).astype(np.float32)     # heavy ties
    scores[::97] = -np.inf
    keep = R.non_max_suppression_3d(boxes, scores, 1500, 0.3)
    # tie-heavy: 200 copies of 20 distinct boxes, equal scores
    base = np.concatenate([lo[:20], lo[:20] + 0.1], 1).astype(np.float32)
    tboxes = np.tile(base, (10, 1))
    tscores = np.full(200, 0.5, np.float32)
    tkeep = R.non_max_suppression_3d(tboxes, tscores, 200, 0.5)
    # 2-D mode (DetectionLayer uses tf.image.non_max_suppression on (y1,x1,y2,x2))
    b2 = boxes[:, [0, 1, 3, 4]].copy()
    keep2d = R.non_max_suppression_3d(b2, scores, 800, 0.45, mode="2d")
    np.savez_compressed(os.path.join(HERE, "nms.npz"), boxes=boxes, scores=scores, keep=keep,
                        thr=np.float32(0.3), max_out=np.int32(1500), tie_boxes=tboxes,
                        tie_scores=tscores, tie_keep=tkeep, boxes2d=b2, keep2d=keep2d)


def pyramid():
    rng = np.random.default_rng(102)
    C = 8
    maps = [rng.normal(size=(2, s, s, 16, C)).astype(np.float32) for s in (16, 8, 4, 2)]
    boxes = np.stack([rand_boxes(rng, 20, lo=-0.05, hi=1.05, min_size=0.005, max_size=0.9)
                      for _ in range(2)])
    meta = np.zeros((2, 18), np.float32)
    meta[:, 5:8] = [512, 512, 256]         # image shape drives the level (levels 2..5 reachable)
    out7 = R.pyramid_roi_align(boxes, meta, maps, (7, 7, 7))
    out3 = R.pyramid_roi_align(boxes, meta, maps, (3, 3, 3))
    lv = np.stack([R.roi_prepare(boxes[b], meta[b, 5:8])[1] for b in range(2)])
    np.savez_compressed(os.path.join(HERE, "pyramid.npz"), p2=maps[0], p3=maps[1], p4=maps[2],
                        p5=maps[3], boxes=boxes, meta=meta, out7=out7, out3=out3, levels=lv)


def proposal():
    rng = np.random.default_rng(103)
    A = 4000
    logits = rng.normal(size=(A, 2)).astype(np.float32)
    logits[::7] = logits[::7].round(1)                      # score ties
    e = np.exp(logits - logits.max(1, keepdims=True))
    probs = (e / e.sum(1, keepdims=True)).astype(np.float32)
    deltas = rng.normal(0, 1.0, (A, 6)).astype(np.float32)
    anchors = rand_boxes(rng, A, lo=0.0, hi=1.0, min_size=0.05, max_size=0.4)
    std = np.array([0.1, 0.1, 0.1, 0.213, 0.21, 0.15], np.float32)
    boxes, s, order = R.proposal_decode(probs, deltas, anchors, 1500, std, 32)
    keep = R.non_max_suppression_3d(boxes, s, 300, 0.7)
    props = R.proposal_layer(probs[None], deltas[None], anchors[None], 300, 0.7, 1500, std, 32)
    np.savez_compressed(os.path.join(HERE, "proposal.npz"), probs=probs, deltas=deltas,
                        anchors=anchors, std=std, order=order.astype(np.int64), boxes=boxes,
                        scores=s, keep=keep, proposals=props[0])


if __name__ == "__main__":
    crop()
    nms()
    pyramid()
    proposal()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
