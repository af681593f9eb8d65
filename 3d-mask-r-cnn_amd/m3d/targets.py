"""Training-target layers on the GPU.

``DetectionTargetLayer(config, train_rois_per_image, roi_positive_ratio,
bbox_std_dev, use_mini_mask, mask_shape, images_per_gpu,
positive_iou_threshold, negative_iou_threshold)([proposals, gt_class_ids,
gt_boxes, gt_masks])`` -> [rois, target_gt_boxes, target_class_ids,
target_bbox, target_mask] (core/models.py:1043-1118 / detection_targets_graph
736-1040): sampling, box refinement and mask targets run as two libm3d
launches per image (m3d_detection_targets + m3d_mask_targets3d), sizes fixed
by TRAIN_ROIS_PER_IMAGE, nothing returns to the host.  When ``config`` is
given, the IoU thresholds come from RPN_POSITIVE_IOU / RPN_NEGATIVE_IOU as in
the reference.  The reference's tf.random.shuffle becomes a seeded random
order (``seed`` advances per call), so runs are reproducible.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib, ops
from ._lib import check, ptr, stream


class DetectionTargetLayer:
    def __init__(self, config, train_rois_per_image, roi_positive_ratio, bbox_std_dev, use_mini_mask,
                 mask_shape, images_per_gpu, positive_iou_threshold=0.5, negative_iou_threshold=0.1,
                 seed=0, name="proposal_targets", **kwargs):
        self.config = config
        self.T = int(train_rois_per_image)
        self.ratio = float(roi_positive_ratio)
        self.std = [float(np.float32(v)) for v in bbox_std_dev]
        self.use_mini_mask = bool(use_mini_mask)
        self.mask_shape = tuple(int(v) for v in mask_shape)
        self.images_per_gpu = int(images_per_gpu)
        self.pos_thr = float(positive_iou_threshold)
        self.neg_thr = float(negative_iou_threshold)
        if config is not None:            # detection_targets_graph(config=...) overrides (core/models.py:750-758)
            self.T = int(getattr(config, "TRAIN_ROIS_PER_IMAGE", 256))
            self.ratio = float(getattr(config, "ROI_POSITIVE_RATIO", 0.5))
            self.std = [float(np.float32(v)) for v in getattr(config, "BBOX_STD_DEV", self.std)]
            self.use_mini_mask = bool(getattr(config, "USE_MINI_MASK", True))
            self.mask_shape = tuple(int(v) for v in getattr(config, "MASK_SHAPE", (28, 28, 28)))
            self.pos_thr = float(getattr(config, "RPN_POSITIVE_IOU", 0.25))
            self.neg_thr = float(getattr(config, "RPN_NEGATIVE_IOU", 0.15))
        self.seed = int(seed)
        self.name = name

    def __call__(self, inputs, seed=None):
        proposals, gt_class_ids, gt_boxes, gt_masks = inputs
        ops._dev(proposals, gt_class_ids, gt_boxes, gt_masks)
        L = _lib.load()
        B, N = proposals.shape[:2]
        G = gt_boxes.shape[1]
        T = self.T
        dev = proposals.device
        mh, mw, md = self.mask_shape
        out = {k: torch.zeros((B, T, 6), device=dev) for k in ("rois", "gt", "deltas", "mask_boxes")}
        cls = torch.zeros((B, T), device=dev, dtype=torch.int32)
        assign = torch.empty((B, T), device=dev, dtype=torch.int32)
        counts = torch.zeros((B, 2), device=dev, dtype=torch.int32)
        masks = torch.empty((B, T, mh, mw, md), device=dev)
        wsb = int(L.m3d_detection_targets_workspace_bytes(N))
        ws = torch.empty(max(wsb // 4, 1), device=dev, dtype=torch.int32)
        sd = (_lib.c_f * 6)(*self.std)
        s0 = self.seed if seed is None else int(seed)
        for b in range(B):
            p = proposals[b].detach().float().contiguous()
            gc = gt_class_ids[b].to(torch.int32).contiguous()
            gb = gt_boxes[b].detach().float().contiguous()
            check(L.m3d_detection_targets(ptr(p), N, ptr(gc), ptr(gb), G, T, self.ratio, self.pos_thr,
                                          self.neg_thr, sd, 1 if self.use_mini_mask else 0,
                                          (s0 * 1000003 + b) & 0xFFFFFFFF, out["rois"][b].data_ptr(),
                                          out["gt"][b].data_ptr(), cls[b].data_ptr(), out["deltas"][b].data_ptr(),
                                          out["mask_boxes"][b].data_ptr(), assign[b].data_ptr(),
                                          counts[b].data_ptr(), ptr(ws), wsb, stream()), "detection_targets")
            m = gt_masks[b]
            H, W, D, Gm = m.shape
            mu8 = m.to(torch.uint8).contiguous()
            check(L.m3d_mask_targets3d(ptr(mu8), H, W, D, Gm, out["mask_boxes"][b].data_ptr(),
                                       assign[b].data_ptr(), T, mh, mw, md, masks[b].data_ptr(), stream()),
                  "mask_targets3d")
        if seed is None:
            self.seed += 1
        self.last_counts = counts
        return [out["rois"], out["gt"], cls, out["deltas"], masks]

    def compute_output_shape(self, input_shape):
        return [(None, self.T, 6), (None, self.T, 6), (None, self.T), (None, self.T, 6),
                (None, self.T) + self.mask_shape]


def build_rpn_targets(anchors, gt_class_ids, gt_boxes, config, seed=0, list_cap=None):
    """build_rpn_targets(anchors, gt_class_ids, gt_boxes, config)
    (core/data_generators.py:2031-2178) on the GPU.

    anchors: device tensor [A,6], normalised (RPN.get_anchors); gt_boxes: [G,6]
    pixel or normalised (the reference's auto-detection: GT with max > 2 are
    divided by (H,W,D,H,W,D) and clipped to [0,1]).  Returns (rpn_match [A]
    int32, rpn_bbox [RPN_TRAIN_ANCHORS_PER_IMAGE, 6] float32), device tensors.
    The dropped negatives are a seeded random subset (np.random.choice in the
    reference)."""
    L = _lib.load()
    ops._dev(anchors)
    dev = anchors.device
    A = anchors.shape[0]
    total = int(getattr(config, "RPN_TRAIN_ANCHORS_PER_IMAGE", 2048))
    gt = np.asarray(gt_boxes, np.float32).reshape(-1, 6)
    G = gt.shape[0]
    if G and float(np.max(np.abs(gt))) > 2.0:           # anchors are normalised: normalise the GT
        H = int(getattr(config, "IMAGE_SIZE", config.IMAGE_SHAPE[0]))
        W = int(getattr(config, "IMAGE_SIZE", config.IMAGE_SHAPE[1]))
        D = int(getattr(config, "IMAGE_DEPTH", config.IMAGE_SHAPE[2]))
        gt = np.clip(gt / np.array([H, W, D, H, W, D], np.float32), 0.0, 1.0).astype(np.float32)
    gtd = torch.from_numpy(np.ascontiguousarray(gt)).to(dev)
    match8 = torch.empty((A,), device=dev, dtype=torch.int8)
    bbox = torch.empty((total, 6), device=dev, dtype=torch.float32)
    cap = int(list_cap or A)                          # a GT's IoU > 0 list never exceeds A
    wsb = int(L.m3d_rpn_targets_workspace_bytes(A, G, cap))
    ws = torch.empty(max(wsb, 1), device=dev, dtype=torch.uint8)
    sd = (_lib.c_f * 6)(*[float(np.float32(v)) for v in config.RPN_BBOX_STD_DEV])
    cnt = (ctypes.c_int32 * 2)()
    check(L.m3d_rpn_targets(ptr(anchors.contiguous()), A, ptr(gtd), G,
                            float(getattr(config, "RPN_POSITIVE_IOU", 0.15)),
                            float(getattr(config, "RPN_NEGATIVE_IOU", 0.05)), total,
                            float(getattr(config, "RPN_POSITIVE_RATIO", 0.5)),
                            int(getattr(config, "ATSS_TOPK", 24)), int(getattr(config, "ATSS_MIN_POS_PER_GT", 4)),
                            sd, int(seed) & 0xFFFFFFFF, ptr(match8), ptr(bbox), cap, ptr(ws), wsb, cnt,
                            stream()), "rpn_targets")
    return match8.to(torch.int32), bbox


class RPNTargetBuilder:
    """``build_rpn_targets`` inside the training step: the same ATSS labels,
    balancing and deltas as :func:`build_rpn_targets`
    (core/data_generators.py:2031-2178, called per volume at :986), through
    the stream-ordered ``m3d_rpn_targets_async`` -- no host round trip, so the
    GPU builds each step's targets right before its forward.  Workspace and
    outputs are allocated once for the anchor set and reused.

    builder(gt_boxes, seed) with gt_boxes a normalised [G,6] DEVICE tensor
    returns m3d.model.DeviceRPNTargets (rpn_match int8 [A], rpn_bbox
    [RPN_TRAIN_ANCHORS_PER_IMAGE, 6]); ``counts`` (device int32[3]) holds the
    last call's positives, negatives and list-overflow flag.

    Same contract as the synchronous builder, which returns M3D_EINVAL when a
    GT's IoU > 0 candidate list passes ``list_cap``: by default the cap is A,
    so no list can be truncated.  With a smaller explicit cap, each call queues
    a copy of its flag to pinned host memory, and the next call (or
    ``check()``, which waits for it) raises RuntimeError when it was set --
    truncated lists would label from an atomic-order-dependent subset.
    The error therefore arrives ONE STEP LATE by default: the training step
    that used the truncated targets has already run.  A caller that must not
    apply such a step calls ``check()`` at a sync point it already has in the
    same step (e.g. where it reads the loss back) before the optimizer."""

    def __init__(self, anchors, config, max_gt=64, list_cap=None):
        ops._dev(anchors)
        self.L = _lib.load()
        self.anchors = anchors.contiguous()
        self.A = int(anchors.shape[0])
        self.max_gt = int(max_gt)
        dev = anchors.device
        self.total = int(getattr(config, "RPN_TRAIN_ANCHORS_PER_IMAGE", 2048))
        self.pos_iou = float(getattr(config, "RPN_POSITIVE_IOU", 0.15))
        self.neg_iou = float(getattr(config, "RPN_NEGATIVE_IOU", 0.05))
        self.ratio = float(getattr(config, "RPN_POSITIVE_RATIO", 0.5))
        self.topk = int(getattr(config, "ATSS_TOPK", 24))
        self.min_pos = int(getattr(config, "ATSS_MIN_POS_PER_GT", 4))
        self.sd = (_lib.c_f * 6)(*[float(np.float32(v)) for v in config.RPN_BBOX_STD_DEV])
        self.cap = int(list_cap or self.A)
        self.wsb = int(self.L.m3d_rpn_targets_workspace_bytes(self.A, self.max_gt, self.cap))
        self.ws = torch.empty(max(self.wsb, 1), device=dev, dtype=torch.uint8)
        self.match = torch.empty((self.A,), device=dev, dtype=torch.int8)
        self.bbox = torch.empty((self.total, 6), device=dev, dtype=torch.float32)
        self.counts = torch.zeros((3,), device=dev, dtype=torch.int32)
        self._flag_host = torch.zeros((3,), dtype=torch.int32, pin_memory=True) if self.cap < self.A else None
        self._flag_event = None

    def check(self, wait=True):
        """Raise if the last call's candidate lists overflowed ``list_cap``.
        wait=False only looks at a flag whose copy has already landed."""
        ev = self._flag_event
        if ev is None:
            return
        if not wait and not ev.query():
            return
        ev.synchronize()
        self._flag_event = None
        if int(self._flag_host[2]) != 0:
            raise RuntimeError(f"rpn_targets_async: a GT overlaps more than list_cap={self.cap} anchors "
                               f"(its ATSS candidate list was truncated); raise list_cap (A = {self.A})")

    def __call__(self, gt_boxes, seed=0):
        from .model import DeviceRPNTargets
        ops._dev(gt_boxes)
        gt = gt_boxes.detach().float().reshape(-1, 6).contiguous()
        G = int(gt.shape[0])
        if G > self.max_gt:
            raise ValueError(f"{G} GT boxes, builder sized for max_gt={self.max_gt}")
        self.check()                                  # the previous call's flag (copy landed long ago)
        check(self.L.m3d_rpn_targets_async(ptr(self.anchors), self.A, ptr(gt), G, self.pos_iou, self.neg_iou,
                                           self.total, self.ratio, self.topk, self.min_pos, self.sd,
                                           int(seed) & 0xFFFFFFFF, ptr(self.match), ptr(self.bbox), self.cap,
                                           ptr(self.ws), self.wsb, ptr(self.counts), stream()),
              "rpn_targets_async")
        if self._flag_host is not None:
            self._flag_host.copy_(self.counts, non_blocking=True)
            self._flag_event = torch.cuda.Event()
            self._flag_event.record()
        return DeviceRPNTargets(self.match, self.bbox)
