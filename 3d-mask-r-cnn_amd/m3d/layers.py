"""Keras-layer surface of the hot path (drop-in for core/models.py callers).

``ProposalLayer(proposal_count, nms_threshold, pre_nms_limit, images_per_gpu,
rpn_bbox_std_dev, image_depth, name=...)([rpn_class, rpn_bbox, anchors])``
and ``PyramidROIAlign(pool_shape, name=...)([boxes, image_meta, P2..P5])``
take the reference's constructor arguments and call signature
(core/models.py:369-503, 597-687) and run entirely on the GPU: top-k with TF's
tie order, fused delta decode, bit-exact 3-D NMS and zero padding without a
host round trip; fused multi-level trilinear ROI align in original order.
"""
from __future__ import annotations

import torch

from . import ops


class ProposalLayer:
    def __init__(self, proposal_count, nms_threshold, pre_nms_limit, images_per_gpu,
                 rpn_bbox_std_dev, image_depth, name="ROI", **kwargs):
        self.proposal_count = int(proposal_count)
        self.nms_threshold = float(nms_threshold)
        self.pre_nms_limit = int(pre_nms_limit)
        self.images_per_gpu = int(images_per_gpu)
        self.rpn_bbox_std_dev = [float(v) for v in rpn_bbox_std_dev]
        self.image_depth = int(image_depth)
        self.name = name

    def __call__(self, inputs, return_counts=False):
        probs, deltas, anchors = inputs
        B, A = probs.shape[:2]
        if anchors.shape[1] != A or deltas.shape[1] != A:
            # the reference would gather past its anchor constant
            raise ValueError(f"ProposalLayer: {anchors.shape[1]} anchors, {deltas.shape[1]} deltas rows "
                             f"and {A} rpn_class rows must be equal")
        if anchors.shape[0] not in (1, B):
            raise ValueError("ProposalLayer: anchors batch must be 1 or IMAGES_PER_GPU")
        k = min(self.pre_nms_limit, A)
        out = torch.empty((B, self.proposal_count, 6), device=probs.device, dtype=torch.float32)
        counts = []
        with torch.no_grad():
            for b in range(B):
                pb = probs[b].detach().float().contiguous()
                db = deltas[b].detach().float().contiguous()
                ab = anchors[b if anchors.shape[0] > 1 else 0].detach().float().contiguous()
                order = ops.topk_order(pb, k)
                boxes, scores = ops.proposal_decode(pb, db, ab, order, self.rpn_bbox_std_dev,
                                                    self.image_depth, check_indices=False)
                keep, num = ops.non_max_suppression_3d_padded(boxes, scores, self.proposal_count,
                                                              self.nms_threshold)
                out[b] = ops.proposal_gather(boxes, keep, num, self.proposal_count)
                counts.append(num)
        if return_counts:
            return out, torch.cat(counts)
        return out

    def call_slab(self, inputs, sg, local_index):
        """The same proposals when this rank holds one depth slab of the volume
        (m3d.slab): probs/deltas [1,A_local,*] are the slab's RPN rows,
        local_index [A_local] their global anchor indices, anchors [1,A,6] the
        whole volume's.  Each slab's top-k candidates (global-order keys) are
        all-gathered, merged into the global top-k, and every rank runs the same
        decode + 3-D NMS -> rpn_rois [1,proposal_count,6] identical on all ranks
        and to the unsharded layer."""
        probs, deltas, anchors = inputs
        if probs.shape[0] != 1:
            raise ValueError("depth-slab proposals need IMAGES_PER_GPU = 1")
        A = anchors.shape[1]
        k = min(self.pre_nms_limit, A)
        with torch.no_grad():
            pb = probs[0].detach().float().contiguous()
            db = deltas[0].detach().float().contiguous()
            keys = ops.score_keys(pb, local_index)
            kl = min(k, keys.shape[0])
            vals, pos = ops.topk_keys(keys, kl, positions=True)
            # padding keys below every score key and distinct (m3d_topk_keys wants distinct keys);
            # never selected: the slabs hold at least k real candidates together (sum A_local = A >= k)
            ck = torch.iinfo(torch.int64).min + torch.arange(k, device=pb.device, dtype=torch.int64)
            cp = torch.zeros((k, 2), device=pb.device)
            cd = torch.zeros((k, 6), device=pb.device)
            ck[:kl], cp[:kl], cd[:kl] = vals, pb[pos], db[pos]
            gk = sg.all_gather(ck).reshape(-1)
            gp = sg.all_gather(cp).reshape(-1, 2)
            gd = sg.all_gather(cd).reshape(-1, 6)
            top, where = ops.topk_keys(gk, k, positions=True)
            gidx = 0xFFFFFFFF - (top & 0xFFFFFFFF)
            sel_p = gp.index_select(0, where).contiguous()
            sel_d = gd.index_select(0, where).contiguous()
            sel_a = anchors[0].detach().float().index_select(0, gidx).contiguous()
            order = torch.arange(k, device=pb.device, dtype=torch.int64)
            boxes, scores = ops.proposal_decode(sel_p, sel_d, sel_a, order, self.rpn_bbox_std_dev,
                                                self.image_depth, check_indices=False)
            keep, num = ops.non_max_suppression_3d_padded(boxes, scores, self.proposal_count,
                                                          self.nms_threshold)
            return ops.proposal_gather(boxes, keep, num, self.proposal_count)[None]

    def compute_output_shape(self, input_shape):
        return (None, self.proposal_count, 6)


class PyramidROIAlign:
    def __init__(self, pool_shape, name=None, **kwargs):
        self.pool_shape = tuple(int(v) for v in pool_shape)
        self.name = name

    def __call__(self, inputs):
        boxes, image_meta = inputs[0], inputs[1]
        return ops.pyramid_roi_align(boxes, image_meta, list(inputs[2:6]), self.pool_shape)

    def compute_output_shape(self, input_shape):
        return tuple(input_shape[0][:2]) + self.pool_shape + (input_shape[2][-1],)
