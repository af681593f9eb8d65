"""torch-level wrappers over libm3d.so.

Mirrors the Python surface of the reference's custom ops
(``core/custom_op/custom_op.py:22-65``): same names, argument order and
meaning, same InvalidArgument texts (raised as ``ValueError``), and the same
registered gradient ([grad_image, grad_boxes, None, None]).

Every op runs the HIP kernels of libm3d.so on the current HIP stream and
fails loudly (``ValueError`` / ``M3DError``) on CPU tensors -- there is no CPU
fallback in the product path.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import check, ptr, stream

_METHODS = {"trilinear": 0, "bilinear": 0, "nearest": 1}


def _L():
    return _lib.load()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("m3d ops run on the GPU only: got a CPU tensor (no CPU fallback)")


def _c(t, dtype=torch.float32):
    return t.contiguous() if t.dtype == dtype else t.to(dtype).contiguous()


# ---------------------------------------------------------------------------
# CropAndResize3D  (core/custom_op/custom_op.py:22-24, gradient 28-65)
# ---------------------------------------------------------------------------
def _check_crop(image, boxes, box_ind, crop_size):
    if image.dim() != 5:
        raise ValueError("input image must be 5-D")
    if boxes.dim() != 2:
        raise ValueError("boxes must be 2-D")
    if boxes.shape[1] != 6:
        raise ValueError("boxes must have 6 columns")
    if box_ind.dim() != 1 or box_ind.shape[0] != boxes.shape[0]:
        raise ValueError("box_index has incompatible shape")
    if len(crop_size) != 3:
        raise ValueError("crop_size must have three elements")
    if any(int(c) <= 0 for c in crop_size):
        raise ValueError("crop dimensions must be positive")


def _crop_fwd(image, boxes, box_ind, crop_size, method, extrap):
    B, H, W, D, C = image.shape
    ch, cw, cd = (int(c) for c in crop_size)
    N = boxes.shape[0]
    out = torch.empty((N, ch, cw, cd, C), device=image.device, dtype=torch.float32)
    check(_L().m3d_crop_and_resize3d_fwd(ptr(image), B, H, W, D, C, ptr(boxes), ptr(box_ind), N,
                                         ch, cw, cd, method, float(extrap), ptr(out), stream()),
          "crop_and_resize_3d")
    return out


def crop_and_resize_3d_grad_image(grads, boxes, box_ind, image_size, T=torch.float32,
                                  method_name="trilinear", deterministic=False):
    """grads [N,ch,cw,cd,C] -> d image [B,H,W,D,C].

    deterministic: False / 0 -- fp32 atomics (fast, last bits vary with arrival
    order); True / 1 -- destination-owned sums in the reference's sequential
    summation order (bit-identical to the wheel's CPU scatter, parallel over
    voxels); 2 -- the single-thread-per-channel sequential replay (the same
    bits, slow; kept as the in-library check of mode 1)."""
    _dev(grads, boxes, box_ind)
    if method_name not in _METHODS:
        raise ValueError("method must be 'trilinear' or 'nearest'")
    grads, boxes, box_ind = _c(grads), _c(boxes), _c(box_ind, torch.int32)
    B, H, W, D, C = (int(v) for v in image_size)
    N, ch, cw, cd, _ = grads.shape
    out = torch.empty((B, H, W, D, C), device=grads.device, dtype=torch.float32)
    check(_L().m3d_crop_and_resize3d_bwd_image(ptr(grads), ptr(boxes), ptr(box_ind), N, ch, cw, cd,
                                               B, H, W, D, C, _METHODS[method_name],
                                               int(deterministic), ptr(out), stream()),
          "crop_and_resize_3d_grad_image")
    return out.to(T) if T != torch.float32 else out


def crop_and_resize_3d_grad_boxes(grads, image, boxes, box_ind, method_name="trilinear"):
    """d boxes [N,6] of the trilinear sampling (also used for 'nearest', as the reference)."""
    _dev(grads, image, boxes, box_ind)
    grads, image, boxes, box_ind = _c(grads), _c(image), _c(boxes), _c(box_ind, torch.int32)
    B, H, W, D, C = image.shape
    N, ch, cw, cd, _ = grads.shape
    out = torch.empty((N, 6), device=grads.device, dtype=torch.float32)
    check(_L().m3d_crop_and_resize3d_bwd_boxes(ptr(grads), ptr(image), B, H, W, D, C, ptr(boxes),
                                               ptr(box_ind), N, ch, cw, cd, ptr(out), stream()),
          "crop_and_resize_3d_grad_boxes")
    return out


class _CropAndResize3D(torch.autograd.Function):
    @staticmethod
    def forward(ctx, image, boxes, box_ind, crop_size, method, extrap):
        out = _crop_fwd(image, boxes, box_ind, crop_size, method, extrap)
        ctx.save_for_backward(image, boxes, box_ind)
        ctx.method = method
        return out

    @staticmethod
    def backward(ctx, grad):
        image, boxes, box_ind = ctx.saved_tensors
        grad = grad.contiguous()
        mname = "nearest" if ctx.method == 1 else "trilinear"
        g_img = None
        if ctx.needs_input_grad[0]:
            g_img = crop_and_resize_3d_grad_image(grad, boxes, box_ind, image.shape,
                                                  method_name=mname)
        g_box = None
        if ctx.needs_input_grad[1]:
            g_box = crop_and_resize_3d_grad_boxes(grad, image, boxes, box_ind)
        return g_img, g_box, None, None, None, None


def crop_and_resize_3d(image, boxes, box_ind, crop_size, method_name="trilinear",
                       extrapolation_value=0.0, validate=True):
    """CropAndResize3D: image [B,H,W,D,C], boxes [N,6] normalised, box_ind [N] ->
    crops [N,ch,cw,cd,C]."""
    _dev(image, boxes, box_ind)
    if method_name not in _METHODS:
        raise ValueError("method must be 'trilinear' or 'nearest'")
    crop_size = [int(c) for c in (crop_size.tolist() if torch.is_tensor(crop_size) else crop_size)]
    _check_crop(image, boxes, box_ind, crop_size)
    image, boxes, box_ind = _c(image), _c(boxes), _c(box_ind, torch.int32)
    if validate and box_ind.numel():
        lo, hi = int(box_ind.min()), int(box_ind.max())
        if lo < 0 or hi >= image.shape[0]:
            raise ValueError("box_index has values outside [0, batch_size)")
    return _CropAndResize3D.apply(image, boxes, box_ind, crop_size, _METHODS[method_name],
                                  float(extrapolation_value))


def detection_mask_targets(gt_masks, positive_rois, roi_gt_box_assignment, mask_shape,
                           use_mini_mask=False, roi_gt_boxes=None):
    """Mask targets of detection_targets_graph (core/models.py:972-996).

    gt_masks [H,W,D,G] bool/uint8, positive_rois [P,6], roi_gt_box_assignment [P]
    -> [P, mh, mw, md] float32 in {0,1} (tf.round of the trilinear crop)."""
    _dev(gt_masks, positive_rois, roi_gt_box_assignment)
    H, W, D, G = gt_masks.shape
    boxes = _c(positive_rois.detach())
    if use_mini_mask:
        gb = roi_gt_boxes.detach().float()
        gh, gw, gd = gb[:, 3] - gb[:, 0], gb[:, 4] - gb[:, 1], gb[:, 5] - gb[:, 2]
        den = torch.stack([gh, gw, gd, gh, gw, gd], 1)
        off = torch.cat([gb[:, :3], gb[:, :3]], 1)
        boxes = ((boxes - off) / den).contiguous()
    m = gt_masks.to(torch.uint8).contiguous()
    assign = _c(roi_gt_box_assignment, torch.int32)
    P = boxes.shape[0]
    mh, mw, md = (int(v) for v in mask_shape)
    out = torch.empty((P, mh, mw, md), device=boxes.device, dtype=torch.float32)
    check(_L().m3d_mask_targets3d(ptr(m), H, W, D, G, ptr(boxes), ptr(assign), P, mh, mw, md,
                                  ptr(out), stream()), "mask_targets3d")
    return out


# ---------------------------------------------------------------------------
# NonMaxSuppression3D (core/custom_op/custom_op.py:25)
# ---------------------------------------------------------------------------
def non_max_suppression_3d_padded(boxes, scores, max_output_size, iou_threshold=0.5, mode="3d"):
    """Sync-free NMS: returns (keep int32 [max_output_size], num_keep int32 [1] on device).

    Entries of ``keep`` past ``num_keep`` are undefined."""
    _dev(boxes, scores)
    cols = 4 if mode == "2d" else 6
    if boxes.dim() != 2:
        raise ValueError("boxes must be 2-D")
    if boxes.shape[1] != cols:
        raise ValueError(f"boxes must have {cols} columns")
    if scores.dim() != 1:
        raise ValueError("scores must be 1-D")
    if scores.shape[0] != boxes.shape[0]:
        raise ValueError("scores has incompatible shape")
    if torch.is_tensor(max_output_size) and max_output_size.dim() != 0:
        raise ValueError("max_output_size must be 0-D")
    max_out = int(max_output_size)
    thr = float(iou_threshold)
    if not (0.0 <= thr <= 1.0):
        raise ValueError("iou_threshold must be in [0, 1]")
    boxes, scores = _c(boxes), _c(scores)
    N = boxes.shape[0]
    keep = torch.empty(max(max_out, 1), device=boxes.device, dtype=torch.int32)
    num = torch.empty(1, device=boxes.device, dtype=torch.int32)
    wsb = int(_L().m3d_nms3d_workspace_bytes(N))
    ws = torch.empty(max(wsb, 1), device=boxes.device, dtype=torch.uint8)
    check(_L().m3d_nms3d(ptr(boxes), ptr(scores), N, max_out, thr, 1 if mode == "2d" else 0,
                         ptr(keep), ptr(num), ptr(ws), wsb, stream()), "non_max_suppression_3d")
    return keep[:max(max_out, 0)], num


def non_max_suppression_3d(boxes, scores, max_output_size, iou_threshold=0.5, name=None):
    """Reference signature; returns int32 selected indices [M <= max_output_size]
    (un-padded, as the reference op).  Synchronises once to read M."""
    keep, num = non_max_suppression_3d_padded(boxes, scores, max_output_size, iou_threshold)
    return keep[: int(num.item())]


# ---------------------------------------------------------------------------
# PyramidROIAlign (core/models.py:597-687)
# ---------------------------------------------------------------------------
class _PyramidROIAlign(torch.autograd.Function):
    @staticmethod
    def forward(ctx, boxes, image_meta, pool_shape, p2, p3, p4, p5):
        fmaps = [p2, p3, p4, p5]
        B, N = boxes.shape[:2]
        C = p2.shape[-1]
        ph, pw, pd = pool_shape
        out = torch.empty((B, N, ph, pw, pd, C), device=p2.device, dtype=torch.float32)
        boxes_adj = torch.empty((B, N, 6), device=p2.device, dtype=torch.float32)
        levels = torch.empty((B, N), device=p2.device, dtype=torch.int32)
        fptrs = (_lib.c_p * 4)(*[f.data_ptr() for f in fmaps])
        fshape = ((_lib.c_i64 * 3) * 4)(*[(_lib.c_i64 * 3)(*f.shape[1:4]) for f in fmaps])
        # workspace of the spatially sorted line order (overlapping ROIs share rows in L2)
        wsb = int(_L().m3d_pyramid_roi_align3d_fwd_workspace_bytes(fshape, B, N, ph, pw))
        ws = torch.empty(wsb, device=boxes.device, dtype=torch.uint8)
        check(_L().m3d_pyramid_roi_align3d_fwd_ws(fptrs, fshape, C, ptr(boxes), ptr(image_meta),
                                                  image_meta.shape[1], B, N, ph, pw, pd, ptr(out),
                                                  ptr(boxes_adj), ptr(levels), ptr(ws), wsb, stream()),
              "pyramid_roi_align")
        ctx.save_for_backward(boxes_adj, levels)
        ctx.shapes = [tuple(f.shape) for f in fmaps]
        ctx.pool = (ph, pw, pd)
        ctx.mark_non_differentiable(boxes_adj, levels)
        return out, boxes_adj, levels

    @staticmethod
    def backward(ctx, grad, _g1, _g2):
        boxes_adj, levels = ctx.saved_tensors
        grad = grad.contiguous()
        gmaps = [torch.empty(s, device=grad.device, dtype=torch.float32) for s in ctx.shapes]
        B, N = boxes_adj.shape[:2]
        ph, pw, pd = ctx.pool
        gptrs = (_lib.c_p * 4)(*[g.data_ptr() for g in gmaps])
        fshape = ((_lib.c_i64 * 3) * 4)(*[(_lib.c_i64 * 3)(*s[1:4]) for s in ctx.shapes])
        if _lib.deterministic() and max(ph, pw, pd) <= 64:
            # bitwise reproducible: per level, the destination-owned sums in the reference's order
            bi = torch.empty(4 * B * N, device=grad.device, dtype=torch.int32)
            check(_L().m3d_pyramid_roi_align3d_bwd_det(ptr(grad), ptr(boxes_adj), ptr(levels), B, N, ph, pw,
                                                       pd, gptrs, fshape, ctx.shapes[0][-1], ptr(bi), stream()),
                  "pyramid_roi_align bwd (deterministic)")
        else:
            check(_L().m3d_pyramid_roi_align3d_bwd(ptr(grad), ptr(boxes_adj), ptr(levels), B, N, ph, pw,
                                                   pd, gptrs, fshape, ctx.shapes[0][-1], stream()),
                  "pyramid_roi_align bwd")
        return (None, None, None) + tuple(gmaps)


def pyramid_roi_align(boxes, image_meta, feature_maps, pool_shape, return_levels=False):
    """boxes [B,N,6] (stop-gradient, as the reference), image_meta [B,M],
    feature_maps [P2,P3,P4,P5] each [B,H,W,D,C] -> pooled [B,N,ph,pw,pd,C]."""
    _dev(boxes, image_meta, *feature_maps)
    if len(feature_maps) != 4:
        raise ValueError("PyramidROIAlign needs the four maps P2..P5")
    C = feature_maps[0].shape[-1]
    for f in feature_maps:
        if f.dim() != 5 or f.shape[-1] != C or f.shape[0] != boxes.shape[0]:
            raise ValueError("feature maps must be [B,H,W,D,C] with equal B and C")
    boxes = _c(boxes.detach())
    image_meta = _c(image_meta.detach())
    fm = [_c(f) for f in feature_maps]
    out, boxes_adj, levels = _PyramidROIAlign.apply(boxes, image_meta, tuple(int(v) for v in pool_shape),
                                                    *fm)
    if return_levels:
        return out, boxes_adj, levels
    return out


# ---------------------------------------------------------------------------
# ProposalLayer device pipeline (core/models.py:382-500), one image.
# ---------------------------------------------------------------------------
def topk_keys(keys, k, positions=False):
    """tf.nn.top_k(keys, k, sorted=True) on distinct int64 keys (m3d_topk_keys,
    the hand-written radix select + rank sort; core/models.py:403-404):
    values [k] descending, and with ``positions`` their indices in ``keys``."""
    keys = _c(keys, torch.int64)
    n = keys.shape[0]
    vals = torch.empty(k, device=keys.device, dtype=torch.int64)
    pos = torch.empty(k, device=keys.device, dtype=torch.int64) if positions else None
    nb = int(_L().m3d_topk_workspace_bytes(n, k))
    ws = torch.empty(nb // 8 + 1, device=keys.device, dtype=torch.int64)
    check(_L().m3d_topk_keys(ptr(keys), n, k, ptr(vals), ptr(pos), ptr(ws), nb, stream()), "topk_keys")
    return (vals, pos) if positions else vals


def topk_order(probs, k):
    """tf.nn.top_k(probs[:,1], k, sorted=True).indices with TF's tie order
    (lower index first) via unique int64 keys built on the GPU."""
    A = probs.shape[0]
    keys = torch.empty(A, device=probs.device, dtype=torch.int64)
    check(_L().m3d_score_keys(ptr(probs), A, ptr(keys), stream()), "score_keys")
    vals = topk_keys(keys, k)
    return (0xFFFFFFFF - (vals & 0xFFFFFFFF)).to(torch.int64)


def score_keys(probs, global_index=None):
    """int64 top-k keys of probs[:,1] (score desc, lower GLOBAL index first);
    global_index [A] int64 maps rows to whole-volume anchor indices (depth slabs)."""
    A = probs.shape[0]
    keys = torch.empty(A, device=probs.device, dtype=torch.int64)
    gi = None if global_index is None else _c(global_index, torch.int64)
    check(_L().m3d_score_keys_mapped(ptr(probs), A, ptr(gi), ptr(keys), stream()), "score_keys")
    return keys


def proposal_decode(probs, deltas, anchors, order, std_dev, image_depth, check_indices=True):
    """Top-k gather + apply_box_deltas_graph + clips + min sizes
    (core/models.py:391-447) for one image: probs [A,2], deltas [A,6], anchors
    [A,6], order [k] int64 anchor indices.  An order index outside [0, A) is
    the reference's tf.gather InvalidArgument: the kernel never reads it and
    raises a device flag; with check_indices (default) the flag is read back
    here (one sync) and ValueError raised.  ProposalLayer passes False: its
    order comes from top-k over the same A rows, checked on the host."""
    A = anchors.shape[0]
    if probs.shape[0] != A or deltas.shape[0] != A:
        raise ValueError(f"proposal_decode: probs {tuple(probs.shape)} / deltas {tuple(deltas.shape)} "
                         f"rows differ from the {A} anchors")
    k = order.shape[0]
    if k > A:
        raise ValueError(f"proposal_decode: {k} indices for {A} anchors")
    boxes = torch.empty((k, 6), device=probs.device, dtype=torch.float32)
    scores = torch.empty((k,), device=probs.device, dtype=torch.float32)
    err = torch.zeros((1,), device=probs.device, dtype=torch.int32) if check_indices else None
    sd = (_lib.c_f * 6)(*[float(torch.tensor(v, dtype=torch.float32)) for v in std_dev])
    check(_L().m3d_proposal_decode(ptr(probs), ptr(deltas), ptr(anchors), A, ptr(order), k, sd,
                                   float(image_depth), ptr(boxes), ptr(scores), ptr(err), stream()),
          "proposal_decode")
    if err is not None and int(err.item()) != 0:
        raise ValueError(f"indices[...] is not in [0, {A}): a top-k index names no anchor "
                         "(GatherV2 InvalidArgument in the reference graph)")
    return boxes, scores


def proposal_gather(boxes, keep, num_keep, P):
    out = torch.empty((P, 6), device=boxes.device, dtype=torch.float32)
    check(_L().m3d_proposal_gather(ptr(boxes), ptr(keep), ptr(num_keep), P, ptr(out), stream()),
          "proposal_gather")
    return out
