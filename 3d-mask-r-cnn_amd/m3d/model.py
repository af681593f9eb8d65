"""RPN training model (RPN.build / compile / one fit step) on the libm3d kernels.

Mirrors core/models.py:3162-3387:
  inputs [image, rpn_match, rpn_bbox] -> resnet_graph(stage5) -> FPN -> shared
  RPN head on P2..P6 -> (rpn_class_logits, rpn_class, rpn_bbox) -> ProposalLayer
  (POST_NMS_ROIS_TRAINING) -> rpn_class_loss (focal CE, 1589-1625) and
  rpn_bbox_loss (XY/Z Huber, 1629-1673), weighted 1.0 / 1.5 (3366-3376), plus
  the L2 term WEIGHT_DECAY*0.5*||w||^2/size(w) on every non-gamma/beta weight
  (3378-3384), optimised by the compiled Keras optimizer (m3d.optim: SGD,
  Adam or Adadelta with clipnorm and decay, 3349-3357).
The two losses run on the GPU as one fused libm3d pass (m3d_rpn_loss_fwd: both
terms and their gradients per anchor, fixed-order sums; rpn_losses) -- the
framework-op form below (rpn_class_loss / rpn_bbox_loss) is kept for host
tensors and as the GPU test's second reference; all convolution / pooling /
NMS work is libm3d.
"""
from __future__ import annotations


import numpy as np
import torch

from . import _lib
from .anchors import model_anchors
from .backbone import FPN, ResNet3D, RPNHead
from .layers import ProposalLayer
from .optim import KerasOptimizer
from .params import ParamStore

# Enqueue the ProposalLayer (side stream) after the loss instead of before it.
# Same work and dependencies; in a HIP-graph capture the loss / backward then is
# the forward's first successor (see nn.WGRAD_LAST).
PROPOSALS_AFTER_LOSS = False


# ---------------------------------------------------------------------------
# losses
# ---------------------------------------------------------------------------
class RPNTargets:
    """Host-side prepared RPN targets: the tf.where index sets of the loss
    graphs are fixed per batch, so they are built once on the host (where
    rpn_match is produced) instead of a device nonzero() + sync."""

    def __init__(self, rpn_match, rpn_bbox, device):
        m = np.asarray(rpn_match).reshape(rpn_match.shape[0], -1)
        B, A = m.shape
        flat = m.reshape(-1)
        cls_idx = np.nonzero(flat != 0)[0]                       # tf.where row-major order
        pos_idx = np.nonzero(flat == 1)[0]
        counts = (m == 1).sum(axis=1)
        rb = np.asarray(rpn_bbox, np.float32)
        gt = np.concatenate([rb[b, :counts[b]] for b in range(B)], axis=0) if B else rb[:0, 0]
        self.cls_idx = torch.from_numpy(cls_idx.astype(np.int64)).to(device)
        self.cls_labels = torch.from_numpy((flat[cls_idx] == 1).astype(np.int64)).to(device)
        self.pos_idx = torch.from_numpy(pos_idx.astype(np.int64)).to(device)
        self.gt_bbox = torch.from_numpy(gt.reshape(-1, 6).astype(np.float32)).to(device)
        self.n_cls, self.n_pos = len(cls_idx), len(pos_idx)
        # K.mean denominators (global counts; a depth slab holds only part of the anchors)
        self.cls_denom, self.pos_denom = self.n_cls, self.n_pos
        self._dense(flat, device)

    def _dense(self, flat_match, device):
        """Per-anchor form for the fused loss kernel (m3d_rpn_loss_fwd):
        match int8 [A] and each positive's row in gt_bbox (rank in flat order)."""
        fm = np.asarray(flat_match).reshape(-1)
        pos = fm == 1
        row = np.cumsum(pos, dtype=np.int64) - 1
        self.match8 = torch.from_numpy(np.sign(fm).astype(np.int8)).to(device)
        self.row32 = torch.from_numpy(np.maximum(row, 0).astype(np.int32)).to(device)

    @classmethod
    def for_slab(cls, rpn_match, rpn_bbox, local_index, device):
        """The targets of one depth slab (m3d.slab): rpn_match [1,A,1] and
        rpn_bbox [1,n,6] of the WHOLE volume, local_index [A_local] the global
        anchor index of each local RPN row.  Loss terms are restricted to the
        slab's anchors and divided by the whole volume's counts, so the sum of
        the ranks' losses is the single-volume loss."""
        m = np.asarray(rpn_match).reshape(-1)
        if np.asarray(rpn_match).shape[0] != 1:
            raise ValueError("depth-slab sharding runs one volume (IMAGES_PER_GPU = 1)")
        gidx = np.asarray(local_index, np.int64)
        lm = m[gidx]
        t = cls.__new__(cls)
        cls_idx = np.nonzero(lm != 0)[0]
        pos_idx = np.nonzero(lm == 1)[0]
        gpos = np.nonzero(m == 1)[0]                               # global positive order
        rows = np.searchsorted(gpos, gidx[pos_idx])
        rb = np.asarray(rpn_bbox, np.float32).reshape(-1, 6)
        t.cls_idx = torch.from_numpy(cls_idx.astype(np.int64)).to(device)
        t.cls_labels = torch.from_numpy((lm[cls_idx] == 1).astype(np.int64)).to(device)
        t.pos_idx = torch.from_numpy(pos_idx.astype(np.int64)).to(device)
        t.gt_bbox = torch.from_numpy(rb[rows].reshape(-1, 6)).to(device)
        t.n_cls, t.n_pos = len(cls_idx), len(pos_idx)
        t.cls_denom, t.pos_denom = int((m != 0).sum()), len(gpos)
        t._dense(lm, device)
        return t


class DeviceRPNTargets:
    """RPN targets resident on the device (m3d.targets.RPNTargetBuilder builds
    them inside the step): rpn_match int8 [A] and rpn_bbox [n, 6] (positives in
    anchor order).  The loss graphs' tf.where index sets become masks over all
    anchors and their counts stay on the device, so nothing waits for the host;
    the sums run in a different order than the index-set form (same terms)."""

    def __init__(self, rpn_match, rpn_bbox):
        self.match = rpn_match.reshape(-1)
        self.bbox = rpn_bbox.reshape(-1, 6)


def _rpn_class_loss_device(t: DeviceRPNTargets, rpn_class_logits, alpha, gamma):
    m = t.match
    logits = rpn_class_logits.reshape(-1, 2)
    labels = (m == 1).long()
    valid = (m != 0).to(logits.dtype)
    ce = torch.nn.functional.cross_entropy(logits, labels, reduction="none")
    p_t = torch.softmax(logits, dim=-1).gather(1, labels[:, None])[:, 0]
    ce = torch.pow(1.0 - p_t, gamma) * ce
    alpha_t = torch.where(labels == 1, torch.full_like(ce, alpha), torch.full_like(ce, 1.0 - alpha))
    return (alpha_t * ce * valid).sum() / valid.sum().clamp(min=1.0)


def _rpn_bbox_loss_device(t: DeviceRPNTargets, rpn_bbox):
    pos = t.match == 1
    rows = (torch.cumsum(pos.to(torch.int32), 0) - 1).clamp(0, t.bbox.shape[0] - 1)
    pred = rpn_bbox.reshape(-1, 6).clamp(-5.0, 5.0)
    diff = (t.bbox.index_select(0, rows.long()) - pred).clamp(-2.0, 2.0)
    ad = diff.abs()
    xy, zm = _xy_z_masks(diff.device)
    h = torch.where(ad < 1.0, 0.5 * diff * diff, ad - 0.5) * xy + \
        torch.where(ad < 0.5, 0.5 * diff * diff, 0.5 * ad - 0.25) * zm
    posf = pos.to(h.dtype)
    return (h * posf[:, None]).sum() / (6.0 * posf.sum().clamp(min=1.0))


def rpn_class_loss(t: RPNTargets, rpn_class_logits, alpha=0.90, gamma=1.5):
    """core/models.py:1589-1625."""
    if isinstance(t, DeviceRPNTargets):
        return _rpn_class_loss_device(t, rpn_class_logits, alpha, gamma)
    if t.n_cls == 0:
        return rpn_class_logits.sum() * 0.0
    logits = rpn_class_logits.reshape(-1, 2).index_select(0, t.cls_idx)
    ce = torch.nn.functional.cross_entropy(logits, t.cls_labels, reduction="none")
    probs = torch.softmax(logits, dim=-1)
    p_t = probs.gather(1, t.cls_labels[:, None])[:, 0]
    ce = torch.pow(1.0 - p_t, gamma) * ce
    alpha_t = torch.where(t.cls_labels == 1, torch.full_like(ce, alpha), torch.full_like(ce, 1.0 - alpha))
    return (alpha_t * ce).sum() / t.cls_denom


_MASKS = {}


def _xy_z_masks(dev):
    """The (y,x,-,y,x,-) / (-,-,z,-,-,z) coordinate masks, made once per device
    (no host-to-device copy inside a captured step)."""
    if dev not in _MASKS:
        _MASKS[dev] = (torch.tensor([1., 1., 0., 1., 1., 0.], device=dev),
                       torch.tensor([0., 0., 1., 0., 0., 1.], device=dev))
    return _MASKS[dev]


def rpn_bbox_loss(t: RPNTargets, rpn_bbox):
    """core/models.py:1629-1673."""
    if isinstance(t, DeviceRPNTargets):
        return _rpn_bbox_loss_device(t, rpn_bbox)
    if t.n_pos == 0:
        return rpn_bbox.sum() * 0.0
    pred = rpn_bbox.reshape(-1, 6).index_select(0, t.pos_idx).clamp(-5.0, 5.0)
    diff = (t.gt_bbox - pred).clamp(-2.0, 2.0)
    ad = diff.abs()
    xy, zm = _xy_z_masks(diff.device)
    h_xy = torch.where(ad < 1.0, 0.5 * diff * diff, ad - 0.5) * xy
    h_z = torch.where(ad < 0.5, 0.5 * diff * diff, 0.5 * ad - 0.25) * zm
    return (h_xy + h_z).sum() / (6 * t.pos_denom)




class _RPNLossFused(torch.autograd.Function):
    """Both RPN losses and their weighted total in two launches
    (m3d_rpn_loss_fwd; the per-anchor gradients are computed in the same pass
    and scaled in place by one launch in the backward), replacing ~100 small
    framework launches the host issues between the forward and the backward."""

    @staticmethod
    def forward(ctx, logits, bbox, match, row, gt, den_cls, den_pos, w_cls, w_box, alpha, gamma):
        A = match.numel()
        if logits.numel() != 2 * A or bbox.numel() != 6 * A:
            raise ValueError("rpn loss: logits / rpn_bbox do not match the targets' anchor count")
        logits = logits.contiguous()
        bbox = bbox.contiguous()
        dev = logits.device
        g_logits = torch.empty_like(logits)
        g_bbox = torch.empty_like(bbox)
        total, lc, lb = (torch.empty((), device=dev, dtype=torch.float32) for _ in range(3))
        scales = torch.empty(2, device=dev, dtype=torch.float32)
        L = _lib.load()
        ws = torch.empty(max(int(L.m3d_rpn_loss_workspace_bytes(A)), 1), device=dev, dtype=torch.uint8)
        if gt.shape[0] == 0:
            gt = torch.zeros(1, 6, device=dev, dtype=torch.float32)
        _lib.check(L.m3d_rpn_loss_fwd(_lib.ptr(logits), _lib.ptr(bbox), _lib.ptr(match),
                             _lib.ptr(row), _lib.ptr(gt), int(gt.shape[0]), A, float(alpha), float(gamma),
                             int(den_cls), int(den_pos), float(w_cls), float(w_box), _lib.ptr(g_logits),
                             _lib.ptr(g_bbox), _lib.ptr(total), _lib.ptr(lc), _lib.ptr(lb), _lib.ptr(scales),
                             _lib.ptr(ws), ws.numel(), _lib.stream()),
                   "m3d_rpn_loss_fwd")
        ctx.saved = (g_logits, g_bbox, scales, A)
        ctx.mark_non_differentiable(lc, lb)
        return total, lc, lb

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g_total, _g_lc, _g_lb):
        g_logits, g_bbox, scales, A = ctx.saved
        if g_total is None:
            return (None,) * 11
        if g_logits is None:
            raise RuntimeError("rpn loss: backward called twice on one forward (the kept per-anchor "
                               "gradients were scaled in place by the first call)")
        ctx.saved = (None, None, scales, A)
        g_total = g_total.contiguous().to(torch.float32)
        _lib.check(_lib.load().m3d_rpn_loss_bwd(_lib.ptr(g_logits), _lib.ptr(g_bbox), A, _lib.ptr(g_total),
                             _lib.ptr(scales), _lib.stream()), "m3d_rpn_loss_bwd")
        return (g_logits, g_bbox) + (None,) * 9


def rpn_losses(t, rpn_class_logits, rpn_bbox, w_cls=1.0, w_box=1.0, alpha=0.90, gamma=1.5):
    """(total, rpn_class_loss, rpn_bbox_loss): core/models.py:1589-1673 weighted
    as 3366-3376.  On the GPU through the fused libm3d kernel; host tensors
    (the CPU depth-slab tests) take the framework-op form below."""
    if rpn_class_logits.is_cuda:
        if isinstance(t, DeviceRPNTargets):
            pos = (t.match == 1).to(torch.int32)
            match8, row32 = t.match.to(torch.int8), torch.cumsum(pos, 0, dtype=torch.int32) - 1
            gt, den_c, den_p = t.bbox, 0, 0
        else:
            match8, row32, gt, den_c, den_p = t.match8, t.row32, t.gt_bbox, t.cls_denom, t.pos_denom
        return _RPNLossFused.apply(rpn_class_logits, rpn_bbox, match8, row32, gt.contiguous(), den_c, den_p,
                                   w_cls, w_box, alpha, gamma)
    lc = rpn_class_loss(t, rpn_class_logits, alpha, gamma)
    lb = rpn_bbox_loss(t, rpn_bbox)
    return lc * w_cls + lb * w_box, lc.detach(), lb.detach()


# ---------------------------------------------------------------------------
# model
# ---------------------------------------------------------------------------
class RPN:
    """The RPN of the reference in training mode, built on a flat ParamStore."""

    LOSS_WEIGHTS = {"rpn_class_loss": 1.0, "rpn_bbox_loss": 1.5}   # core/models.py:3366-3369

    def __init__(self, config, device="cuda", seed=1):
        h, w = int(config.IMAGE_SHAPE[0]), int(config.IMAGE_SHAPE[1])
        if h % 64 or w % 64:
            raise ValueError("IMAGE_SHAPE height & width must be multiples of 64")
        anchors = model_anchors(config)          # z-stride patch + row-count check, before any device work
        _lib.load()
        self.config = config
        self.device = torch.device(device)
        self.store = ParamStore()
        self.backbone = ResNet3D(self.store, config.BACKBONE, stage5=True, train_bn=config.TRAIN_BN)
        self.fpn = FPN(self.store, config.TOP_DOWN_PYRAMID_SIZE)
        self.rpn = RPNHead(self.store, config.RPN_ANCHOR_STRIDE, len(config.RPN_ANCHOR_RATIOS),
                           config.TOP_DOWN_PYRAMID_SIZE, backbone=self.backbone)
        self.store.finalize(self.device, seed=seed, weight_decay=float(config.WEIGHT_DECAY))
        self.anchors = torch.from_numpy(anchors).to(self.device)[None]
        self.proposal_layer = ProposalLayer(
            proposal_count=config.POST_NMS_ROIS_TRAINING, nms_threshold=config.RPN_NMS_THRESHOLD,
            pre_nms_limit=config.PRE_NMS_LIMIT, images_per_gpu=config.IMAGES_PER_GPU,
            rpn_bbox_std_dev=config.RPN_BBOX_STD_DEV, image_depth=config.IMAGE_DEPTH, name="ROI")
        self.optimizer = KerasOptimizer(config.OPTIMIZER)      # RPN.compile, core/models.py:3349-3357

    # -- forward ----------------------------------------------------------
    def features(self, image):
        _, C2, C3, C4, C5 = self.backbone(image)
        return self.fpn(C2, C3, C4, C5)

    def forward(self, image, proposals=True):
        from . import nn as _nn
        batch = _nn.BiasSums() if torch.is_grad_enabled() else None
        prev, _nn.BIAS_BATCH = _nn.BIAS_BATCH, batch
        if _nn.X3_PLANES_BATCHED:
            _nn.X3_PLANES.refresh(self.device)   # live for this forward (nn.X3Planes)
        _nn.WINO_V.active_fwd = _nn.WINO_V.active_dgrad = (
            _nn.WINO_V_PREPASS and torch.is_grad_enabled() and image[0].numel() >= _nn.WINO_V_PREPASS_MIN_VOXELS)
        if _nn.WINO_V.active_dgrad:
            _nn.WINO_V.refresh(self.device)     # Winograd weight transforms on a side stream (nn.WinoVPrep)
        try:
            fmaps = self.features(image)
            logits, probs, bbox = self.rpn(fmaps)
        finally:
            _nn.BIAS_BATCH = prev
            _nn.X3_PLANES.invalidate()          # the backward takes its planes through ctx
            _nn.WINO_V.invalidate()
            _nn.WINO_V.active_fwd = _nn.WINO_V.active_dgrad = False
        if batch is not None:
            self.rpn.bias_batch = batch         # flushed by RPNHead.finish_backward
        rois = None
        if proposals:
            rois = self.proposal_layer([probs, bbox, self.anchors])
        return {"rpn_class_logits": logits, "rpn_class": probs, "rpn_bbox": bbox,
                "rpn_rois": rois, "feature_maps": fmaps}

    def losses(self, out, targets: RPNTargets):
        lc = rpn_class_loss(targets, out["rpn_class_logits"])
        lb = rpn_bbox_loss(targets, out["rpn_bbox"])
        return lc, lb

    def loss_total(self, out, targets: RPNTargets):
        """(weighted total, rpn_class_loss, rpn_bbox_loss) -- the fused kernel on the GPU."""
        return rpn_losses(targets, out["rpn_class_logits"], out["rpn_bbox"],
                          self.LOSS_WEIGHTS["rpn_class_loss"], self.LOSS_WEIGHTS["rpn_bbox_loss"])

    # -- one fit step -----------------------------------------------------
    @property
    def iterations(self):
        return self.optimizer.iterations

    def current_lr(self):
        return self.optimizer.current_lr()

    def proposals_async(self, out):
        """Launch the ProposalLayer (top-k, decode, 3-D NMS) of a forward's
        outputs on a side HIP stream, so it runs concurrently with the backward
        (nothing in the backward depends on it; its serial NMS reduce occupies
        one CU).  Returns (rois, join): call join() before using rois on the
        current stream."""
        main = torch.cuda.current_stream(self.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(self.device)
        side = self._side
        side.wait_stream(main)
        probs, bbox = out["rpn_class"].detach(), out["rpn_bbox"].detach()
        with torch.cuda.stream(side):
            rois = self.proposal_layer([probs, bbox, self.anchors])
        probs.record_stream(side)
        bbox.record_stream(side)

        def join():
            main.wait_stream(side)
            rois.record_stream(main)
            return rois
        return rois, join

    def forward_backward(self, image, targets: RPNTargets, proposals=True):
        """One step up to (not including) the optimizer: gradients in
        store.grad_flat, the ProposalLayer overlapped on its side stream."""
        self.store.zero_grad()
        out = self.forward(image, proposals=False)
        join = self.proposals_async(out)[1] if proposals and not PROPOSALS_AFTER_LOSS else None
        total, lc, lb = self.loss_total(out, targets)
        if proposals and PROPOSALS_AFTER_LOSS:
            join = self.proposals_async(out)[1]
        total.backward()
        self.rpn.finish_backward()
        return {"loss": total.detach(), "rpn_class_loss": lc.detach(), "rpn_bbox_loss": lb.detach(),
                "rpn_rois": join() if join is not None else None}

    def train_step(self, image, targets: RPNTargets, proposals=True):
        r = self.forward_backward(image, targets, proposals)
        self.sgd_step()
        return r

    def graphed_train_step(self, image, targets: RPNTargets, proposals=True, warmup=2):
        """The training step with its forward + backward (+ ProposalLayer on
        the side stream) captured once into a HIP graph: ~680 launches replay
        without the host's per-launch overhead (host 6.6 ms per replay against
        16.5 ms eager, step 26.04 vs 26.23 ms at 128^3; the replay runs each
        stream's chain on its own queue once every fork is captured compute
        path first, nn.WGRAD_LAST).
        The optimizer runs eagerly after each replay
        (its learning rate decays per iteration).  ``image`` and ``targets``
        are the graph's static inputs: copy new data into them in place.
        Returns step() -> the result dict of the captured step (same tensors
        every call, refreshed by each replay)."""
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(side):                 # lazy streams / caches, allocator warm-up
            for _ in range(warmup):
                self.train_step(image, targets, proposals)
        torch.cuda.current_stream(self.device).wait_stream(side)
        torch.cuda.synchronize(self.device)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            res = self.forward_backward(image, targets, proposals)
        self._graph = graph                           # keep the graph (and its pool) alive

        def step():
            graph.replay()
            self.sgd_step()
            return res
        return step

    def load_weights(self, filepath, by_name=True, skip_mismatch=False, exclude=()):
        """keras_model.load_weights(filepath, by_name=True, ...) on the Keras-H5 format (m3d.weights)."""
        from .weights import load_weights
        return load_weights(self.store, filepath, by_name=by_name, skip_mismatch=skip_mismatch, exclude=exclude)

    def save_weights(self, filepath):
        """keras_model.save_weights(filepath): Keras-H5 layout, readable by the reference."""
        from .weights import save_weights
        save_weights(self.store, filepath)

    def optimizer_step(self):
        """Apply the compiled Keras optimizer (SGD / Adam / Adadelta) to store.grad_flat."""
        self.optimizer.step(self.store)

    sgd_step = optimizer_step          # name kept for callers written against the SGD-only path

    def l2_loss(self):
        with torch.no_grad():
            tot = torch.zeros((), device=self.device)
            for p in self.store.params:
                if p.l2:
                    tot = tot + (self.config.WEIGHT_DECAY * 0.5) * (p.data * p.data).sum() / p.numel
            return tot


# ---------------------------------------------------------------------------
# synthetic inputs
# ---------------------------------------------------------------------------
def synthetic_volume(size, depth=None, batch=1, seed=0):
    """x = tanh(0.5 * N(0,1)), [B,S,S,D,1] float32 (range of core/data_generators.py:1612-1628)."""
    g = torch.Generator().manual_seed(seed)
    d = size if depth is None else depth
    return torch.tanh(0.5 * torch.randn((batch, size, size, d, 1), generator=g))


def synthetic_rpn_targets(n_anchors, n_train=1536, pos_frac=0.5, batch=1, seed=2):
    """Seeded rpn_match [B,A,1] (+1/-1/0) with <= n_train non-zero entries and
    rpn_bbox [B,n_train,6] delta targets (std-normalised scale).  Stands in for
    the host target builder (core/data_generators.py:2031-2178, out of scope)."""
    rng = np.random.default_rng(seed)
    match = np.zeros((batch, n_anchors, 1), np.int32)
    bbox = np.zeros((batch, n_train, 6), np.float32)
    for b in range(batch):
        sel = rng.choice(n_anchors, size=min(n_train, n_anchors), replace=False)
        npos = int(len(sel) * pos_frac)
        match[b, sel[:npos], 0] = 1
        match[b, sel[npos:], 0] = -1
        bbox[b, :npos] = rng.normal(0.0, 1.0, size=(npos, 6)).astype(np.float32)
    return match, bbox


def compose_image_meta(image_id, original_shape, image_shape, window, scale, active_class_ids):
    """core/models.py compose_image_meta layout: [id, orig(4), shape(4), window(6), scale, classes]."""
    return np.array([image_id] + list(original_shape) + list(image_shape) + list(window) + [scale] +
                    list(active_class_ids), dtype=np.float32)
