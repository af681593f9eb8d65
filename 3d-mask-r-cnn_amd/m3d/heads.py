"""Mask R-CNN heads, DetectionLayer and the full inference model on libm3d.

Mirrors the reference's inference graph (MaskRCNN.build, MODE "inference",
core/models.py:5473-5760):

  backbone + FPN + RPN -> ProposalLayer(POST_NMS_ROIS_INFERENCE)
  -> PyramidROIAlign(POOL_SIZE) -> fpn_classifier_graph   (1121-1186)
  -> DetectionLayer (refine_detections_graph)            (1415-1575)
  -> PyramidROIAlign(MASK_POOL_SIZE) on the detections -> build_fpn_mask_graph (1190-1234)

Layer names follow the Keras weights (mrcnn_class_conv1, mrcnn_class_bn1, ...,
mrcnn_mask_deconv, mrcnn_mask) so an H5 importer maps 1:1.  Every op is a
libm3d kernel:
  * mrcnn_class_conv1 (a pool^3 'valid' conv = one GEMM with K = pool^3*C):
    split-K batched GEMM + deterministic reduce with the fused BN/ReLU;
  * mrcnn_class_conv2 (1^3): conv kernel with fused bias/BN/ReLU;
  * the two Dense heads: one GEMM over the concatenated kernels, then
    m3d_head_outputs (clip, softmax, bbox reshape);
  * mask convs: conv kernel (Winograd for 3^3 'same'), the dilated conv3b with
    its post-activation residual Add fused in the epilogue, the 2x2x2 stride-2
    transposed conv as one GEMM with a scattering epilogue, the sigmoid 1^3 conv;
  * DetectionLayer: m3d_refine_detections + 2-D m3d_nms3d + m3d_detections_gather.
Inference only (TRAIN_BN=False: BN uses moving statistics).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib, ops
from ._lib import check, ptr, stream
from .anchors import model_anchors
from .backbone import FPN, ResNet3D, RPNHead
from .layers import ProposalLayer, PyramidROIAlign
from .nn import conv_bn_act, conv_geom
from .params import BNLayer, ConvLayer, ParamStore


def _L():
    return _lib.load()


def _bn_affine(bn):
    aff = torch.empty((3, bn.c), device=bn.gamma.data.device, dtype=torch.float32)
    check(_L().m3d_bn_affine(ptr(bn.gamma.data), ptr(bn.beta.data), ptr(bn.moving_mean),
                             ptr(bn.moving_variance), float(bn.eps), bn.c, ptr(aff[1]), ptr(aff[2]),
                             ptr(aff[0]), stream()), "bn_affine")
    return aff[1], aff[2]


class DenseLayer:
    """KL.Dense kernel [in, out] + bias (Keras names <name>/kernel:0, bias:0)."""

    def __init__(self, store, name, cin, cout, kernel_init="glorot_uniform", bias_init="zeros"):
        self.name, self.cin, self.cout = name, cin, cout
        self.kernel = store.add(f"{name}/kernel:0", (cin, cout), kernel_init, True)
        self.bias = store.add(f"{name}/bias:0", (cout,), bias_init, True)


class ClassifierHead:
    """fpn_classifier_graph(y, pool_size, num_classes, fc_layers_size, train_bn=False)."""

    SPLITK_TARGET_BLOCKS = 512

    def __init__(self, store, pool_size, num_classes, fc_layers_size, channels=256):
        p, fc = pool_size, fc_layers_size
        self.pool, self.C, self.fc, self.cin = p, num_classes, fc, channels
        self.conv1 = ConvLayer(store, "mrcnn_class_conv1", (p, p, p), channels, fc)
        self.bn1 = BNLayer(store, "mrcnn_class_bn1", fc)
        self.conv2 = ConvLayer(store, "mrcnn_class_conv2", (1, 1, 1), fc, fc)
        self.bn2 = BNLayer(store, "mrcnn_class_bn2", fc)
        fg = 0.15
        self.logits = DenseLayer(store, "mrcnn_class_logits", fc, num_classes, ("normal", 0.01),
                                 ("const", [-math.log((1 - fg) / fg), math.log(fg / (1 - fg))]))
        self.bbox = DenseLayer(store, "mrcnn_bbox_fc", fc, num_classes * 6, ("normal", 0.001))

    def _conv1(self, x2d):
        """[M, K] @ [K, fc] with split-K (K = pool^3 * C is ~88k for 7^3x256)."""
        L = _L()
        M, K = x2d.shape
        fc = self.fc
        tiles = -(-M // 128) * -(-fc // 128)
        splits = max(1, min(64, self.SPLITK_TARGET_BLOCKS // max(tiles, 1), K // 1024))
        kc = -(-(-(-K // splits)) // 32) * 32                  # slice width, multiple of 32
        splits = -(-K // kc)
        ws = torch.empty((splits, M, fc), device=x2d.device, dtype=torch.float32)
        w = self.conv1.kernel.data.reshape(K, fc)
        full = K // kc
        if full:
            check(L.m3d_gemm_f32_ex(ptr(x2d), K, kc, ptr(w), kc * fc, ptr(ws), M * fc, full, M, kc, fc,
                                    None, 0, 0, stream()), "class_conv1 gemm")
        if full < splits:
            rem = K - full * kc
            check(L.m3d_gemm_f32_ex(x2d.data_ptr() + 4 * full * kc, K, 0, w[full * kc:].data_ptr(), 0,
                                    ws[full].data_ptr(), 0, 1, M, rem, fc, None, 0, 0, stream()),
                  "class_conv1 gemm tail")
        scale, shift = _bn_affine(self.bn1)
        h = torch.empty((M, fc), device=x2d.device, dtype=torch.float32)
        check(L.m3d_splitk_reduce(ptr(ws), splits, M, fc, ptr(self.conv1.bias.data), ptr(scale), ptr(shift),
                                  1, ptr(h), stream()), "class_conv1 reduce")
        return h

    def __call__(self, pooled):
        B, N = pooled.shape[:2]
        M = B * N
        L = _L()
        x = pooled.reshape(M, -1).contiguous()
        h = self._conv1(x)
        scale, shift = _bn_affine(self.bn2)
        h2 = torch.empty_like(h)
        check(L.m3d_conv3d_fwd(ptr(h), 1, 1, 1, M, self.fc, ptr(self.conv2.kernel.data), 1, 1, 1, self.fc,
                               1, 1, M, 1, 1, 1, 0, 0, 0, ptr(self.conv2.bias.data), ptr(scale),
                               ptr(shift), None, 0, 1, None, ptr(h2), self.fc, None, 0, 0, stream()),
              "class_conv2")
        C = self.C
        nraw = -(-7 * C // 4) * 4
        wcat = torch.zeros((self.fc, nraw), device=h.device, dtype=torch.float32)
        wcat[:, :C] = self.logits.kernel.data
        wcat[:, C:7 * C] = self.bbox.kernel.data
        bcat = torch.zeros((nraw,), device=h.device, dtype=torch.float32)
        bcat[:C] = self.logits.bias.data
        bcat[C:7 * C] = self.bbox.bias.data
        raw = torch.empty((M, nraw), device=h.device, dtype=torch.float32)
        check(L.m3d_gemm_f32_ex(ptr(h2), self.fc, 0, ptr(wcat), 0, ptr(raw), 0, 1, M, self.fc, nraw,
                                ptr(bcat), 0, 0, stream()), "class dense")
        logits = torch.empty((B, N, C), device=h.device, dtype=torch.float32)
        probs = torch.empty_like(logits)
        bbox = torch.empty((B, N, C, 6), device=h.device, dtype=torch.float32)
        check(L.m3d_head_outputs(ptr(raw), M, nraw, C, ptr(logits), ptr(probs), ptr(bbox), stream()),
              "head_outputs")
        return logits, probs, bbox


class MaskHead:
    """build_fpn_mask_graph(y, num_classes, conv_channel, train_bn=False)."""

    def __init__(self, store, num_classes, conv_channel, channels=256):
        ch = conv_channel
        self.C, self.ch = num_classes, ch
        self.convs = {}
        cin = channels
        for name in ("conv1", "conv2", "conv3", "conv3b", "conv4"):
            self.convs[name] = (ConvLayer(store, f"mrcnn_mask_{name}", (3, 3, 3), cin, ch),
                                BNLayer(store, f"mrcnn_mask_bn{name[4:]}", ch))
            cin = ch
        self.deconv = store.add("mrcnn_mask_deconv/kernel:0", (2, 2, 2, ch, ch), "glorot_uniform", True)
        self.deconv_b = store.add("mrcnn_mask_deconv/bias:0", (ch,), "zeros", True)
        self.mask = ConvLayer(store, "mrcnn_mask", (1, 1, 1), ch, num_classes)

    def _same(self, x, name, **kw):
        layer, bn = self.convs[name]
        geo = conv_geom(tuple(x.shape[1:4]), (3, 3, 3), (1, 1, 1), "same")
        return conv_bn_act(x, layer, geo, True, bn=bn, need_dx=False, **kw)

    def __call__(self, pooled):
        B, N, ph, pw, pd, Cin = pooled.shape
        L = _L()
        x = pooled.reshape(B * N, ph, pw, pd, Cin).contiguous()
        M = B * N
        x = self._same(x, "conv1")
        x = self._same(x, "conv2")
        res = self._same(x, "conv3")
        # x = res + relu(bn(conv3b_dilated(res)))   (mrcnn_mask_res3, post-activation Add)
        layer, bn = self.convs["conv3b"]
        scale, shift = _bn_affine(bn)
        x = torch.empty_like(res)
        check(L.m3d_conv3d_fwd_dil(ptr(res), M, ph, pw, pd, self.ch, ptr(layer.kernel.data), 3, 3, 3, self.ch,
                                   ph, pw, pd, 1, 1, 1, 2, 2, 2, 2, 2, 2, ptr(layer.bias.data), ptr(scale),
                                   ptr(shift), ptr(res), 3, 1, None, ptr(x), self.ch, None, 0, 0, stream()),
              "mask_conv3b")
        x = self._same(x, "conv4")
        up = torch.empty((M, 2 * ph, 2 * pw, 2 * pd, self.ch), device=x.device, dtype=torch.float32)
        check(L.m3d_deconv3d_k2s2(ptr(x), M, ph, pw, pd, self.ch, ptr(self.deconv.data), self.ch,
                                  ptr(self.deconv_b.data), 1, ptr(up), stream()), "mask_deconv")
        C = self.C
        cp = -(-C // 4) * 4
        w = torch.zeros((self.ch, cp), device=x.device, dtype=torch.float32)
        w[:, :C] = self.mask.kernel.data.reshape(self.ch, C)
        b = torch.zeros((cp,), device=x.device, dtype=torch.float32)
        b[:C] = self.mask.bias.data
        out = torch.empty((B, N, 2 * ph, 2 * pw, 2 * pd, C), device=x.device, dtype=torch.float32)
        spill = torch.empty((M * 8 * ph * pw * pd, max(cp - C, 1)), device=x.device, dtype=torch.float32)
        V = M * 8 * ph * pw * pd
        check(L.m3d_conv3d_fwd(ptr(up), 1, 1, 1, V, self.ch, ptr(w), 1, 1, 1, cp, 1, 1, V, 1, 1, 1, 0, 0, 0,
                               ptr(b), None, None, None, 0, 2, None, ptr(out), C, ptr(spill), cp - C,
                               C if cp > C else 0, stream()), "mrcnn_mask")
        return out


class DetectionLayer:
    """DetectionLayer(bbox_std_dev, detection_min_confidence,
    detection_max_instances, detection_nms_threshold, images_per_gpu)
    ([rois, mrcnn_class, mrcnn_bbox, image_meta]) -> [B, max_inst, 8]."""

    def __init__(self, bbox_std_dev, detection_min_confidence, detection_max_instances,
                 detection_nms_threshold, images_per_gpu, *args, name="mrcnn_detection", **kwargs):
        self.std = [float(v) for v in bbox_std_dev]
        self.min_conf = float(detection_min_confidence)
        self.max_inst = int(detection_max_instances)
        self.nms_thr = float(detection_nms_threshold)
        self.images_per_gpu = int(images_per_gpu)
        self.name = name

    def __call__(self, inputs):
        rois, probs, deltas, meta = inputs
        ops._dev(rois, probs, deltas, meta)
        L = _L()
        B, N = rois.shape[:2]
        C = probs.shape[-1]
        dev = rois.device
        det = torch.empty((B, self.max_inst, 8), device=dev, dtype=torch.float32)
        sd = (_lib.c_f * 6)(*[float(np.float32(v)) for v in self.std])
        with torch.no_grad():
            for b in range(B):
                r, p, d = (t[b].detach().float().contiguous() for t in (rois, probs, deltas))
                m = meta[b].detach().float().contiguous()
                bpx = torch.empty((N, 6), device=dev, dtype=torch.float32)
                b2d = torch.empty((N, 4), device=dev, dtype=torch.float32)
                sc = torch.empty((N,), device=dev, dtype=torch.float32)
                check(L.m3d_refine_detections(ptr(r), ptr(p), ptr(d), N, C, ptr(m), sd, self.min_conf,
                                              ptr(bpx), ptr(b2d), ptr(sc), stream()), "refine_detections")
                keep, num = ops.non_max_suppression_3d_padded(b2d, sc, self.max_inst, self.nms_thr, mode="2d")
                check(L.m3d_detections_gather(ptr(bpx), ptr(sc), ptr(keep), ptr(num), self.max_inst, ptr(m),
                                              det[b].data_ptr(), stream()), "detections_gather")
        return det

    def compute_output_shape(self, input_shape):
        return (None, self.max_inst, 8)


class MaskRCNN:
    """MaskRCNN(mode="inference") of the reference on a flat ParamStore:
    detect(image, image_meta) -> detections [B,max_inst,8], mrcnn_class,
    mrcnn_bbox, mrcnn_mask [B,max_inst,2M,2M,2M,C], rpn_rois."""

    def __init__(self, config, device="cuda", seed=1):
        anchors = model_anchors(config, inplace=False)  # patched copy + row-count check (m3d.anchors)
        _lib.load()
        self.config = c = config
        self.device = torch.device(device)
        self.store = ParamStore()
        self.backbone = ResNet3D(self.store, c.BACKBONE, stage5=True, train_bn=c.TRAIN_BN)
        self.fpn = FPN(self.store, c.TOP_DOWN_PYRAMID_SIZE)
        self.rpn = RPNHead(self.store, c.RPN_ANCHOR_STRIDE, len(c.RPN_ANCHOR_RATIOS), c.TOP_DOWN_PYRAMID_SIZE)
        fc = int(getattr(c, "FPN_CLASSIF_FC_LAYERS_SIZE", 512))
        mask_ch = int(getattr(c, "HEAD_CONV_CHANNEL", 256))
        self.classifier = ClassifierHead(self.store, c.POOL_SIZE, c.NUM_CLASSES, fc, c.TOP_DOWN_PYRAMID_SIZE)
        self.mask_head = MaskHead(self.store, c.NUM_CLASSES, mask_ch, c.TOP_DOWN_PYRAMID_SIZE)
        self.store.finalize(self.device, seed=seed)
        self.anchors = torch.from_numpy(anchors).to(self.device)[None]
        self.proposal_layer = ProposalLayer(
            proposal_count=c.POST_NMS_ROIS_INFERENCE, nms_threshold=c.RPN_NMS_THRESHOLD,
            pre_nms_limit=c.PRE_NMS_LIMIT, images_per_gpu=c.IMAGES_PER_GPU,
            rpn_bbox_std_dev=c.RPN_BBOX_STD_DEV, image_depth=c.IMAGE_DEPTH, name="ROI")
        self.roi_align_classifier = PyramidROIAlign([c.POOL_SIZE] * 3, name="roi_align_classifier")
        self.roi_align_mask = PyramidROIAlign([c.MASK_POOL_SIZE] * 3, name="roi_align_mask")
        self.detection = DetectionLayer(c.BBOX_STD_DEV, float(c.DETECTION_MIN_CONFIDENCE),
                                        int(c.DETECTION_MAX_INSTANCES), float(c.DETECTION_NMS_THRESHOLD),
                                        int(c.IMAGES_PER_GPU), name="mrcnn_detection")

    def load_weights(self, filepath, by_name=True, skip_mismatch=False, exclude=()):
        """keras_model.load_weights(filepath, by_name=True, ...) on the Keras-H5 format (m3d.weights)."""
        from .weights import load_weights
        return load_weights(self.store, filepath, by_name=by_name, skip_mismatch=skip_mismatch, exclude=exclude)

    def save_weights(self, filepath):
        """keras_model.save_weights(filepath): Keras-H5 layout, readable by the reference."""
        from .weights import save_weights
        save_weights(self.store, filepath)

    @torch.no_grad()
    def detect(self, image, image_meta):
        _, C2, C3, C4, C5 = self.backbone(image)
        fmaps = self.fpn(C2, C3, C4, C5)
        _, rpn_probs, rpn_bbox = self.rpn(fmaps)
        rpn_rois = self.proposal_layer([rpn_probs, rpn_bbox, self.anchors])
        mrcnn_maps = fmaps[:4]
        pooled = self.roi_align_classifier([rpn_rois, image_meta] + mrcnn_maps)
        _, mrcnn_class, mrcnn_bbox = self.classifier(pooled)
        detections = self.detection([rpn_rois, mrcnn_class, mrcnn_bbox, image_meta])
        mpooled = self.roi_align_mask([detections[..., :6].contiguous(), image_meta] + mrcnn_maps)
        mrcnn_mask = self.mask_head(mpooled)
        return {"detections": detections, "mrcnn_class": mrcnn_class, "mrcnn_bbox": mrcnn_bbox,
                "mrcnn_mask": mrcnn_mask, "rpn_rois": rpn_rois, "feature_maps": fmaps,
                "pooled": pooled, "mask_pooled": mpooled, "rpn_class": rpn_probs, "rpn_bbox": rpn_bbox}
