"""ResNet-3D backbone, FPN and RPN head on the libm3d kernels.

Structure and layer names follow the reference exactly:
  resnet_graph / conv_block / identity_block / BatchNorm  core/models.py:102-273
  FPN top-down + smoothing + P6                             core/models.py:3190-3214
  rpn_graph / build_rpn_model                               core/models.py:512-584
Depth is never strided (all strides (2,2,1)), BN runs in inference mode with
trainable gamma/beta (TRAIN_BN=False), every conv has a bias.
"""
from __future__ import annotations

import torch

from .nn import BNFuse, GradLink, _RPNOut, conv_bn_act, conv_geom, max_pool3d, subsample221
from .params import BNLayer, ConvLayer

# the RPN head's shared conv transforms its weights once per pass for all
# pyramid levels (False: once per level, A/B; tests/test_gpu_determinism.py)
SHARE_WINO_WEIGHTS = True


class _Unit:
    """Conv3D + BatchNorm pair with its geometry chosen at call time."""

    def __init__(self, store, conv_name, bn_name, k, cin, cout, stride, padding):
        self.conv = ConvLayer(store, conv_name, k, cin, cout)
        self.bn = BNLayer(store, bn_name, cout)
        self.stride, self.padding = tuple(stride), padding

    def __call__(self, x, relu, residual=None, need_dx=True, link=None, fuse=None, fuse_in=None):
        geo = conv_geom(tuple(x.shape[1:4]), self.conv.k, self.stride, self.padding)
        return conv_bn_act(x, self.conv, geo, relu, residual=residual,
                           res_mode=1 if residual is not None else 0, bn=self.bn, need_dx=need_dx,
                           link=link, fuse=fuse, fuse_in=fuse_in)


class _Block:
    """conv_block (shortcut conv) or identity_block (core/models.py:157-232)."""

    def __init__(self, store, cin, filters, stage, block, strides, shortcut):
        f1, f2, f3 = filters
        c, b = f"res{stage}{block}_branch", f"bn{stage}{block}_branch"
        self.a = _Unit(store, c + "2a", b + "2a", (1, 1, 1), cin, f1, strides, "valid")
        self.b = _Unit(store, c + "2b", b + "2b", (3, 3, 3), f1, f2, (1, 1, 1), "same")
        self.c = _Unit(store, c + "2c", b + "2c", (1, 1, 1), f2, f3, (1, 1, 1), "valid")
        self.sc = _Unit(store, c + "1", b + "1", (1, 1, 1), cin, f3, strides, "valid") if shortcut else None

    def __call__(self, x, links=None, fuse_in=None, fuse_out=None, fuses=None):
        """``fuse_in``: the BNFuse of the unit that made x, when this block is
        x's only consumer (an identity block inside a stage: its 2a data
        gradient, after the GradLink summed 2c's residual gradient, is x's whole
        gradient); ``fuse_out``: this block's output unit's BNFuse for the next."""
        # the two gradients of x are summed by the bwd-data kernel (GradLink)
        # instead of an autograd add: identity block 2c's residual gradient
        # into 2a's data gradient; conv block shortcut's and 2a's data gradients
        x = x.contiguous()
        train = torch.is_grad_enabled() and x.requires_grad
        # 2a -> 2b -> 2c: each unit's output has one consumer, whose data
        # gradient applies its BN-ReLU backward (nn.BNFuse)
        fa, fb = (BNFuse(fuses), BNFuse(fuses)) if train else (None, None)
        if self.sc is None:
            link = GradLink("res", x, links) if train else None
            y = self.a(x, relu=True, link=link, fuse=fa, fuse_in=fuse_in)
            y = self.b(y, relu=True, fuse=fb, fuse_in=fa)
            return self.c(y, relu=True, residual=x, link=link, fuse=fuse_out, fuse_in=fb)
        link = GradLink("dx2", x, links) if train else None
        short = self.sc(x, relu=False, link=link, fuse_in=fuse_in)
        y = self.a(x, relu=True, link=link, fuse=fa, fuse_in=fuse_in)
        y = self.b(y, relu=True, fuse=fb, fuse_in=fa)
        return self.c(y, relu=True, residual=short, fuse=fuse_out, fuse_in=fb)


BN_AFFINE_BATCHED = True


class ResNet3D:
    """resnet_graph(input_image, architecture, stage5, train_bn) -> [C1..C5]."""

    def __init__(self, store, architecture="resnet50", stage5=True, train_bn=False):
        assert architecture in ("resnet50", "resnet101")
        if train_bn:
            raise NotImplementedError("TRAIN_BN=True (batch-statistics BN) is not on the hot path")
        self.store = store
        self.stem = _Unit(store, "conv1", "bn_conv1", (7, 7, 7), 1, 64, (2, 2, 1), 3)
        s = (2, 2, 1)
        self.stages = []
        spec = [(2, [64, 64, 256], 3, (1, 1, 1)), (3, [128, 128, 512], 4, s),
                (4, [256, 256, 1024], {"resnet50": 6, "resnet101": 23}[architecture], s)]
        if stage5:
            spec.append((5, [512, 512, 2048], 3, s))
        cin = 64
        for stage, filters, n, strides in spec:
            blocks = [_Block(store, cin, filters, stage, "a", strides, True)]
            for i in range(n - 1):
                blocks.append(_Block(store, filters[2], filters, stage, chr(98 + i), (1, 1, 1), False))
            cin = filters[2]
            self.stages.append(blocks)
        self.stage5 = stage5
        self.links = []
        self.fuses = []

    def __call__(self, image):
        self.links = []                 # GradLinks of this forward (checked by check_links)
        self.fuses = []                 # BNFuse records of this forward (checked by check_fuses)
        # every BN layer's affine in one launch for this forward (ParamStore.bn_affine_refresh;
        # BN_AFFINE_BATCHED False: one m3d_bn_affine per BN conv unit, A/B)
        if not BN_AFFINE_BATCHED:
            return self._forward(image)
        self.store.bn_aff_live = self.store.bn_affine_refresh()
        try:
            return self._forward(image)
        finally:
            self.store.bn_aff_live = False

    def _forward(self, image):
        x = self.stem(image, relu=True, need_dx=False)
        c1 = x = max_pool3d(x, (3, 3, 3), (2, 2, 1), "same")
        outs = [c1]
        train = torch.is_grad_enabled() and x.requires_grad
        for blocks in self.stages:
            # a block output feeding the next block of its stage has that block
            # as its only consumer; a stage's last output also feeds the FPN
            fuse = None
            for i, blk in enumerate(blocks):
                nxt = BNFuse(self.fuses) if train and i + 1 < len(blocks) else None
                x = blk(x, self.links, fuse_in=fuse, fuse_out=nxt, fuses=self.fuses)
                fuse = nxt
            outs.append(x)
        if not self.stage5:
            outs.append(None)
        return outs


def resnet_graph(input_image, architecture, stage5=False, train_bn=False, store=None, model=None):
    """Functional form of the reference's resnet_graph; pass a built ResNet3D as ``model``."""
    if model is None:
        raise ValueError("resnet_graph needs a ResNet3D built on a ParamStore (model=...)")
    return model(input_image)


class FPN:
    """Top-down pathway of RPN.build (core/models.py:3190-3214)."""

    def __init__(self, store, size=256, c_channels=(256, 512, 1024, 2048)):
        c2, c3, c4, c5 = c_channels
        self.c5p5 = ConvLayer(store, "fpn_c5p5", (1, 1, 1), c5, size)
        self.c4p4 = ConvLayer(store, "fpn_c4p4", (1, 1, 1), c4, size)
        self.c3p3 = ConvLayer(store, "fpn_c3p3", (1, 1, 1), c3, size)
        self.c2p2 = ConvLayer(store, "fpn_c2p2", (1, 1, 1), c2, size)
        self.p = [ConvLayer(store, f"fpn_p{i}", (3, 3, 3), size, size) for i in (2, 3, 4, 5)]

    @staticmethod
    def _c(x, layer, k, padding, residual=None):
        geo = conv_geom(tuple(x.shape[1:4]), k, (1, 1, 1), padding)
        return conv_bn_act(x, layer, geo, relu=False, residual=residual,
                           res_mode=2 if residual is not None else 0)

    def __call__(self, C2, C3, C4, C5):
        P5 = self._c(C5, self.c5p5, (1, 1, 1), "valid")
        P4 = self._c(C4, self.c4p4, (1, 1, 1), "valid", residual=P5)   # up(P5) + c4p4(C4)
        P3 = self._c(C3, self.c3p3, (1, 1, 1), "valid", residual=P4)
        P2 = self._c(C2, self.c2p2, (1, 1, 1), "valid", residual=P3)
        P2, P3, P4, P5 = (self._c(x, l, (3, 3, 3), "same") for x, l in zip((P2, P3, P4, P5), self.p))
        P6 = subsample221(P5)
        return [P2, P3, P4, P5, P6]


class RPNHead:
    """build_rpn_model(anchor_stride, anchors_per_location, channel): one shared
    head applied to every pyramid level (core/models.py:512-584)."""

    def __init__(self, store, anchor_stride, anchors_per_location, channel, backbone=None):
        if anchor_stride != 1:
            raise NotImplementedError("RPN_ANCHOR_STRIDE != 1")
        self.apl = anchors_per_location
        self.shared1 = ConvLayer(store, "rpn_conv_shared1", (3, 3, 3), channel, 512)
        self.shared2 = ConvLayer(store, "rpn_conv_shared2", (1, 1, 1), 512, 256)
        self.cls = ConvLayer(store, "rpn_class_raw", (1, 1, 1), 256, 2 * self.apl)
        self.bbox = ConvLayer(store, "rpn_bbox_pred", (1, 1, 1), 256, 6 * self.apl,
                              kernel_init=("normal", 0.001))
        self.w_grad = None
        self.b_grad = None
        self.backbone = backbone        # its GradLinks / BNFuse records are checked in finish_backward
        self.fuse_records = []

    def __call__(self, feature_maps):
        shared, fuses = [], []
        self.fuse_records = []
        # rpn_conv_shared1 is one kernel on every level: its Winograd weight
        # transform is done once per pass (forward and data gradient) and reused
        wshare = {} if SHARE_WINO_WEIGHTS else None
        for p in feature_maps:
            g1 = conv_geom(tuple(p.shape[1:4]), (3, 3, 3), (1, 1, 1), "same")
            # shared1 -> shared2 -> the class / bbox heads: sole consumers (nn.BNFuse)
            f1, f2 = (BNFuse(self.fuse_records), BNFuse(self.fuse_records)) if torch.is_grad_enabled() \
                else (None, None)
            s = conv_bn_act(p, self.shared1, g1, relu=True, wshare=wshare, fuse=f1)
            g2 = conv_geom(tuple(s.shape[1:4]), (1, 1, 1), (1, 1, 1), "valid")
            shared.append(conv_bn_act(s, self.shared2, g2, relu=True, fuse=f2, fuse_in=f1))
            fuses.append(f2)
        if wshare is not None:
            wshare.pop("fwd", None)        # the forward's workspace is not needed past the loop
        apl = self.apl
        cin = 256
        w24 = torch.cat([self.cls.kernel.data.reshape(cin, 2 * apl),
                         self.bbox.kernel.data.reshape(cin, 6 * apl)], dim=1).contiguous()
        b24 = torch.cat([self.cls.bias.data, self.bbox.bias.data]).contiguous()
        grads = None
        self.w_grad = self.b_grad = None           # a new forward drops any unfinished head gradient
        if torch.is_grad_enabled():
            npad = -(-8 * apl // 32) * 32
            self.w_grad = torch.zeros((cin, npad), device=w24.device, dtype=torch.float32)
            self.b_grad = torch.zeros((npad,), device=w24.device, dtype=torch.float32)
            grads = {"kernel": self.w_grad, "bias": self.b_grad}
        logits, bbox = _RPNOut.apply(w24, b24, grads, apl, tuple(fuses), *shared)
        probs = torch.softmax(logits, dim=-1)
        return logits, probs, bbox

    def finish_backward(self):
        """Join the side-stream weight gradients (m3d.nn.join_wgrad) and fold the
        padded combined-head gradients into rpn_class_raw / rpn_bbox_pred."""
        from .nn import WINO_V, check_fuses, check_links, join_wgrad
        batch, self.bias_batch = getattr(self, "bias_batch", None), None
        if batch is not None:
            batch.flush()          # the batched bias gradients (nn.BiasSums), on the compute stream
        join_wgrad()
        WINO_V.join()              # the Winograd weight pre-pass's side stream (nn.WinoVPrep)
        check_fuses(self.fuse_records)
        if self.backbone is not None:
            check_links(self.backbone.links)
            check_fuses(self.backbone.fuses)
        if self.w_grad is None:
            return
        apl, cin = self.apl, 256
        with torch.no_grad():
            self.cls.kernel.grad.view(cin, 2 * apl).add_(self.w_grad[:, :2 * apl])
            self.bbox.kernel.grad.view(cin, 6 * apl).add_(self.w_grad[:, 2 * apl:8 * apl])
            self.cls.bias.grad.add_(self.b_grad[:2 * apl])
            self.bbox.bias.grad.add_(self.b_grad[2 * apl:8 * apl])
        self.w_grad = self.b_grad = None
