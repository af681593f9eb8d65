"""CPU restatement (oracle) of the backbone / FPN / RPN graph and RPN losses.

TEST INFRASTRUCTURE ONLY (see oracle/ops_ref.py header); the product never
imports it.  PyTorch-CPU (float64 by default) with explicit Keras/TF
conventions, written from the reference's source text:

* Conv3D channels-last, kernel [kh,kw,kd,Cin,Cout], 'same' = TF SAME padding,
  'valid', ZeroPadding3D(3) for the stem  (core/models.py:157-273)
* BatchNormalization inference mode, eps 1e-3: x*inv + (beta - mean*inv),
  inv = rsqrt(var+eps)*gamma                 (core/models.py:102-114)
* MaxPooling3D SAME (asymmetric: extra pad after)   (core/models.py:245)
* FPN nearest (2,2,1) upsampling + add, 3x3x3 smoothing, P6 = P5[::2, ::2]
                                             (core/models.py:3190-3214)
* RPN head conv 3^3 512 relu, 1^3 256 relu, class 2A / bbox 6A, reshape
  (y,x,z,a) and concat over P2..P6           (core/models.py:512-584, 3250-3263)
* rpn_class_loss / rpn_bbox_loss             (core/models.py:1589-1673)

Parity status for this file: "parity unpinned" -- TF/Keras are absent and the
reference may not be executed here; the conventions above are restated from
the source and checked against analytic cases in tests/test_oracle.py.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F


def _same(n, k, s):
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return total // 2, total - total // 2


def conv3d(x, w, b=None, stride=(1, 1, 1), padding="same"):
    """x [B,H,W,D,C], w [kh,kw,kd,Cin,Cout] -> [B,OH,OW,OD,Cout]."""
    k = w.shape[:3]
    xt = x.permute(0, 4, 1, 2, 3)
    if padding == "same":
        pads = [_same(n, kk, s) for n, kk, s in zip(x.shape[1:4], k, stride)]
    elif padding == "valid":
        pads = [(0, 0)] * 3
    else:
        p = int(padding)
        pads = [(p, p)] * 3
    fp = []
    for lo, hi in reversed(pads):
        fp += [lo, hi]
    xt = F.pad(xt, fp)
    wt = w.permute(4, 3, 0, 1, 2)
    y = F.conv3d(xt, wt, None, stride=tuple(stride))
    y = y.permute(0, 2, 3, 4, 1)
    if b is not None:
        y = y + b
    return y


def batchnorm(x, gamma, beta, mean, var, eps=1e-3):
    inv = torch.rsqrt(var + eps) * gamma
    return x * inv + (beta - mean * inv)


def maxpool3d_same(x, k=(3, 3, 3), stride=(2, 2, 1)):
    xt = x.permute(0, 4, 1, 2, 3)
    fp = []
    for n, kk, s in reversed(list(zip(x.shape[1:4], k, stride))):
        lo, hi = _same(n, kk, s)
        fp += [lo, hi]
    xt = F.pad(xt, fp, value=-math.inf)
    y = F.max_pool3d(xt, k, stride)
    return y.permute(0, 2, 3, 4, 1)


def upsample221(x):
    return x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2)


class RefRPN:
    """Functional restatement driven by a {keras_name: tensor} dict."""

    def __init__(self, params, architecture="resnet50", dtype=torch.float64, apl=3, relu_masks=None):
        """relu_masks: {layer name: [bool mask per call]} (m3d.nn.RELU_CAPTURE of
        a GPU forward): each ReLU then takes the branches recorded there
        (y * mask) instead of deciding them in this precision, so gradients
        are compared on the same piecewise-linear branch."""
        self.p = {k: torch.as_tensor(np.asarray(v)).to(dtype) for k, v in params.items()}
        self.dtype = dtype
        self.arch = architecture
        self.apl = apl
        self.relu_masks = relu_masks
        self._calls = {}

    def _cb(self, x, conv, bn, stride=(1, 1, 1), padding="valid", relu=True, res=None):
        p = self.p
        y = conv3d(x, p[f"{conv}/kernel:0"], p[f"{conv}/bias:0"], stride, padding)
        if bn is not None:
            y = batchnorm(y, p[f"{bn}/gamma:0"], p[f"{bn}/beta:0"], p[f"{bn}/moving_mean:0"],
                          p[f"{bn}/moving_variance:0"])
        if res is not None:
            y = y + res
        if relu and self.relu_masks is not None:
            i = self._calls.get(conv, 0)
            self._calls[conv] = i + 1
            m = self.relu_masks[conv][i]
            if tuple(m.shape) != tuple(y.shape):
                raise ValueError(f"relu mask of {conv} call {i}: {tuple(m.shape)} vs {tuple(y.shape)}")
            return y * m.to(y.dtype)
        return torch.relu(y) if relu else y

    def _block(self, x, stage, block, strides, shortcut):
        c, b = f"res{stage}{block}_branch", f"bn{stage}{block}_branch"
        y = self._cb(x, c + "2a", b + "2a", strides)
        y = self._cb(y, c + "2b", b + "2b", padding="same")
        sc = self._cb(x, c + "1", b + "1", strides, relu=False) if shortcut else x
        return self._cb(y, c + "2c", b + "2c", res=sc)

    def backbone(self, image):
        x = self._cb(image, "conv1", "bn_conv1", (2, 2, 1), padding=3)
        x = maxpool3d_same(x)
        outs = [x]
        n4 = {"resnet50": 6, "resnet101": 23}[self.arch]
        for stage, n, s in ((2, 3, (1, 1, 1)), (3, 4, (2, 2, 1)), (4, n4, (2, 2, 1)), (5, 3, (2, 2, 1))):
            x = self._block(x, stage, "a", s, True)
            for i in range(n - 1):
                x = self._block(x, stage, chr(98 + i), (1, 1, 1), False)
            outs.append(x)
        return outs

    def fpn(self, C2, C3, C4, C5):
        cb = lambda x, n, pad="valid": self._cb(x, n, None, padding=pad, relu=False)  # noqa: E731
        P5 = cb(C5, "fpn_c5p5")
        P4 = upsample221(P5) + cb(C4, "fpn_c4p4")
        P3 = upsample221(P4) + cb(C3, "fpn_c3p3")
        P2 = upsample221(P3) + cb(C2, "fpn_c2p2")
        P2, P3, P4, P5 = (cb(x, f"fpn_p{i}", "same") for x, i in zip((P2, P3, P4, P5), (2, 3, 4, 5)))
        P6 = P5[:, ::2, ::2]
        return [P2, P3, P4, P5, P6]

    def rpn_head(self, fmaps):
        logits, bbox = [], []
        for f in fmaps:
            s = self._cb(f, "rpn_conv_shared1", None, padding="same")
            s = self._cb(s, "rpn_conv_shared2", None)
            lg = self._cb(s, "rpn_class_raw", None, relu=False)
            bb = self._cb(s, "rpn_bbox_pred", None, relu=False)
            logits.append(lg.reshape(lg.shape[0], -1, 2))
            bbox.append(bb.reshape(bb.shape[0], -1, 6))
        logits = torch.cat(logits, 1)
        return logits, torch.softmax(logits, -1), torch.cat(bbox, 1)

    def forward(self, image):
        self._calls = {}
        _, C2, C3, C4, C5 = self.backbone(image)
        fm = self.fpn(C2, C3, C4, C5)
        logits, probs, bbox = self.rpn_head(fm)
        return {"feature_maps": fm, "rpn_class_logits": logits, "rpn_class": probs, "rpn_bbox": bbox,
                "C": (C2, C3, C4, C5)}


def rpn_class_loss(rpn_match, logits, alpha=0.90, gamma=1.5):
    m = rpn_match.reshape(-1)
    idx = torch.nonzero(m != 0)[:, 0]
    if idx.numel() == 0:
        return logits.sum() * 0
    lg = logits.reshape(-1, 2)[idx]
    labels = (m[idx] == 1).long()
    ce = F.cross_entropy(lg, labels, reduction="none")
    p_t = torch.softmax(lg, -1).gather(1, labels[:, None])[:, 0]
    ce = torch.pow(1.0 - p_t, gamma) * ce
    alpha_t = torch.where(labels == 1, torch.full_like(ce, alpha), torch.full_like(ce, 1 - alpha))
    return (alpha_t * ce).mean()


def rpn_bbox_loss(target_bbox, rpn_match, rpn_bbox):
    B = rpn_match.shape[0]
    m = rpn_match.reshape(B, -1)
    pos = torch.nonzero(m.reshape(-1) == 1)[:, 0]
    if pos.numel() == 0:
        return rpn_bbox.sum() * 0
    pred = rpn_bbox.reshape(-1, 6)[pos].clamp(-5, 5)
    counts = (m == 1).sum(1)
    gt = torch.cat([target_bbox[b, :counts[b]] for b in range(B)], 0)
    diff = (gt - pred).clamp(-2, 2)
    ad = diff.abs()
    xy = torch.tensor([1., 1., 0., 1., 1., 0.], dtype=diff.dtype)
    zm = torch.tensor([0., 0., 1., 0., 0., 1.], dtype=diff.dtype)
    h = torch.where(ad < 1.0, 0.5 * diff * diff, ad - 0.5) * xy + \
        torch.where(ad < 0.5, 0.5 * diff * diff, 0.5 * ad - 0.25) * zm
    return h.mean()
