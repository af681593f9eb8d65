"""Flat parameter / gradient / momentum storage with Keras layer naming.

All trainable tensors are views into one fp32 device buffer (and the same for
gradients and SGD moments), each segment padded to whole 1024-float chunks, so
one memset zeroes every gradient and one fused kernel (m3d_sgd_keras) applies
the optimizer step.  Names follow the reference's Keras weights
("res2a_branch2a/kernel:0", "bn2a_branch2a/gamma:0", ...; H5 layout
core/models.py:5150-5188), so a Keras-H5 importer maps 1:1.
"""
from __future__ import annotations

import math

import numpy as np
import torch

CHUNK = 1024


class Param:
    def __init__(self, name, shape, init, l2):
        self.name, self.shape, self.init, self.l2 = name, tuple(shape), init, l2
        self.numel = int(np.prod(shape)) if len(shape) else 1
        self.offset = None
        self.data = None
        self.grad = None


class ConvLayer:
    def __init__(self, store, name, k, cin, cout, bias=True, kernel_init="glorot_uniform"):
        self.name, self.k, self.cin, self.cout = name, tuple(k), cin, cout
        self.kernel = store.add(f"{name}/kernel:0", (*self.k, cin, cout), kernel_init, True)
        self.bias = store.add(f"{name}/bias:0", (cout,), "zeros", True) if bias else None

    def grad_dict(self, bn=None):
        g = {"kernel": self.kernel.grad, "bias": self.bias.grad if self.bias is not None else None}
        if bn is not None:
            g["gamma"] = bn.gamma.grad
            g["beta"] = bn.beta.grad
        return g


class BNLayer:
    """Keras BatchNormalization in inference mode (TRAIN_BN=False): frozen
    moving statistics, trainable gamma/beta, epsilon 1e-3."""

    def __init__(self, store, name, c, eps=1e-3):
        self.name, self.c, self.eps = name, c, eps
        self.store = store
        self.aff = None            # [3, c] (rstd, scale, shift) of ParamStore.bn_affine_refresh
        self.gamma = store.add(f"{name}/gamma:0", (c,), "ones", False)
        self.beta = store.add(f"{name}/beta:0", (c,), "zeros", False)
        self.moving_mean = None
        self.moving_variance = None
        store.bns.append(self)


class ParamStore:
    def __init__(self):
        self.params: list[Param] = []
        self.bns: list[BNLayer] = []
        # every BN layer's affine from one launch (bn_affine_refresh); the views
        # bn.aff are current while bn_aff_live is set (a model forward's span)
        self._bn_items = self._bn_key = None
        self.bn_aff_live = False
        self.bn_gen = 0            # refreshes of the shared affine buffer (nn._check_generations)
        self.by_name = {}
        self.flat = self.grad_flat = self.moments = None

    def add(self, name, shape, init, l2):
        p = Param(name, shape, init, l2)
        if name in self.by_name:
            raise ValueError(f"duplicate parameter {name}")
        self.params.append(p)
        self.by_name[name] = p
        return p

    def finalize(self, device, seed=1, weight_decay=0.0):
        off = 0
        for p in self.params:
            p.offset = off
            off += -(-p.numel // CHUNK) * CHUNK
        self.total = off
        self.n_chunks = off // CHUNK
        flat = torch.zeros(off, dtype=torch.float32)
        g = torch.Generator().manual_seed(seed)
        for p in self.params:
            v = flat[p.offset:p.offset + p.numel].view(p.shape)
            if p.init == "zeros":
                v.zero_()
            elif p.init == "ones":
                v.fill_(1.0)
            elif p.init == "glorot_uniform":
                rf = int(np.prod(p.shape[:-2])) if len(p.shape) > 2 else 1
                fan_in, fan_out = p.shape[-2] * rf, p.shape[-1] * rf
                lim = math.sqrt(6.0 / (fan_in + fan_out))
                v.uniform_(-lim, lim, generator=g)
            elif isinstance(p.init, tuple) and p.init[0] == "normal":
                v.normal_(0.0, p.init[1], generator=g)
            elif isinstance(p.init, tuple) and p.init[0] == "const":
                v.copy_(torch.as_tensor(p.init[1], dtype=torch.float32).reshape(p.shape))
            else:
                raise ValueError(p.init)
        self.flat = flat.to(device).requires_grad_(True)
        self.grad_flat = torch.zeros(off, dtype=torch.float32, device=device)
        self.moments = torch.zeros(off, dtype=torch.float32, device=device)
        seg = np.zeros(self.n_chunks, np.int32)
        l2 = np.zeros(len(self.params), np.float32)
        for i, p in enumerate(self.params):
            c0 = p.offset // CHUNK
            seg[c0:c0 + -(-p.numel // CHUNK)] = i
            l2[i] = weight_decay / p.numel if p.l2 else 0.0
        self.seg_of_chunk = torch.from_numpy(seg).to(device)
        self.l2_coef = torch.from_numpy(l2).to(device)
        self.norms = torch.zeros(len(self.params), dtype=torch.float32, device=device)
        for p in self.params:
            p.data = self.flat[p.offset:p.offset + p.numel].view(p.shape)
            p.grad = self.grad_flat[p.offset:p.offset + p.numel].view(p.shape)
        for bn in self.bns:
            bn.moving_mean = torch.zeros(bn.c, dtype=torch.float32, device=device)
            bn.moving_variance = torch.ones(bn.c, dtype=torch.float32, device=device)
        return self

    def zero_grad(self):
        self.grad_flat.zero_()

    def bn_affine_refresh(self):
        """(rstd, scale, shift) of every BN layer into bn.aff by ONE launch of
        m3d_bn_affine_batched on the current stream (was one m3d_bn_affine per
        BN conv unit per forward).  The descriptor table is built once and
        rebuilt if any parameter / statistics buffer moved.  Returns whether
        bn.aff is current: under HIP-graph capture a missing / stale table
        cannot be rebuilt (a pageable host-to-device copy), so the forward then
        runs each unit's own m3d_bn_affine instead (as X3Planes.refresh)."""
        from . import _lib
        import torch
        if not self.bns:
            return False
        key = tuple((bn.gamma.data.data_ptr(), bn.beta.data.data_ptr(), bn.moving_mean.data_ptr(),
                     bn.moving_variance.data_ptr()) for bn in self.bns)
        if (self._bn_items is None or key != self._bn_key) and torch.cuda.is_current_stream_capturing():
            return False
        if self._bn_items is None or key != self._bn_key:
            dev = self.bns[0].gamma.data.device
            total = sum(3 * bn.c for bn in self.bns)
            self._bn_out = torch.empty(total, dtype=torch.float32, device=dev)
            items = (_lib.BnAffineItem * len(self.bns))()
            off = 0
            for i, bn in enumerate(self.bns):
                bn.aff = self._bn_out[off:off + 3 * bn.c].view(3, bn.c)
                items[i] = _lib.BnAffineItem(bn.gamma.data.data_ptr(), bn.beta.data.data_ptr(),
                                             bn.moving_mean.data_ptr(), bn.moving_variance.data_ptr(),
                                             bn.aff.data_ptr(), float(bn.eps), int(bn.c))
                off += 3 * bn.c
            host = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8)
            self._bn_items = host.to(dev)
            self._bn_key = key
            self._bn_max_c = max(bn.c for bn in self.bns)
        L = _lib.load()
        _lib.check(L.m3d_bn_affine_batched(self._bn_items.data_ptr(), len(self.bns), self._bn_max_c,
                                           _lib.stream()), "bn_affine_batched")
        self.bn_gen += 1
        return True

    def state_dict(self):
        d = {p.name: p.data.detach().cpu().clone() for p in self.params}
        for bn in self.bns:
            d[f"{bn.name}/moving_mean:0"] = bn.moving_mean.cpu().clone()
            d[f"{bn.name}/moving_variance:0"] = bn.moving_variance.cpu().clone()
        return d

    def load_state_dict(self, d, strict=True):
        with torch.no_grad():
            for p in self.params:
                if p.name in d:
                    p.data.copy_(torch.as_tensor(d[p.name]).reshape(p.shape))
                elif strict:
                    raise KeyError(p.name)
            for bn in self.bns:
                for attr in ("moving_mean", "moving_variance"):
                    k = f"{bn.name}/{attr}:0"
                    if k in d:
                        getattr(bn, attr).copy_(torch.as_tensor(d[k]))
