"""Keras 2.3.1 optimizers of RPN.compile on the flat ParamStore buffers.

core/models.py:3349-3357 picks the optimizer by ``OPTIMIZER.name``: "SGD" ->
keras.optimizers.SGD, "ADADELTA" -> Adadelta, anything else -> Adam, with the
parameters renamed by ``_keras_opt_params`` (core/models.py:117-125:
learning_rate -> lr, beta1 -> beta_1, beta2 -> beta_2).  Each step is one fused
libm3d kernel over the whole flat buffer (plus the per-tensor clip-norm pass
when ``clipnorm`` is set); the scalar schedule (time decay of lr, Adam's bias
correction) is computed here in float32, as TF evaluates it in the graph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib

_F = np.float32
K_EPSILON = 1e-7          # keras.backend.epsilon()


def keras_opt_params(p):
    """core/models.py:117-125."""
    p = dict(p or {})
    if "learning_rate" in p and "lr" not in p:
        p["lr"] = p.pop("learning_rate")
    if "beta1" in p and "beta_1" not in p:
        p["beta_1"] = p.pop("beta1")
    if "beta2" in p and "beta_2" not in p:
        p["beta_2"] = p.pop("beta2")
    return p


class KerasOptimizer:
    """SGD / Adam / Adadelta with Keras 2.3.1 defaults and update formulas.

    ``iterations`` counts applied steps (Keras' ``self.iterations``)."""

    DEFAULTS = {
        "SGD": {"lr": 0.01, "momentum": 0.0, "nesterov": False},
        "ADAM": {"lr": 0.001, "beta_1": 0.9, "beta_2": 0.999, "epsilon": None, "amsgrad": False},
        "ADADELTA": {"lr": 1.0, "rho": 0.95, "epsilon": None},
    }

    def __init__(self, optimizer_cfg):
        cfg = dict(optimizer_cfg or {})
        name = str(cfg.get("name", "SGD")).upper()
        self.kind = name if name in ("SGD", "ADADELTA") else "ADAM"     # core/models.py:3352-3357
        p = keras_opt_params(cfg.get("parameters", {}))
        self.decay = float(p.pop("decay", 0.0))
        self.clipnorm = float(p.pop("clipnorm", 0.0) or 0.0)
        if p.pop("clipvalue", None) is not None:
            raise NotImplementedError("clipvalue is not used by any reference config")
        d = dict(self.DEFAULTS[self.kind])
        unknown = set(p) - set(d)
        if unknown:
            raise TypeError(f"Unexpected keyword argument(s) for {self.kind}: {sorted(unknown)}")
        d.update(p)
        if d.get("nesterov"):
            raise NotImplementedError("SGD nesterov=True")
        if "epsilon" in d and d["epsilon"] is None:
            d["epsilon"] = K_EPSILON
        self.params = d
        self.lr = float(d["lr"])
        self.iterations = 0
        self._state = None

    # -- schedule (float32, as the TF graph computes it) -----------------
    def current_lr(self):
        lr = _F(self.lr)
        if self.decay > 0:
            lr = lr * (_F(1.0) / (_F(1.0) + _F(self.decay) * _F(self.iterations)))
        return float(_F(lr))

    def adam_lr_t(self):
        t = _F(self.iterations + 1)
        b1, b2 = _F(self.params["beta_1"]), _F(self.params["beta_2"])
        lr = _F(self.current_lr())
        return float(_F(lr * (np.sqrt(_F(1.0) - np.power(b2, t)) / (_F(1.0) - np.power(b1, t)))))

    # -- state -----------------------------------------------------------
    def state(self, store):
        """Optimizer slots as flat buffers shaped like store.flat (the SGD
        velocity reuses store.moments)."""
        if self._state is None:
            n, dev = store.total, store.flat.device
            if self.kind == "SGD":
                self._state = [store.moments]
            elif self.kind == "ADAM":
                k = 3 if self.params["amsgrad"] else 2
                self._state = [store.moments] + [torch.zeros(n, dtype=torch.float32, device=dev)
                                                 for _ in range(k - 1)]
            else:
                self._state = [store.moments, torch.zeros(n, dtype=torch.float32, device=dev)]
        return self._state

    def step(self, store):
        from . import nn as mnn
        L = _lib.load()
        s = self.state(store)
        t0 = mnn._span()
        common = (store.n_chunks, store.seg_of_chunk.data_ptr(), store.l2_coef.data_ptr(), len(store.params))
        if self.kind == "SGD":
            rc = L.m3d_sgd_keras(store.flat.data_ptr(), store.grad_flat.data_ptr(), s[0].data_ptr(), *common,
                                 self.current_lr(), float(self.params["momentum"]), self.clipnorm,
                                 store.norms.data_ptr(), _lib.stream())
        elif self.kind == "ADAM":
            vhat = s[2].data_ptr() if len(s) > 2 else None
            rc = L.m3d_adam_keras(store.flat.data_ptr(), store.grad_flat.data_ptr(), s[0].data_ptr(),
                                  s[1].data_ptr(), vhat, *common, self.adam_lr_t(),
                                  float(self.params["beta_1"]), float(self.params["beta_2"]),
                                  float(self.params["epsilon"]), self.clipnorm, store.norms.data_ptr(),
                                  _lib.stream())
        else:
            rc = L.m3d_adadelta_keras(store.flat.data_ptr(), store.grad_flat.data_ptr(), s[0].data_ptr(),
                                      s[1].data_ptr(), *common, self.current_lr(), float(self.params["rho"]),
                                      float(self.params["epsilon"]), self.clipnorm, store.norms.data_ptr(),
                                      _lib.stream())
        _lib.check(rc, self.kind.lower())
        # compulsory bytes: read w, g and the slots, write w and the slots (+ the clip-norm read of g)
        nslot = len(s)
        mnn._log("optimizer", 0, 0, 4.0 * store.total * (2 + 2 * nslot + 1 + (self.clipnorm > 0)),
                 "optimizer", self.kind, t0)
        self.iterations += 1
