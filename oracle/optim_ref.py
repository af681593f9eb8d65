"""TEST INFRASTRUCTURE ONLY (oracle): numpy restatement of the Keras 2.3.1
optimizer updates that RPN.compile builds (core/models.py:3349-3357, parameter
renaming core/models.py:117-125), applied per weight tensor with the RPN L2
term's gradient (core/models.py:3380-3384) and tf.clip_by_norm.

Keras 2.3.1 keras/optimizers.py (a pinned third-party dependency,
requirements.txt:4, absent here) -- the published update rules restated:
  SGD       v = momentum*v - lr*g;  p += v
  Adam      t = it+1; lr_t = lr*sqrt(1-b2^t)/(1-b1^t)
            m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g^2; p -= lr_t*m/(sqrt(v)+eps)
            (amsgrad: vhat = max(vhat, v) replaces v in the denominator)
  Adadelta  a = rho*a + (1-rho)*g^2; u = g*sqrt(d+eps)/sqrt(a+eps);
            p -= lr*u; d = rho*d + (1-rho)*u^2
  lr decays as lr/(1+decay*it) in every optimizer; eps defaults to 1e-7.
Only tests import this module.  Parity unpinned against the reference (it
cannot be run here); the formulas are pinned by hand-computed single-step
known answers in tests/test_host.py.
"""
import numpy as np

F = np.float32


def clip_by_norm(g, clipnorm):
    """tf.clip_by_norm (TF 2.2): t*clip / max(||t||, clip)."""
    if not clipnorm or clipnorm <= 0:
        return g
    n = np.sqrt(np.sum(g.astype(np.float64) ** 2))
    return (g * F(clipnorm) / F(max(n, clipnorm))).astype(F)


def step(kind, p, g, state, it, lr, decay=0.0, clipnorm=0.0, l2coef=0.0, **hp):
    """One Keras update of tensor p (float32) with raw gradient g.
    state: dict of slot arrays (created on first use).  Returns new p."""
    p = p.astype(F)
    g = clip_by_norm((g + F(l2coef) * p).astype(F), clipnorm)
    lr = F(lr)
    if decay > 0:
        lr = F(lr * (F(1) / (F(1) + F(decay) * F(it))))
    if kind == "SGD":
        v = state.setdefault("v", np.zeros_like(p))
        v[...] = F(hp.get("momentum", 0.0)) * v - lr * g
        return p + v
    eps = F(hp.get("epsilon") or 1e-7)
    if kind == "ADAM":
        b1, b2 = F(hp.get("beta_1", 0.9)), F(hp.get("beta_2", 0.999))
        t = F(it + 1)
        lr_t = F(lr * (np.sqrt(F(1) - np.power(b2, t)) / (F(1) - np.power(b1, t))))
        m = state.setdefault("m", np.zeros_like(p))
        v = state.setdefault("v", np.zeros_like(p))
        m[...] = b1 * m + (F(1) - b1) * g
        v[...] = b2 * v + (F(1) - b2) * (g * g)
        den = v
        if hp.get("amsgrad"):
            vh = state.setdefault("vhat", np.zeros_like(p))
            vh[...] = np.maximum(vh, v)
            den = vh
        return p - (lr_t * m) / (np.sqrt(den) + eps)
    if kind == "ADADELTA":
        rho = F(hp.get("rho", 0.95))
        a = state.setdefault("a", np.zeros_like(p))
        d = state.setdefault("d", np.zeros_like(p))
        a[...] = rho * a + (F(1) - rho) * (g * g)
        u = (g * np.sqrt(d + eps)) / np.sqrt(a + eps)
        d[...] = rho * d + (F(1) - rho) * (u * u)
        return p - lr * u
    raise ValueError(kind)
