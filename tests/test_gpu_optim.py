"""GPU parity of the fused Keras optimizer kernels (m3d_sgd_keras,
m3d_adam_keras, m3d_adadelta_keras, driven by m3d.optim.KerasOptimizer)
against the numpy restatement oracle/optim_ref.py over several steps, with the
L2 term, per-tensor clip norms and lr time decay (core/models.py:3349-3384).
Tolerance: 1e-6 relative to the weight scale (float32 update arithmetic; the
clip norm's summation order differs)."""
import numpy as np
import pytest
import torch

from oracle import optim_ref as O

pytestmark = pytest.mark.gpu

CASES = [
    ("SGD", {"learning_rate": 0.05, "momentum": 0.9, "clipnorm": 5.0, "decay": 0.01}),
    ("ADAM", {"learning_rate": 0.01, "beta1": 0.85, "beta2": 0.99, "clipnorm": 2.0, "decay": 0.05}),
    ("ADAM", {"lr": 0.003, "amsgrad": True}),
    ("Nadam", {"learning_rate": 0.002}),            # any other name -> Adam (core/models.py:3356-3357)
    ("ADADELTA", {"learning_rate": 1.0, "rho": 0.9, "clipnorm": 1.0, "decay": 0.02}),
    ("ADADELTA", {"epsilon": 1e-6}),
]


@pytest.mark.parametrize("name,params", CASES)
def test_keras_optimizer_steps(cuda, name, params):
    from m3d.optim import KerasOptimizer, keras_opt_params
    from m3d.params import ParamStore
    st = ParamStore()
    ps = [st.add("a/kernel:0", (3, 3, 3, 8, 40), "glorot_uniform", True),
          st.add("bn/gamma:0", (40,), "ones", False),
          st.add("c/bias:0", (2100,), ("normal", 0.1), True)]
    wd = 0.01
    st.finalize(cuda, seed=3, weight_decay=wd)
    opt = KerasOptimizer({"name": name, "parameters": params})
    hp = keras_opt_params(params)
    clip, decay, lr = hp.pop("clipnorm", 0.0), hp.pop("decay", 0.0), hp.pop("lr", opt.lr)
    kind = opt.kind
    ref = {p.name: p.data.detach().cpu().numpy().copy() for p in ps}
    states = {p.name: {} for p in ps}
    rng = np.random.default_rng(5)
    for it in range(4):
        grads = {p.name: (rng.normal(size=p.shape) * (3.0 if it % 2 else 0.3)).astype(np.float32) for p in ps}
        st.grad_flat.zero_()
        for p in ps:
            p.grad.copy_(torch.from_numpy(grads[p.name]))
        opt.step(st)
        for p in ps:
            l2c = wd / p.numel if p.l2 else 0.0
            ref[p.name] = O.step(kind, ref[p.name], grads[p.name], states[p.name], it, lr, decay=decay,
                                 clipnorm=clip, l2coef=l2c, **hp)
        torch.cuda.synchronize()
        for p in ps:
            got = p.data.detach().cpu().numpy()
            want = ref[p.name]
            err = np.abs(got.astype(np.float64) - want).max()
            assert err <= 1e-6 * (np.abs(want).max() + 1e-12), (name, it, p.name, err)
    # the padding of each segment stays zero (it is never read as a weight)
    pad = st.flat.detach()[ps[0].offset + ps[0].numel: ps[1].offset]
    assert float(pad.abs().max()) == 0.0
