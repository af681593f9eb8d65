"""Debug: tests/test_gpu_conv.py::test_conv_block_fwd_bwd case 2 (wino) over many seeds."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
import m3d.nn as mnn
from m3d.nn import conv_bn_act, conv_geom, join_wgrad
from oracle import model_ref as MR
from test_gpu_conv import _Layer, _BN, CASES

mnn.WINOGRAD = True
mnn.WINO_MIN_C = 32
cuda = torch.device("cuda")
ci = int(sys.argv[1]) if len(sys.argv) > 1 else 2
nseeds = int(sys.argv[2]) if len(sys.argv) > 2 else 60


def rel(got, ref):
    got = got.detach().double().cpu(); ref = ref.detach().double().cpu()
    return float((got - ref).abs().max()) / (float(ref.abs().max()) + 1e-12)


bad = 0
for seed in range(nseeds):
    sp, cin, cout, k, stride, padding, use_bn, relu, use_res = CASES[ci]
    rng = np.random.default_rng(seed)
    x = torch.tensor(rng.normal(size=(2, *sp, cin)), dtype=torch.float32)
    w = torch.tensor(rng.normal(0, 1.0 / np.sqrt(np.prod(k) * cin), (*k, cin, cout)), dtype=torch.float32)
    b = torch.tensor(rng.normal(0, 0.1, cout), dtype=torch.float32)
    geo = conv_geom(sp, k, stride, padding)
    res = torch.tensor(rng.normal(size=(2, *geo.out, cout)), dtype=torch.float32) if use_res else None
    layer = _Layer(w.to(cuda), b.to(cuda))
    bn = _BN(cout, cuda, rng) if use_bn else None
    xg = x.to(cuda).requires_grad_(cin != 1)
    rg = res.to(cuda).requires_grad_(True) if use_res else None
    layer.kernel.data.requires_grad_(True)
    y = conv_bn_act(xg, layer, geo, relu, residual=rg, res_mode=1 if use_res else 0, bn=bn, need_dx=cin != 1)
    xr = x.double().requires_grad_(True); wr = w.double().requires_grad_(True); br = b.double().requires_grad_(True)
    yr = MR.conv3d(xr, wr, br, stride, padding)
    if use_bn:
        gr = bn.gamma.data.cpu().double().requires_grad_(True)
        ber = bn.beta.data.cpu().double().requires_grad_(True)
        yr = MR.batchnorm(yr, gr, ber, bn.moving_mean.cpu().double(), bn.moving_variance.cpu().double())
    if use_res:
        rr = res.double().requires_grad_(True); yr = yr + rr
    flips = 0
    if relu:
        flips = int(((yr > 0) != (y.detach().double().cpu() > 0)).sum())
        yr = torch.relu(yr)
    e_y = rel(y, yr)
    g = torch.tensor(rng.normal(size=yr.shape), dtype=torch.float32)
    y.backward(g.to(cuda))
    join_wgrad()
    yr.backward(g.double())
    e = [e_y, rel(layer.kernel.grad, wr.grad), rel(layer.bias.grad, br.grad)]
    if cin != 1:
        e.append(rel(xg.grad, xr.grad))
    if use_bn:
        e += [rel(bn.gamma.grad, gr.grad), rel(bn.beta.grad, ber.grad)]
    flag = max(e) > 1e-4
    bad += flag
    if flag or seed < 3:
        print(seed, " ".join(f"{v:.2e}" for v in e), "BAD" if flag else "", "relu flips", flips, flush=True)
print("bad", bad, "of", nseeds)
