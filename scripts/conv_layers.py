"""Per-layer conv table of the RPN training step (GPU): every distinct
conv_bn_act call of the backbone / FPN / RPN head at the bench size is replayed
alone on random tensors and timed (forward with HIP events; backward = data +
weight gradients, side stream joined, wall clock around a synchronize), with its
direct-conv FLOPs, compulsory bytes and the achieved rates.

    python scripts/conv_layers.py [--size 128] [--reps 5] > gpurun_out/conv_layers.txt
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from m3d import backbone, nn as mnn
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    model = RPN(synthetic_rpn_config(a.size), device=dev, seed=1)
    image = synthetic_volume(a.size, seed=100).to(dev)
    calls = []
    orig = backbone.conv_bn_act

    def rec(x, layer, geo, relu, residual=None, res_mode=0, bn=None, need_dx=True, link=None, **kw):
        calls.append((tuple(x.shape), layer, geo, relu, None if residual is None else tuple(residual.shape),
                      res_mode, bn, need_dx))
        return orig(x, layer, geo, relu, residual=residual, res_mode=res_mode, bn=bn, need_dx=need_dx, link=link,
                    **kw)

    backbone.conv_bn_act = rec
    with torch.no_grad():
        fm = model.features(image)
        model.rpn(fm)
    backbone.conv_bn_act = orig
    groups = {}
    for c in calls:
        xs, layer, geo, relu, rs, rm, bn, nd = c
        key = (xs, tuple(layer.kernel.data.shape), geo.k, geo.stride, geo.out, rs, rm, bn is not None, relu, nd)
        groups.setdefault(key, []).append(c)
    print(f"{'x shape':>26} {'k':>7} {'Cin':>5} {'Cout':>5} {'n':>2} {'alg':>5} "
          f"{'fwd_ms':>7} {'TF/s':>6} {'GB/s':>6} {'bwd_ms':>7} {'TF/s':>6} {'tot_ms*n':>8}")
    tot = 0.0
    tot_f = tot_f1 = 0.0
    rows = []
    for key, cs in groups.items():
        xs, layer, geo, relu, rs, rm, bn, nd = cs[0]
        Cin, Cout = xs[-1], layer.kernel.data.shape[-1]
        x = torch.randn(xs, device=dev).requires_grad_(nd)
        r = torch.randn(rs, device=dev) if rs is not None else None
        wino = mnn.use_winograd(geo, Cin, Cout, xs[1:4]) and rm != 2

        def fwd():
            return mnn.conv_bn_act(x, layer, geo, relu, residual=r, res_mode=rm, bn=bn, need_dx=nd)

        y = fwd()
        dy = torch.randn_like(y)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            y = fwd()
        e1.record()
        torch.cuda.synchronize()
        tf = e0.elapsed_time(e1) / a.reps
        tb = []
        for i in range(a.reps + 1):
            y = fwd()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if y.requires_grad:
                torch.autograd.backward(y, dy)
            mnn.join_wgrad()
            torch.cuda.synchronize()
            if i:
                tb.append(time.perf_counter() - t0)
            x.grad = None
        tbm = 1e3 * sorted(tb)[len(tb) // 2]
        M = 1
        for v in y.shape[:-1]:
            M *= v
        kk = geo.k[0] * geo.k[1] * geo.k[2]
        fl = 2.0 * M * kk * Cin * Cout
        nb = 4.0 * (x.numel() + layer.kernel.data.numel() + 2 * y.numel() + (r.numel() if r is not None else 0))
        n = len(cs)
        tot += n * (tf + tbm)
        tot_f += n * tf
        tot_f1 += n * tf if geo.k == (1, 1, 1) else 0.0
        rows.append((n * (tf + tbm), f"{str(xs):>26} {str(geo.k):>7} {Cin:>5} {Cout:>5} {n:>2} "
                     f"{'wino' if wino else 'dir':>5} {tf:7.3f} {fl / tf / 1e9:6.1f} {nb / tf / 1e6:6.0f} "
                     f"{tbm:7.3f} {2 * fl / tbm / 1e9:6.1f} {n * (tf + tbm):8.3f}"))
        del x, y, dy, r
        torch.cuda.empty_cache()
    for _, line in sorted(rows, reverse=True):
        print(line, flush=True)
    print(f"total fwd {tot_f:.2f} ms (1x1x1 {tot_f1:.2f}); total fwd+bwd over layers: {tot:.2f} ms")


if __name__ == "__main__":
    main()
