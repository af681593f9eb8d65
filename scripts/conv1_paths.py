"""1x1x1 conv paths at the backbone / FPN shapes of 128^3 and 256^3 (VERDICT
r4 item 4: the 1^3 forward group): the path m3d.nn picks today (x3 when
nn._conv1_x3, else split-K when nn._splitk > 1, else the implicit GEMM) vs the
256x256 bf16-split GEMM (m3d_conv3d_fwd_x3 / _bwd_data_x3), for the training
forward (bias, BN affine, ReLU, z stored) and the data gradient; max relative
difference between the two.  HIP events, median of 5 after 2 warm-ups.
python scripts/conv1_paths.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402
from m3d import nn as mnn  # noqa: E402

L = _lib.load()
dev = torch.device("cuda:0")
S = _lib.stream


def timeit(fn, n=5):
    for _ in range(2):
        fn()
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[n // 2]


def levels(s):
    return [(1, s // 4, s // 4, s), (1, s // 8, s // 8, s), (1, s // 16, s // 16, s), (1, s // 32, s // 32, s)]


chans = [[(64, 256), (256, 64), (64, 64)], [(128, 512), (512, 128), (256, 128)],
         [(256, 1024), (1024, 256), (512, 256)], [(512, 2048), (2048, 512), (1024, 512)]]
fpn = [(256, 256), (512, 256), (1024, 256), (2048, 256)]
g = torch.Generator(device="cpu").manual_seed(0)
print(f"{'x':>20} {'Cin':>5} {'Cout':>5} | {'fwd cur':>12} {'fwd x3':>7} | {'dgrad cur':>12} {'dgrad x3':>8} | rel")
for size in (128, 256):
    for li, sp in enumerate(levels(size)):
        for cin, cout in chans[li] + [fpn[li]]:
            B, H, W, D = sp
            M = B * H * W * D
            geo = mnn.ConvGeom((1, 1, 1), (1, 1, 1), (0, 0, 0), (H, W, D))
            x = torch.randn((B, H, W, D, cin), generator=g).to(dev)
            w = (torch.randn((1, 1, 1, cin, cout), generator=g) / cin ** 0.5).to(dev)
            bias = torch.randn(cout, generator=g).to(dev)
            scale = torch.rand(cout, generator=g).to(dev) + 0.5
            shift = torch.randn(cout, generator=g).to(dev)
            y1, y2 = torch.empty((B, H, W, D, cout), device=dev), torch.empty((B, H, W, D, cout), device=dev)
            z1, z2 = torch.empty_like(y1), torch.empty_like(y1)
            dz = torch.randn((B, H, W, D, cout), generator=g).to(dev)
            dx1, dx2 = torch.empty_like(x), torch.empty_like(x)
            pf = torch.empty(3 * cin * cout, device=dev, dtype=torch.int16)
            pb = torch.empty(3 * cin * cout, device=dev, dtype=torch.int16)
            _lib.check(L.m3d_conv1_x3_planes(w.data_ptr(), cin, cout, 1, pf.data_ptr(), S()), "planes")
            _lib.check(L.m3d_conv1_x3_planes(w.data_ptr(), cin, cout, 0, pb.data_ptr(), S()), "planes")
            f_x3, d_x3 = mnn._conv1_x3(x.shape, geo, cin, cout), mnn._conv1_x3(x.shape, geo, cout, cin, bwd_data=True)
            f_sk, d_sk = mnn._splitk(x.shape, geo, cin, cout, 0), mnn._splitk(x.shape, geo, cin, cout, 1)
            wsf = torch.empty(max(f_sk, 1) * M * cout, device=dev) if f_sk > 1 else None
            wsd = torch.empty(max(d_sk, 1) * M * cin, device=dev) if d_sk > 1 else None

            def fwd_x3():
                _lib.check(L.m3d_conv3d_fwd_x3(x.data_ptr(), B, H, W, D, cin, pf.data_ptr(), cout, bias.data_ptr(),
                                               scale.data_ptr(), shift.data_ptr(), None, 0, 1, z2.data_ptr(),
                                               y2.data_ptr(), S()), "fwd_x3")

            def fwd_cur():
                if f_x3:
                    _lib.check(L.m3d_conv3d_fwd_x3(x.data_ptr(), B, H, W, D, cin, pf.data_ptr(), cout,
                                                   bias.data_ptr(), scale.data_ptr(), shift.data_ptr(), None, 0, 1,
                                                   z1.data_ptr(), y1.data_ptr(), S()), "fwd_x3")
                elif f_sk > 1:
                    _lib.check(L.m3d_conv3d_fwd_splitk(x.data_ptr(), B, H, W, D, cin, w.data_ptr(), cout, H, W, D,
                                                       1, 1, 1, bias.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                                       None, 0, 1, z1.data_ptr(), y1.data_ptr(), f_sk,
                                                       wsf.data_ptr(), wsf.numel() * 4, S()), "fwd_splitk")
                else:
                    _lib.check(L.m3d_conv3d_fwd(x.data_ptr(), B, H, W, D, cin, w.data_ptr(), 1, 1, 1, cout, H, W, D,
                                                1, 1, 1, 0, 0, 0, bias.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                                None, 0, 1, z1.data_ptr(), y1.data_ptr(), cout, None, 0, 0, S()), "fwd")

            def dg_x3():
                _lib.check(L.m3d_conv3d_bwd_data_x3(dz.data_ptr(), pb.data_ptr(), B, H, W, D, cin, cout,
                                                    dx2.data_ptr(), S()), "bwd_data_x3")

            def dg_cur():
                if d_x3:
                    _lib.check(L.m3d_conv3d_bwd_data_x3(dz.data_ptr(), pb.data_ptr(), B, H, W, D, cin, cout,
                                                        dx1.data_ptr(), S()), "bwd_data_x3")
                elif d_sk > 1:
                    _lib.check(L.m3d_conv3d_bwd_data_splitk(dz.data_ptr(), w.data_ptr(), B, H, W, D, cin, cout,
                                                            H, W, D, 1, 1, 1, dx1.data_ptr(), 0, d_sk, wsd.data_ptr(),
                                                            wsd.numel() * 4, S()), "bwd_data_splitk")
                else:
                    _lib.check(L.m3d_conv3d_bwd_data(dz.data_ptr(), w.data_ptr(), B, H, W, D, cin, 1, 1, 1, cout,
                                                     H, W, D, 1, 1, 1, 0, 0, 0, dx1.data_ptr(), 0, S()), "bwd_data")
            tf = timeit(fwd_cur)
            tfx = timeit(fwd_x3) if cout % 256 == 0 else float("nan")
            td = timeit(dg_cur)
            tdx = timeit(dg_x3) if cin % 256 == 0 else float("nan")
            torch.cuda.synchronize()
            rel = []
            if cout % 256 == 0:
                rel.append(float((y1 - y2).abs().max()) / float(y1.abs().max()))
            if cin % 256 == 0:
                rel.append(float((dx1 - dx2).abs().max()) / float(dx1.abs().max()))
            cf = "x3" if f_x3 else (f"sk{f_sk}" if f_sk > 1 else "gemm")
            cd = "x3" if d_x3 else (f"sk{d_sk}" if d_sk > 1 else "gemm")
            print(f"{str(sp):>20} {cin:5d} {cout:5d} | {cf:>5} {tf:6.3f} {tfx:7.3f} | {cd:>5} {td:6.3f} {tdx:8.3f} | "
                  f"{max(rel) if rel else float('nan'):.1e}", flush=True)
            del x, w, y1, y2, z1, z2, dz, dx1, dx2, wsf, wsd
