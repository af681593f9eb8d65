"""bn_act_bwd_kernel bandwidth at the step's large shapes (GPU).  Prints one
line per shape: ms, GB/s on the bytes it must move, and a checksum of the
outputs (compare across M3D_BN_UNROLL settings: must be identical).

    M3D_BN_UNROLL=4 python scripts/bn_bench.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import torch  # noqa: E402


def main():
    from m3d import nn as mnn
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1)
    # (M, C, bn, relu, residual): RPN shared1 at P2, res2 2a/2b (BN), res2 2c (BN + residual)
    shapes = [(131072, 512, False, True, False), (131072, 64, True, True, False), (131072, 256, True, True, True),
              (32768, 512, True, True, True)]
    for M, C, bn, relu, res in shapes:
        dy = torch.randn((M, C), device=dev, generator=g)
        y = torch.randn((M, C), device=dev, generator=g)
        z = torch.randn((M, C), device=dev, generator=g) if bn else None
        scale = torch.rand(C, device=dev, generator=g) + 0.5 if bn else None
        mean = torch.randn(C, device=dev, generator=g) if bn else None
        rstd = torch.rand(C, device=dev, generator=g) + 0.5 if bn else None
        dz = torch.empty_like(dy)
        dres = torch.empty_like(dy) if res else None
        s0, s1, s2 = (torch.zeros(C, device=dev) for _ in range(3))

        def run():
            mnn.bn_act_bwd(dy, y, z, M, C, relu, scale, mean, rstd, dz, dres, s0 if bn else None,
                           s1 if bn else None, s2)
        run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        nb = 4.0 * M * C * (1 + (1 if relu else 0) + (1 if bn else 0) + 1 + (1 if res else 0))
        s0.zero_(); s1.zero_(); s2.zero_()
        run()
        torch.cuda.synchronize()
        ck = float(dz.double().sum()) + float(s0.double().sum()) + float(s1.double().sum()) + float(s2.double().sum())
        print(f"M={M} C={C} bn={bn} relu={relu} res={res}: {ms:.3f} ms, {nb / ms / 1e6:.0f} GB/s, check {ck!r}",
              flush=True)


if __name__ == "__main__":
    main()
