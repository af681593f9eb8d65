"""Stem conv (conv1: 7^3, 1 -> 64, strides (2,2,1), ZeroPadding3D(3)) forward
and weight gradient: time per launch at 128^3 / 256^3 through m3d_conv3d_fwd /
m3d_conv3d_bwd_weight (M3D_STEM_MFMA / M3D_STEM_WGRAD pick the kernels, read
once per process) and the error against torch's fp32 conv3d and its weight
gradient (MIOpen) on the same input.  python scripts/stem_ab.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import bench  # noqa: E402
from m3d import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda:0")
res = {k: os.environ[k] for k in os.environ if k.startswith("M3D_STEM")}
for S in (128, 256):
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.tanh(0.5 * torch.randn((1, S, S, S, 1), device=dev, generator=g))
    w = torch.randn((7, 7, 7, 1, 64), device=dev, generator=g) * (2.0 / 343) ** 0.5
    b = torch.randn(64, device=dev, generator=g) * 0.1
    sc = torch.rand(64, device=dev, generator=g) + 0.5
    sh = torch.randn(64, device=dev, generator=g) * 0.1
    O = S // 2
    y = torch.empty((1, O, O, S, 64), device=dev)
    z = torch.empty_like(y)

    def run():
        _lib.check(L.m3d_conv3d_fwd(x.data_ptr(), 1, S, S, S, 1, w.data_ptr(), 7, 7, 7, 64, O, O, S, 2, 2, 1,
                                    3, 3, 3, b.data_ptr(), sc.data_ptr(), sh.data_ptr(), None, 0, 1,
                                    z.data_ptr(), y.data_ptr(), 64, None, 0, 0, _lib.stream()), "stem")
    t = bench._event_time(run, 10)
    flops = 2.0 * O * O * S * 343 * 64
    ref = torch.nn.functional.conv3d(x.permute(0, 4, 1, 2, 3), w.permute(4, 3, 0, 1, 2), b, stride=(2, 2, 1),
                                     padding=3).permute(0, 2, 3, 4, 1)
    ez = float((z - ref).abs().max() / ref.abs().max())
    yr = torch.relu(ref * sc + sh)
    ey = float((y - yr).abs().max() / yr.abs().max())
    dz = torch.randn((1, O, O, S, 64), device=dev, generator=g)
    dw = torch.zeros_like(w)

    def runw():
        _lib.check(L.m3d_conv3d_bwd_weight(x.data_ptr(), dz.data_ptr(), 1, S, S, S, 1, 7, 7, 7, 64, O, O, S,
                                           2, 2, 1, 3, 3, 3, dw.data_ptr(), _lib.stream()), "stem wgrad")
    tw = bench._event_time(runw, 10)
    dw.zero_()
    runw()
    refw = torch.nn.grad.conv3d_weight(x.permute(0, 4, 1, 2, 3), (64, 1, 7, 7, 7), dz.permute(0, 4, 1, 2, 3),
                                       stride=(2, 2, 1), padding=3).permute(2, 3, 4, 1, 0)
    ew = float((dw - refw).abs().max() / refw.abs().max())
    res[f"S{S}"] = {"ms": round(t * 1e3, 4), "tflops": round(flops / t / 1e12, 2),
                    "frac_f32_mfma": round(flops / t / 1e12 / bench.F32_MFMA_PEAK_TFLOPS, 4),
                    "rel_err_z": ez, "rel_err_y": ey,
                    "wgrad_ms": round(tw * 1e3, 4), "wgrad_frac_f32_mfma":
                        round(flops / tw / 1e12 / bench.F32_MFMA_PEAK_TFLOPS, 4), "rel_err_dw": ew}
    del x, y, z, ref, yr, dz, refw
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
