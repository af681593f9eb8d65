"""Winograd conv kernels alone (for rocprofv3 --kernel-trace --stats): forward,
data gradient and weight gradient of 3x3x3 'same' convs at the step's shapes
(rpn_conv_shared1 / fpn_p2 on P2 and a res4 2b conv at 128^3), 5 reps each.
Prints the algorithmic bytes of each transform kernel per launch so the
rocprof durations convert to GB/s.  python scripts/wino_prof.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
from m3d import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda:0")
nz = int(L.m3d_conv3d_wino_tile_z())
out = {}
for name, (H, W, D, Cin, Cout) in {"shared1_P2": (32, 32, 128, 256, 512), "fpn_p2": (32, 32, 128, 256, 256),
                                   "res4_2b": (8, 8, 128, 256, 256)}.items():
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((1, H, W, D, Cin), device=dev, generator=g)
    w = torch.randn((3, 3, 3, Cin, Cout), device=dev, generator=g) * 0.02
    y = torch.empty((1, H, W, D, Cout), device=dev)
    dz = torch.randn_like(y)
    dx = torch.empty_like(x)
    dw = torch.zeros_like(w)
    nb = int(L.m3d_conv3d_wino_workspace_bytes(1, H, W, D, D, Cin, Cout))
    ws = torch.empty(nb // 4 + 64, device=dev)
    for _ in range(5):
        _lib.check(L.m3d_conv3d_fwd_wino(x.data_ptr(), 1, H, W, D, Cin, w.data_ptr(), Cout, D, 1, None, None, None,
                                         None, 0, None, y.data_ptr(), ws.data_ptr(), nb, _lib.stream()), "fwd")
        _lib.check(L.m3d_conv3d_bwd_data_wino(dz.data_ptr(), w.data_ptr(), 1, H, W, D, Cin, Cout, D, 1,
                                              dx.data_ptr(), 0, ws.data_ptr(), nb, _lib.stream()), "dgrad")
        _lib.check(L.m3d_conv3d_bwd_weight_wino(x.data_ptr(), dz.data_ptr(), 1, H, W, D, Cin, Cout, D, 1,
                                                dw.data_ptr(), ws.data_ptr(), nb, _lib.stream()), "wgrad")
    torch.cuda.synchronize()
    T = ((H + 1) // 2) * ((W + 1) // 2) * ((D + nz - 1) // nz)
    P = 16 * (nz + 2)
    out[name] = {"T": T, "points": P,
                 "input_transform_bytes_fwd": 4.0 * (H * W * D * Cin + P * T * Cin),
                 "output_transform_bytes_fwd": 4.0 * (P * T * Cout + H * W * D * Cout),
                 "gemm_fwd_flop": 2.0 * P * T * Cin * Cout}
    del x, w, y, dz, dx, dw, ws
    torch.cuda.empty_cache()
print(json.dumps(out, indent=1))
