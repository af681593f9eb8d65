"""The res2 branch2b convs (3x3x3, 64 -> 64) alone: Winograd forward, data
gradient at tile_y 2 / 4 and weight gradient at 128^3 and 256^3 shapes, timed
with HIP events on the library's stream (and, under rocprofv3, per kernel).
python scripts/r06/res2_prof.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
from m3d import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda:0")
out = {}


def timed(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


for name, (H, W, D) in {"res2_128": (32, 32, 128), "res2_256": (64, 64, 256)}.items():
    C = 64
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn((1, H, W, D, C), device=dev, generator=g)
    w = torch.randn((3, 3, 3, C, C), device=dev, generator=g) * 0.05
    y = torch.empty((1, H, W, D, C), device=dev)
    dz = torch.randn_like(y)
    dx = torch.empty_like(x)
    dw = torch.zeros_like(w)
    nb = int(L.m3d_conv3d_wino_workspace_bytes(1, H, W, D, D, C, C))
    ws = torch.empty(nb // 4 + 64, device=dev)
    s = _lib.stream()
    r = {}
    r["fwd_ms"] = timed(lambda: _lib.check(L.m3d_conv3d_fwd_wino(
        x.data_ptr(), 1, H, W, D, C, w.data_ptr(), C, D, 1, None, None, None, None, 0, None, y.data_ptr(),
        ws.data_ptr(), nb, s), "fwd"))
    for ty in (2, 4):
        r[f"dgrad_y{ty}_ms"] = timed(lambda: _lib.check(L.m3d_conv3d_bwd_data_wino_vy(
            dz.data_ptr(), w.data_ptr(), 1, H, W, D, C, C, D, 1, dx.data_ptr(), 0, ws.data_ptr(), nb, 0, ty, s),
            "dgrad"))
    r["wgrad_ms"] = timed(lambda: _lib.check(L.m3d_conv3d_bwd_weight_wino(
        x.data_ptr(), dz.data_ptr(), 1, H, W, D, C, C, D, 1, dw.data_ptr(), ws.data_ptr(), nb, None, s), "wgrad"))
    for ci, co in ((64, 256), (256, 64), (64, 64)):      # the res2 1x1x1 weight gradients
        x1 = torch.randn((1, H, W, D, ci), device=dev, generator=g)
        dz1 = torch.randn((1, H, W, D, co), device=dev, generator=g)
        dw1 = torch.zeros((1, 1, 1, ci, co), device=dev)
        r[f"wgrad1_{ci}_{co}_ms"] = timed(lambda: _lib.check(L.m3d_conv3d_bwd_weight(
            x1.data_ptr(), dz1.data_ptr(), 1, H, W, D, ci, 1, 1, 1, co, H, W, D, 1, 1, 1, 0, 0, 0, dw1.data_ptr(), s),
            "wgrad1"))
        del x1, dz1, dw1
    r["tensor_mb"] = H * W * D * C * 4 / 1e6
    out[name] = r
    print(name, json.dumps(r), flush=True)
    del x, w, y, dz, dx, dw, ws
    torch.cuda.empty_cache()
print(json.dumps(out))
