"""CropAndResize3DGradImage timing at the bench shapes (bench.py
time_roi_align_bwd's crop_grad_image_P2): atomic vs deterministic mode 1 for
512 ROIs into a 256^3 P2 [1,64,64,256,256] and 128 ROIs into a 128^3 P2
[1,32,32,128,256], 7^3 and 14^3; plus the PyramidROIAlign forward.  Prints one
JSON line.  Usage: python scripts/roi_bwd_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d import layers, ops  # noqa: E402

dev = torch.device("cuda:0")
out = {}
for S, n in ((128, 128), (256, 512)):
    g = torch.Generator(device=dev).manual_seed(1)
    shape = (1, S // 4, S // 4, S, 256)
    boxes = torch.from_numpy(bench.roi_boxes(n, S, hi=S if S == 256 else 128)[0]).to(dev)
    bi = torch.zeros(n, dtype=torch.int32, device=dev)
    for p in (7, 14):
        grad = torch.randn((n, p, p, p, 256), device=dev, generator=g)
        ta = bench._event_time(lambda: ops.crop_and_resize_3d_grad_image(grad, boxes, bi, shape, deterministic=0), 5)
        td = bench._event_time(lambda: ops.crop_and_resize_3d_grad_image(grad, boxes, bi, shape, deterministic=1), 5)
        a = ops.crop_and_resize_3d_grad_image(grad, boxes, bi, shape, deterministic=1)
        b = ops.crop_and_resize_3d_grad_image(grad, boxes, bi, shape, deterministic=1)
        out[f"S{S}_p{p}"] = {"atomic_ms": round(ta * 1e3, 4), "det_ms": round(td * 1e3, 4),
                             "ratio": round(td / ta, 2), "det_repeatable": bool(torch.equal(a, b))}
        print(S, p, out[f"S{S}_p{p}"], flush=True)
print(json.dumps(out))
