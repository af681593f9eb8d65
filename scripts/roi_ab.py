"""A/B of the PyramidROIAlign forward variants (M3D_ROI_REGION, read once per
process) and the CropAndResize3DGradImage modes at the bench's configs[2]
(128^3, 128 ROIs) and configs[3] (256^3, 512 ROIs) shapes on random P2..P5:
ms per launch, HBM fraction on algorithmic bytes, and a checksum of the
output (the variants must agree bit for bit).  Usage: python scripts/roi_ab.py"""
import hashlib
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import bench  # noqa: E402
from m3d import layers, ops  # noqa: E402

dev = torch.device("cuda:0")
res = {"mode": {k: v for k, v in os.environ.items() if k.startswith("M3D_ROI")}}
for S, n_rois in ((128, 128), (256, 512)):
    g = torch.Generator(device=dev).manual_seed(0)
    maps = [torch.randn((1, S // s, S // s, S, 256), device=dev, generator=g) for s in (4, 8, 16, 32)]
    boxes = torch.from_numpy(bench.roi_boxes(n_rois, S, hi=S)).to(dev)
    meta = torch.zeros((1, 18), device=dev)
    meta[0, 5:8] = S
    for p in (7, 14):
        layer = layers.PyramidROIAlign((p, p, p))
        out = layer([boxes, meta] + maps)
        t = bench._event_time(lambda: layer([boxes, meta] + maps), 10)
        u = bench.unique_voxels(boxes.cpu().numpy(), [tuple(m.shape[1:4]) for m in maps], (p, p, p), S)
        alg = 4.0 * n_rois * p ** 3 * 256 + 4.0 * 256 * u
        h = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
        r = {"ms": round(t * 1e3, 4), "frac_hbm": round(alg / t / 1e9 / bench.HBM_PEAK_GBS, 4), "sha": h}
        if p == 14 or S == 128:
            _, badj, lev = ops.pyramid_roi_align(boxes, meta, maps, (p, p, p), return_levels=True)
            gr = torch.randn((n_rois, p, p, p, 256), device=dev, generator=g)
            bi = torch.zeros(n_rois, dtype=torch.int32, device=dev)
            bx = badj.reshape(-1, 6).contiguous()
            shp = tuple(maps[0].shape)
            for mode in ((0, 1) if os.environ.get("ROI_AB_GRAD") else ()):
                tm = bench._event_time(lambda: ops.crop_and_resize_3d_grad_image(gr, bx, bi, shp, deterministic=mode), 3)
                r[f"grad_image_mode{mode}_ms"] = round(tm * 1e3, 3)
        res[f"S{S}_pool{p}"] = r
    del maps
    torch.cuda.empty_cache()
print(json.dumps(res), flush=True)
