"""ROI-align kernel variant timing (M3D_ROI_VARIANT read by libm3d at first launch).
Random P2..P5 of an S^3 volume (C=256), bench.roi_boxes ROIs, pools 7 and 14.
Prints one JSON line: per (S, pool) ms, GB/s (algorithmic), output digest."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from m3d import layers  # noqa: E402

dev = torch.device("cuda")
res = {"variant": os.environ.get("M3D_ROI_VARIANT", "default")}
CASES = [(int(c.split(",")[0]), int(c.split(",")[1])) for c in os.environ.get("ROI_CASES", "128,128 256,512").split()]
POOLS = [int(v) for v in os.environ.get("ROI_POOLS", "7 14").split()]
for S, NR in CASES:
    g = torch.Generator(device=dev).manual_seed(0)
    maps = [torch.randn((1, S // s, S // s, S, 256), device=dev, generator=g) for s in (4, 8, 16, 32)]
    boxes = torch.from_numpy(bench.roi_boxes(NR, S, hi=128 if S == 128 else S)).to(dev)
    meta = torch.zeros((1, 18), device=dev)
    meta[0, 5:8] = S
    fshapes = [tuple(m.shape[1:4]) for m in maps]
    for p in POOLS:
        layer = layers.PyramidROIAlign((p, p, p))
        out = layer([boxes, meta] + maps)
        torch.cuda.synchronize()
        dig = hashlib.sha1(out.cpu().numpy().tobytes()).hexdigest()[:12]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = int(os.environ.get("ROI_REPS", "20"))
        e0.record()
        for _ in range(reps):
            layer([boxes, meta] + maps)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps / 1e3
        u = bench.unique_voxels(boxes.cpu().numpy(), fshapes, (p, p, p), S)
        alg = 4.0 * NR * p ** 3 * 256 + 4.0 * 256 * u
        res[f"S{S}_p{p}"] = {"ms": round(t * 1e3, 4), "GBps": round(alg / t / 1e9, 1),
                             "frac": round(alg / t / 8e12, 4), "digest": dig}
print(json.dumps(res))
