"""Median / max relative gradient error of the GPU RPN backward vs float64, next
to the CPU fp32 restatement's own (tests/test_gpu_model.py's quantities)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from test_gpu_model import _ref_grads, rel_err  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume  # noqa: E402

dev = torch.device("cuda")
cfg = synthetic_rpn_config(64, depth=int(os.environ.get("DEPTH", "8")), PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
model = RPN(cfg, device=dev, seed=5)
image = synthetic_volume(64, cfg.IMAGE_DEPTH, seed=0)
match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
tg = RPNTargets(match, bbox, dev)
model.store.zero_grad()
out = model.forward(image.to(dev), proposals=False)
lc, lb = model.losses(out, tg)
(lc * 1.0 + lb * 1.5).backward()
model.rpn.finish_backward()
_, _, g64 = _ref_grads(model, image, match, bbox, torch.float64)
_, _, g32 = _ref_grads(model, image, match, bbox, torch.float32)
gpu, cpu = [], []
for p in model.store.params:
    r = g64[p.name]
    if r is None or float(r.abs().max()) == 0.0:
        continue
    gpu.append(rel_err(p.grad, r))
    cpu.append(rel_err(g32[p.name], r))
print(f"NZ={os.environ.get('M3D_WINO_NZ', '4')} DGRAD={os.environ.get('M3D_WINO_DGRAD_NZ', '-')} "
      f"gpu median {np.median(gpu):.3e} max {max(gpu):.3e} | cpu-fp32 median {np.median(cpu):.3e} max {max(cpu):.3e}")
