"""Diagnostic: GPU grads vs fp64 reference, and CPU-fp32 reference vs fp64 (precision floor)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import numpy as np, torch
from oracle import model_ref as MR
from m3d.config import synthetic_rpn_config
from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume

dev = torch.device("cuda")
cfg = synthetic_rpn_config(64, depth=8, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
model = RPN(cfg, device=dev, seed=5)
image = synthetic_volume(64, 8, seed=0)
A = model.anchors.shape[1]
match, bbox = synthetic_rpn_targets(A, 256, seed=2)
tg = RPNTargets(match, bbox, dev)
model.store.zero_grad()
out = model.forward(image.to(dev), proposals=False)
lc, lb = model.losses(out, tg)
(lc + 1.5 * lb).backward()
model.rpn.finish_backward()
torch.cuda.synchronize()
st = model.store.state_dict()

def ref_grads(dtype):
    ref = MR.RefRPN(st, dtype=dtype)
    for p in model.store.params:
        ref.p[p.name].requires_grad_(True)
    o = ref.forward(image.to(dtype))
    m = torch.from_numpy(match)
    l = MR.rpn_class_loss(m, o["rpn_class_logits"]) + 1.5 * MR.rpn_bbox_loss(torch.from_numpy(bbox).to(dtype), m, o["rpn_bbox"])
    l.backward()
    return {k: (v.grad.double() if v.grad is not None else None) for k, v in ref.p.items()}

g64 = ref_grads(torch.float64)
g32 = ref_grads(torch.float32)
def rel(a, b):
    return float((a.double().cpu() - b).abs().max()) / (float(b.abs().max()) + 1e-30)
rows = []
for p in model.store.params:
    b = g64[p.name]
    if b is None or float(b.abs().max()) == 0: continue
    rows.append((rel(p.grad, b), rel(g32[p.name], b), p.name))
rows.sort(reverse=True)
print("worst GPU-vs-fp64 | CPUfp32-vs-fp64 | name")
for r in rows[:15]:
    print(f"{r[0]:.3e} {r[1]:.3e} {r[2]}")
print("median gpu", np.median([r[0] for r in rows]), "median cpu32", np.median([r[1] for r in rows]))
