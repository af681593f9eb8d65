"""Debug: per-tensor gradient error of the GPU step vs the float64 restatement
on the configs[0] toy volume, with device vs host targets and vs a synthetic
volume, to locate the source of the larger GPU gradient error."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
from oracle import heads_ref as HR  # noqa: E402
from oracle import model_ref as MR  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, RPNTargets, synthetic_volume  # noqa: E402
from m3d.targets import RPNTargetBuilder  # noqa: E402
from m3d.toydata import network_input, toy_volume  # noqa: E402
from m3d import _lib  # noqa: E402

torch.set_num_threads(16)
dev = torch.device("cuda:0")
S = 64


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


def run(model, image, tgt, rm, rb, label):
    model.store.zero_grad()
    out = model.forward(image.to(dev), proposals=False)
    lc, lb = model.losses(out, tgt)
    (lc + 1.5 * lb).backward()
    model.rpn.finish_backward()
    torch.cuda.synchronize()
    res = {}
    for dt in (torch.float64, torch.float32):
        r = MR.RefRPN(model.store.state_dict(), dtype=dt)
        for p in model.store.params:
            r.p[p.name].requires_grad_(True)
        o = r.forward(image.to(dt))
        m = torch.from_numpy(rm.reshape(1, -1, 1))
        l = MR.rpn_class_loss(m, o["rpn_class_logits"]) + 1.5 * MR.rpn_bbox_loss(torch.from_numpy(rb[None]).to(dt), m, o["rpn_bbox"])
        l.backward()
        res[dt] = ({k: v.grad for k, v in r.p.items()}, o)
    g64, o64 = res[torch.float64]
    g32, o32 = res[torch.float32]
    fm = [rel(a, b) for a, b in zip(out["feature_maps"], o64["feature_maps"])]
    fm32 = [rel(a, b) for a, b in zip(o32["feature_maps"], o64["feature_maps"])]
    print(f"== {label}: fwd P2..P6 GPU {['%.1e' % e for e in fm]} CPU32 {['%.1e' % e for e in fm32]}; logits GPU "
          f"{rel(out['rpn_class_logits'], o64['rpn_class_logits']):.1e} CPU32 {rel(o32['rpn_class_logits'], o64['rpn_class_logits']):.1e}")
    rows = []
    for p in model.store.params:
        gr = g64[p.name]
        if gr is None or float(gr.abs().max()) == 0:
            continue
        rows.append((rel(p.grad, gr), rel(g32[p.name], gr), p.name))
    rows.sort(reverse=True)
    print(f"   grads median GPU {np.median([r[0] for r in rows]):.2e} CPU32 {np.median([r[1] for r in rows]):.2e}")
    for r in rows[:12]:
        print(f"   {r[2]:40s} GPU {r[0]:.2e} CPU32 {r[1]:.2e}")
    # order of layers: print a few in network order
    names = [p.name for p in model.store.params]
    sel = [n for n in names if n.endswith("kernel:0")]
    d = {r[2]: r for r in rows}
    print("   network order (kernel:0):", " ".join(f"{n.split('/')[0]}={d[n][0]:.0e}/{d[n][1]:.0e}" for n in sel if n in d))


v = toy_volume(S, seed=5)
cfg = synthetic_rpn_config(S)
model = RPN(cfg, device=dev, seed=1)
image = torch.from_numpy(network_input(v["image"]))
gt = (v["boxes"] / np.float32(S)).astype(np.float32)
builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), cfg, max_gt=32)
t = builder(torch.from_numpy(gt).to(dev), seed=7)
anchors = model.anchors.reshape(-1, 6).cpu().numpy()
rm, rb = HR.build_rpn_targets(anchors, gt, float(cfg.RPN_POSITIVE_IOU), float(cfg.RPN_NEGATIVE_IOU),
                              int(cfg.RPN_TRAIN_ANCHORS_PER_IMAGE), 0.5, int(cfg.ATSS_TOPK),
                              int(cfg.ATSS_MIN_POS_PER_GT), cfg.RPN_BBOX_STD_DEV, 7)
print("image stats", float(image.min()), float(image.max()), float(image.mean()), "unique", int(torch.unique(image).numel()))
run(model, image, t, rm, rb, "toy, device targets")
run(model, image, RPNTargets(rm.reshape(1, -1, 1), rb[None], dev), rm, rb, "toy, host targets")
syn = synthetic_volume(S, seed=0)
run(model, syn, RPNTargets(rm.reshape(1, -1, 1), rb[None], dev), rm, rb, "synthetic volume, same targets")
_lib.set_deterministic(True)
run(model, image, RPNTargets(rm.reshape(1, -1, 1), rb[None], dev), rm, rb, "toy, host targets, deterministic")
_lib.set_deterministic(False)
import m3d.nn as mnn
mnn.WINOGRAD = False
run(model, image, RPNTargets(rm.reshape(1, -1, 1), rb[None], dev), rm, rb, "toy, host targets, no winograd")
