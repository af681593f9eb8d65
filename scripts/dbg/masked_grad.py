"""Debug/calibration: GPU RPN gradients vs the float64 restatement taking the
GPU's ReLU branches (m3d.nn.RELU_CAPTURE -> RefRPN relu_masks), at the toy 64^3
volume (configs[0]) and the synthetic 128^3 volume (configs[1])."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
from oracle import heads_ref as HR  # noqa: E402
from oracle import model_ref as MR  # noqa: E402
import m3d.nn as mnn  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, RPNTargets, synthetic_volume, synthetic_rpn_targets  # noqa: E402
from m3d.toydata import network_input, toy_volume  # noqa: E402

torch.set_num_threads(16)
dev = torch.device("cuda:0")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max()) / (float(b.abs().max()) + 1e-30)


def run(model, image, rm, rb, label):
    tg = RPNTargets(rm.reshape(1, -1, 1), rb[None], dev)
    mnn.RELU_CAPTURE = {}
    model.store.zero_grad()
    out = model.forward(image.to(dev), proposals=False)
    masks = mnn.RELU_CAPTURE
    mnn.RELU_CAPTURE = None
    lc, lb = model.losses(out, tg)
    (lc + 1.5 * lb).backward()
    model.rpn.finish_backward()
    torch.cuda.synchronize()
    del out
    g = {}
    for key, dt, mk in (("64m", torch.float64, masks), ("32m", torch.float32, masks), ("64", torch.float64, None), ("32", torch.float32, None)):
        t0 = time.time()
        r = MR.RefRPN(model.store.state_dict(), dtype=dt, relu_masks=mk)
        for p in model.store.params:
            r.p[p.name].requires_grad_(True)
        o = r.forward(image.to(dt))
        m = torch.from_numpy(rm.reshape(1, -1, 1))
        l = MR.rpn_class_loss(m, o["rpn_class_logits"]) + 1.5 * MR.rpn_bbox_loss(torch.from_numpy(rb[None]).to(dt), m, o["rpn_bbox"])
        l.backward()
        g[key] = {k: v.grad for k, v in r.p.items()}
        print(f"  ref {key} {time.time() - t0:.1f}s loss {float(l):.6f}", flush=True)
        del r, o, l
    nflip = sum(int(x.numel()) for v in masks.values() for x in v)
    print(f"== {label}: masks {len(masks)} layers, {nflip / 1e6:.1f}M elements")
    rows = []
    for p in model.store.params:
        gr = g["64m"][p.name]
        if gr is None or float(gr.abs().max()) == 0:
            continue
        rows.append((rel(p.grad, gr), rel(g["32m"][p.name], gr), rel(g["32"][p.name], g["64"][p.name]), p.name))
    rows.sort(reverse=True)
    for i, lab in enumerate(("GPU vs 64m", "CPU32m vs 64m", "CPU32 vs 64 (unmasked)")):
        v = [r[i] for r in rows]
        print(f"   {lab:24s} median {np.median(v):.2e} p90 {np.percentile(v, 90):.2e} max {max(v):.2e}")
    for r in rows[:8]:
        print(f"   {r[3]:40s} GPU {r[0]:.2e} CPU32m {r[1]:.2e} CPU32 {r[2]:.2e}")


S = 64
v = toy_volume(S, seed=5)
cfg = synthetic_rpn_config(S)
model = RPN(cfg, device=dev, seed=1)
image = torch.from_numpy(network_input(v["image"]))
gt = (v["boxes"] / np.float32(S)).astype(np.float32)
anchors = model.anchors.reshape(-1, 6).cpu().numpy()
rm, rb = HR.build_rpn_targets(anchors, gt, float(cfg.RPN_POSITIVE_IOU), float(cfg.RPN_NEGATIVE_IOU),
                              int(cfg.RPN_TRAIN_ANCHORS_PER_IMAGE), 0.5, int(cfg.ATSS_TOPK),
                              int(cfg.ATSS_MIN_POS_PER_GT), cfg.RPN_BBOX_STD_DEV, 7)
run(model, image, rm, rb, "configs[0] toy 64^3")
del model
torch.cuda.empty_cache()
S = 128
cfg = synthetic_rpn_config(S)
model = RPN(cfg, device=dev, seed=11)
match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 1536, seed=2)
run(model, synthetic_volume(S, seed=0), match.reshape(-1), bbox[0], "configs[1] synthetic 128^3")
