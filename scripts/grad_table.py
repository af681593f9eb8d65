"""Per-tensor gradient error table of the configs[1] step (128^3): the GPU
weight gradients (deterministic mode) against the float64 restatement on the
GPU forward's ReLU branches, beside the CPU fp32 restatement's error on the
same branches (tests/gradparity.py's yardstick), for one or more host-side
variants of the conv path.  Writes JSON {variant: {median, worst, rows}}.

    python scripts/grad_table.py --out gpurun_out/grad.json [--variants base,wino_min128,...]

Variants are module constants of m3d.nn (the kernel-side tile choice is a
compile-time constant: run another build with M3D_LIB_FILE)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

VARIANTS = {
    "base": {},
    "wino_min128": {"WINO_MIN_C": 128},          # the 64-channel res2 2b convs direct
    "wino_min256": {"WINO_MIN_C": 256},          # res2 + res3 2b direct
    "no_wino": {"WINOGRAD": False},              # every 3^3 conv direct (accuracy floor of the kernels)
    # round 5: the data gradient's y tile per layer (nn.WINO_DGRAD_Y4; F(2x2x4) default)
    "y4_all": {"WINO_DGRAD_Y4": "*"},
    "y4_shared1": {"WINO_DGRAD_Y4": "rpn_conv_shared1"},
    "y4_p2": {"WINO_DGRAD_Y4": "rpn_conv_shared1+fpn_p2"},
    "y4_fpn": {"WINO_DGRAD_Y4": "rpn_conv_shared1+fpn_p2+fpn_p3+fpn_p4+fpn_p5"},
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--variants", default="base")
    ap.add_argument("--size", type=int, default=128)
    a = ap.parse_args()
    import m3d.nn as mnn
    from gradparity import deterministic, ref_grads, rel_err
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    dev = torch.device("cuda", 0)
    cfg = synthetic_rpn_config(a.size)
    model = RPN(cfg, device=dev, seed=1)
    image = synthetic_volume(a.size, seed=100)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=2)
    torch.set_num_threads(min(16, torch.get_num_threads()))
    res = {}
    for name in a.variants.split(","):
        saved = {k: getattr(mnn, k) for k in VARIANTS[name]}
        for k, v in VARIANTS[name].items():
            setattr(mnn, k, v)
        try:
            model.store.zero_grad()
            mnn.RELU_CAPTURE = {}
            with deterministic():
                try:
                    out = model.forward(image.to(dev), proposals=False)
                    masks = mnn.RELU_CAPTURE
                finally:
                    mnn.RELU_CAPTURE = None
                lc, lb = model.losses(out, RPNTargets(match, bbox, dev))
                (lc * 1.0 + lb * 1.5).backward()
                model.rpn.finish_backward()
            torch.cuda.synchronize()
            del out
        finally:
            for k, v in saved.items():
                setattr(mnn, k, v)
        t0 = time.time()
        _, _, g64 = ref_grads(model, image, match, bbox, torch.float64, masks)
        _, _, g32 = ref_grads(model, image, match, bbox, torch.float32, masks)
        rows = []
        for p in model.store.params:
            g = g64[p.name]
            if g is None or float(g.abs().max()) == 0.0:
                continue
            rows.append({"name": p.name, "gpu": rel_err(p.grad.cpu().numpy(), g.numpy()),
                         "cpu32": rel_err(g32[p.name].numpy(), g.numpy())})
        med = float(np.median([r["gpu"] for r in rows]))
        ratio = sorted(rows, key=lambda r: -r["gpu"] / max(r["cpu32"], 1e-30))
        res[name] = {"median": med, "median_cpu32": float(np.median([r["cpu32"] for r in rows])),
                     "worst_ratio": [(r["name"], r["gpu"], r["cpu32"]) for r in ratio[:8]],
                     "n_over_10x": sum(r["gpu"] > 10 * r["cpu32"] for r in rows), "rows": rows}
        print(f"{name}: median {med:.3e} (cpu32 {res[name]['median_cpu32']:.3e}), >10x cpu32: "
              f"{res[name]['n_over_10x']}, worst ratios {res[name]['worst_ratio'][:4]} ({time.time() - t0:.0f} s refs)",
              flush=True)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
