"""Gradient parity helpers of the full-size GPU tests (test_gpu_configs.py,
test_gpu_config0.py): the GPU step's weight gradients against the float64
CPU restatement (oracle/model_ref.py) taking the GPU forward's ReLU branches,
with the CPU fp32 restatement on the same branches as the yardstick."""
import contextlib
import numpy as np
import torch

from oracle import model_ref as MR


def rel_err(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(got - ref).max()) / (float(np.abs(ref).max()) + 1e-30)


def ref_grads(model, image, match, bbox, dtype, relu_masks=None):
    ref = MR.RefRPN(model.store.state_dict(), dtype=dtype, relu_masks=relu_masks)
    for p in model.store.params:
        ref.p[p.name].requires_grad_(True)
    o = ref.forward(image.to(dtype))
    m = torch.from_numpy(match)
    rlc = MR.rpn_class_loss(m, o["rpn_class_logits"])
    rlb = MR.rpn_bbox_loss(torch.from_numpy(bbox).to(dtype), m, o["rpn_bbox"])
    (rlc * 1.0 + rlb * 1.5).backward()
    return float(rlc), float(rlb), {k: (v.grad.clone() if v.grad is not None else None) for k, v in ref.p.items()}


# the median tensor's bar (round 5: 1e-5 -> 3e-6 with the F(2x2x4) data gradients)
MEDIAN_BAR = 3e-6


def grad_parity(model, g64, g32, label):
    """Per weight tensor: GPU gradient vs the float64 restatement that took the
    GPU forward's ReLU branches.  Bars: every tensor within the north-star
    1e-4 of its scale -- or, where the CPU fp32 restatement on the same
    branches is itself further off (the stem conv's gradient: 3^3 max-pool
    ties fp32 and fp64 break differently), within 2x the CPU fp32 error --
    and the median tensor below MEDIAN_BAR."""
    rows = []
    for p in model.store.params:
        g_ref = g64[p.name]
        if g_ref is None or float(g_ref.abs().max()) == 0.0:
            continue
        rows.append((rel_err(p.grad.cpu().numpy(), g_ref.numpy()), rel_err(g32[p.name].numpy(), g_ref.numpy()),
                     p.name))
    rows.sort(reverse=True)
    med = float(np.median([r[0] for r in rows]))
    med32 = float(np.median([r[1] for r in rows]))
    over10 = sum(r[0] > 10.0 * r[1] for r in rows)
    print(f"{label} gradients: {len(rows)} tensors, GPU median {med:.2e} (CPU fp32 on the same branches "
          f"{med32:.2e}), {over10} tensors above 10x their CPU fp32 error, worst {rows[:3]}", flush=True)
    assert med < MEDIAN_BAR, med
    bad = [r for r in rows if r[0] > max(1e-4, 2.0 * r[1])]
    assert not bad, bad[:5]


@contextlib.contextmanager
def deterministic():
    """Run the enclosed GPU step in m3d's deterministic mode (weight-gradient
    splits summed in a fixed order, fixed-tree clip norms, the PyramidROIAlign
    backward in the reference's scatter order), so a parity failure replays
    bit for bit."""
    import torch
    from m3d import _lib
    _lib.set_deterministic(True)
    try:
        yield
    finally:
        torch.cuda.synchronize()
        _lib.set_deterministic(False)
