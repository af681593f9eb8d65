"""Parity at BASELINE.json configs[0]'s own shape: RPN training on one 64^3
toy-shapes volume (generate_data.py:15-231, restated seeded in m3d.toydata;
ToyDataset normalisation core/data_generators.py:1603-1630).

  * the RPN targets built on the GPU inside the step (RPNTargetBuilder ->
    m3d_rpn_targets_async, core/data_generators.py:2031-2178 called at :986)
    against the numpy restatement oracle/heads_ref.build_rpn_targets with the
    same seed: rpn_match bit-exact, rpn_bbox to float32 log rounding;
  * the step's losses on those targets within 1e-4 of the float64 restatement
    of the Keras graph (oracle/model_ref.py) and its weight gradients held to
    the bars of test_gpu_model.py (core/models.py:3320-3387);
  * one full train_step (SGD) runs and moves the weights.
The reference's own TF CPU path cannot run here."""
import numpy as np
import pytest
import torch

from oracle import heads_ref as HR
from oracle import model_ref as MR

pytestmark = pytest.mark.gpu
S = 64


def rel_err(got, ref):
    got = torch.as_tensor(got).detach().double().cpu()
    ref = torch.as_tensor(ref).detach().double().cpu()
    return float((got - ref).abs().max()) / (float(ref.abs().max()) + 1e-30)


@pytest.fixture(scope="module")
def toy(cuda):
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN
    from m3d.targets import RPNTargetBuilder
    from m3d.toydata import network_input, toy_volume
    v = toy_volume(S, seed=5)
    cfg = synthetic_rpn_config(S)
    model = RPN(cfg, device=cuda, seed=1)
    image = torch.from_numpy(network_input(v["image"]))
    gt = (v["boxes"] / np.float32(S)).astype(np.float32)
    builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), cfg, max_gt=32)
    t = builder(torch.from_numpy(gt).to(cuda), seed=7)
    torch.cuda.synchronize()
    builder.check()
    anchors = model.anchors.reshape(-1, 6).cpu().numpy()
    rm, rb = HR.build_rpn_targets(anchors, gt, float(cfg.RPN_POSITIVE_IOU), float(cfg.RPN_NEGATIVE_IOU),
                                  int(cfg.RPN_TRAIN_ANCHORS_PER_IMAGE),
                                  float(getattr(cfg, "RPN_POSITIVE_RATIO", 0.5)), int(cfg.ATSS_TOPK),
                                  int(cfg.ATSS_MIN_POS_PER_GT), cfg.RPN_BBOX_STD_DEV, 7)
    return cfg, model, image, gt, builder, t, rm, rb


def test_config0_toy_volume_shape(toy):
    cfg, model, image, gt, *_ = toy
    assert image.shape == (1, S, S, S, 1) and image.dtype == torch.float32
    assert 3 <= len(gt) <= 20 and np.all(gt[:, 3:] > gt[:, :3])
    assert model.anchors.shape[1] == 65472


def test_config0_rpn_targets_on_gpu(toy):
    cfg, model, image, gt, builder, t, rm, rb = toy
    m = t.match.to(torch.int32).cpu().numpy()
    assert np.array_equal(m, rm), (int((m != rm).sum()), int((m == 1).sum()), int((rm == 1).sum()))
    np.testing.assert_allclose(t.bbox.cpu().numpy(), rb, rtol=1e-5, atol=1e-5)
    cnt = builder.counts.cpu().numpy()
    assert cnt[0] == (rm == 1).sum() > 0 and cnt[1] == (rm == -1).sum() > 0 and cnt[2] == 0
    print(f"configs[0] targets: {len(gt)} GT, {cnt[0]} positives, {cnt[1]} negatives", flush=True)


def test_config0_step_losses_and_gradients(toy, cuda):
    cfg, model, image, gt, builder, t, rm, rb = toy
    model.store.zero_grad()
    out = model.forward(image.to(cuda), proposals=False)
    lc, lb = model.losses(out, t)                      # device-resident targets, mask form
    (lc * 1.0 + lb * 1.5).backward()
    model.rpn.finish_backward()
    torch.cuda.synchronize()

    def ref(dtype):
        r = MR.RefRPN(model.store.state_dict(), dtype=dtype)
        for p in model.store.params:
            r.p[p.name].requires_grad_(True)
        o = r.forward(image.to(dtype))
        match = torch.from_numpy(rm.reshape(1, -1, 1))
        rlc = MR.rpn_class_loss(match, o["rpn_class_logits"])
        rlb = MR.rpn_bbox_loss(torch.from_numpy(rb[None]).to(dtype), match, o["rpn_bbox"])
        (rlc * 1.0 + rlb * 1.5).backward()
        return float(rlc), float(rlb), {k: v.grad for k, v in r.p.items()}
    rlc, rlb, g64 = ref(torch.float64)
    _, _, g32 = ref(torch.float32)
    print(f"configs[0] losses GPU ({float(lc):.6f}, {float(lb):.6f}) fp64 ({rlc:.6f}, {rlb:.6f})", flush=True)
    assert abs(float(lc) - rlc) <= 1e-4 * abs(rlc)
    assert abs(float(lb) - rlb) <= 1e-4 * abs(rlb)
    gpu, cpu32 = [], []
    for p in model.store.params:
        g_ref = g64[p.name]
        if g_ref is None or float(g_ref.abs().max()) == 0.0:
            continue
        gpu.append((rel_err(p.grad, g_ref), p.name))
        cpu32.append(rel_err(g32[p.name], g_ref))
    gpu.sort(reverse=True)
    med, med32 = float(np.median([e for e, _ in gpu])), float(np.median(cpu32))
    print(f"configs[0] gradients: GPU median {med:.2e} worst {gpu[0]}, CPU fp32 median {med32:.2e}", flush=True)
    assert med < 2e-4 and med <= 0.25 * med32, (med, med32)
    assert gpu[0][0] <= max(1e-3, 4 * max(cpu32)), (gpu[:5], max(cpu32))


def test_config0_train_step(toy, cuda):
    cfg, model, image, gt, builder, *_ = toy
    before = model.store.flat.detach().clone()
    r = model.train_step(image.to(cuda), builder(torch.from_numpy(gt).to(cuda), seed=8))
    torch.cuda.synchronize()
    builder.check()
    assert torch.isfinite(r["loss"]).item()
    assert r["rpn_rois"].shape == (1, cfg.POST_NMS_ROIS_TRAINING, 6)
    assert float((model.store.flat.detach() - before).abs().max()) > 0
