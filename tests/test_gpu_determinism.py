"""Deterministic mode (m3d_set_deterministic): the weight-gradient m-splits and
the clip norms summed in a fixed order through a device scratch instead of
fp32 atomics.  Repeated runs must be bitwise identical; against the default
(atomic) mode the results agree within fp32 reassociation (1e-5 of the scale).
The RPN training step and its HIP-graph replay are checked bitwise too."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture
def det(cuda):
    from m3d import _lib
    yield _lib
    _lib.set_deterministic(False)


def _wgrad_direct(L, _lib, x, dz, k, cout, cuda):
    B, H, W, D, Cin = x.shape
    p = (k - 1) // 2
    dw = torch.zeros((k, k, k, Cin, cout), device=cuda)
    _lib.check(L.m3d_conv3d_bwd_weight(x.data_ptr(), dz.data_ptr(), B, H, W, D, Cin, k, k, k, cout, H, W, D,
                                       1, 1, 1, p, p, p, dw.data_ptr(), _lib.stream()), "bwd_weight")
    return dw


def _wgrad_wino(L, _lib, x, dz, cout, cuda):
    B, H, W, D, Cin = x.shape
    nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, Cin, cout))
    ws = torch.empty(nb // 4 + 1, device=cuda)
    dw = torch.zeros((3, 3, 3, Cin, cout), device=cuda)
    _lib.check(L.m3d_conv3d_bwd_weight_wino(x.data_ptr(), dz.data_ptr(), B, H, W, D, Cin, cout, D, 1,
                                            dw.data_ptr(), ws.data_ptr(), nb, _lib.stream()), "wino wgrad")
    return dw


# (kernel, Cin, Cout, algorithm): conv_wgrad_kernel (3^3, 64 ch), x3_wgrad_kernel
# (1^3, 256 -> 128), x3_wgrad_tr_kernel (Winograd 256 -> 256), conv_wgrad 1^3 64 -> 64,
# x3_wgrad64_kernel (Winograd 64 -> 64, the res2 branch2b gradients)
CASES = [(3, 64, 64, "direct"), (1, 256, 128, "direct"), (3, 256, 256, "wino"), (1, 64, 64, "direct"),
         (3, 64, 64, "wino")]


@pytest.mark.parametrize("k,cin,cout,alg", CASES)
def test_weight_gradient_bitwise_repeatable(det, cuda, k, cin, cout, alg):
    _lib = det
    L = _lib.load()
    g = torch.Generator().manual_seed(5)
    x = torch.randn((1, 16, 16, 32, cin), generator=g).to(cuda)
    dz = torch.randn((1, 16, 16, 32, cout), generator=g).to(cuda)

    def run():
        if alg == "wino":
            return _wgrad_wino(L, _lib, x, dz, cout, cuda)
        return _wgrad_direct(L, _lib, x, dz, k, cout, cuda)

    # float64 reference: the weight gradient of a 'same' stride-1 conv
    xd = x.double().permute(0, 4, 1, 2, 3)
    dzd = dz.double().permute(0, 4, 1, 2, 3)
    ref = torch.nn.grad.conv3d_weight(xd, (cout, cin, k, k, k), dzd, padding=(k - 1) // 2)
    ref = ref.permute(2, 3, 4, 1, 0)
    scale = float(ref.abs().max())
    # each mode against float64 (the atomic mode's order differs: stream-K ranges /
    # m splits / arrival order), at the algorithm's bar: the F(4x2x4) Winograd
    # gradient's tile sums ~1.2e-5 of the scale (test_batch_items_past_operand_bound)
    tol = (2e-5 if alg == "wino" else 1e-5) * scale

    def err(o):
        return float((o.double() - ref).abs().max())
    atomic = run()
    assert err(atomic) <= tol
    _lib.set_deterministic(True)
    outs = [run() for _ in range(3)]
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    assert err(outs[0]) <= tol
    # a scratch too small for two splits: one split per tile, plain adds
    _lib.set_deterministic(True, scratch_bytes=4096)
    one = [run() for _ in range(2)]
    torch.cuda.synchronize()
    assert torch.equal(one[0], one[1])
    assert err(one[0]) <= tol


def test_gemm_wgrad_batched_deterministic(det, cuda):
    """m3d_gemm_wgrad_f32 (batched C += A^T B, the Winograd point form) with
    accumulation into a non-zero C: deterministic and equal to fp64."""
    _lib = det
    L = _lib.load()
    g = torch.Generator().manual_seed(9)
    nb, M, K, N = 4, 4096, 256, 256
    A = torch.randn((nb, M, K), generator=g)
    Bm = torch.randn((nb, M, N), generator=g)
    C0 = torch.randn((nb, K, N), generator=g)
    ref = C0.double() + torch.bmm(A.double().transpose(1, 2), Bm.double())
    _lib.set_deterministic(True)
    Ad, Bd = A.to(cuda), Bm.to(cuda)          # held: the launch is stream-ordered
    outs = []
    for _ in range(2):
        Cd = C0.to(cuda)
        _lib.check(L.m3d_gemm_wgrad_f32(Ad.data_ptr(), Bd.data_ptr(), Cd.data_ptr(), nb, M, K, N,
                                        _lib.stream()), "gemm_wgrad")
        outs.append(Cd)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    err = float((outs[0].double().cpu() - ref).abs().max()) / float(ref.abs().max())
    assert err < 1e-5, err


def _train(cuda, steps, graphed=False):
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    cfg = synthetic_rpn_config(64, depth=16, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
    image = synthetic_volume(64, 16, seed=0).to(cuda)
    model = RPN(cfg, device=cuda, seed=5)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
    targets = RPNTargets(match, bbox, cuda)
    if graphed:
        step = model.graphed_train_step(image, targets, proposals=True, warmup=2)
        for _ in range(steps - 2):
            r = step()
    else:
        for _ in range(steps):
            r = model.train_step(image, targets, proposals=True)
    torch.cuda.synchronize()
    return float(r["loss"]), r["rpn_rois"].clone(), model.store.flat.detach().clone()


def test_train_steps_bitwise_repeatable(det, cuda):
    """Four RPN training steps (forward, backward with side-stream weight
    gradients, clip-norm SGD) twice from the same init in deterministic mode:
    identical loss, proposals and weights, bit for bit; and the HIP-graph
    replayed step equal to the eager one bit for bit."""
    _lib = det
    _lib.set_deterministic(True)
    a = _train(cuda, 4)
    b = _train(cuda, 4)
    c = _train(cuda, 4, graphed=True)
    assert a[0] == b[0] and torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert a[0] == c[0] and torch.equal(a[2], c[2])
    _lib.set_deterministic(False)
    d = _train(cuda, 4)
    assert abs(a[0] - d[0]) <= 1e-5 * abs(a[0])
    assert float((a[2] - d[2]).abs().max()) <= 1e-5 * float(a[2].abs().max())


def test_graphed_step_with_in_step_targets_bitwise(det, cuda):
    """The configs[0]-style step with its RPN targets built on the GPU every
    step (RPNTargetBuilder, a new seed each step): eager steps and the
    HIP-graph replay of the step captured over the builder's persistent
    target buffers (the builder launched before each replay, bench.py) give
    the same losses and weights bit for bit (deterministic mode)."""
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    from m3d.targets import RPNTargetBuilder
    _lib = det
    _lib.set_deterministic(True)
    cfg = synthetic_rpn_config(64, depth=16, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
    image = synthetic_volume(64, 16, seed=0).to(cuda)
    gt = torch.tensor([[0.2, 0.2, 0.2, 0.5, 0.45, 0.6], [0.55, 0.5, 0.3, 0.8, 0.9, 0.8]], device=cuda)
    runs = []
    for graphed in (False, True):
        model = RPN(cfg, device=cuda, seed=5)
        builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), cfg, max_gt=4)
        if graphed:
            step = model.graphed_train_step(image, builder(gt, seed=0), warmup=2)   # 2 steps on seed 0
            for i in range(3):
                builder(gt, seed=12 + i)
                r = step()
        else:
            t = builder(gt, seed=0)
            for _ in range(2):
                model.train_step(image, t)
            for i in range(3):
                r = model.train_step(image, builder(gt, seed=12 + i))
        torch.cuda.synchronize()
        runs.append((float(r["loss"]), model.store.flat.detach().clone()))
    assert runs[0][0] == runs[1][0] and torch.equal(runs[0][1], runs[1][1])


def test_rpn_head_shared_wino_policy_bit_identical(det, cuda, monkeypatch):
    """The RPN head's shared Winograd weight transform as the model drives it
    (m3d.nn._shared_wino_ws): forward + backward of the whole RPN with sharing
    on, off (M3D_SHARE_WINO_WEIGHTS=0) and on with a 0-byte cap
    (M3D_SHARE_WINO_MAX_GB=0: every level falls back to its own workspace) give
    bit-identical outputs and gradients (deterministic mode), and the held
    data-gradient workspace is released after the last level's call."""
    from m3d import backbone as BB
    from m3d import nn as NN
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    _lib = det
    _lib.set_deterministic(True)
    cfg = synthetic_rpn_config(64, depth=16, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=200)
    image = synthetic_volume(64, 16, seed=3).to(cuda)
    seen = []
    real_release = NN._shared_wino_release

    def spy(wshare):
        real_release(wshare)
        if wshare is not None:
            seen.append("bwd" in wshare)
    monkeypatch.setattr(NN, "_shared_wino_release", spy)
    res = []
    for share, cap in ((True, NN.SHARE_WINO_MAX_BYTES), (False, NN.SHARE_WINO_MAX_BYTES), (True, 0)):
        monkeypatch.setattr(BB, "SHARE_WINO_WEIGHTS", share)
        monkeypatch.setattr(NN, "SHARE_WINO_MAX_BYTES", cap)
        model = RPN(cfg, device=cuda, seed=7)
        match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
        seen.clear()
        r = model.forward_backward(image, RPNTargets(match, bbox, cuda), proposals=False)
        torch.cuda.synchronize()
        if share and cap > 0:
            assert len(seen) >= 2 and seen[-1] is False and all(seen[:-1]), seen
        res.append((r["loss"].clone(), model.store.grad_flat.clone()))
        del model
    for loss, grad in res[1:]:
        assert torch.equal(loss, res[0][0])
        assert torch.equal(grad, res[0][1])
