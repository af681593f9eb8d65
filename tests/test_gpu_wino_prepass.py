"""The Winograd weight pre-pass (m3d.nn.WinoVPrep: every 3x3x3 kernel's
forward and data-gradient transforms produced by m3d_conv3d_wino_weight_v on a
side stream at the start of the forward, consumed by m3d_conv3d_fwd_wino_kv /
m3d_conv3d_bwd_data_wino_xv): the same kernels on the same inputs, so a
training step with it equals the step without it bit for bit (deterministic
mode), eagerly and as a HIP-graph replay."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dgrad_only_refresh(refresh):
    def wrapped(self, dev):
        self.active_fwd = False          # RPN.forward set both: keep the data gradient's only
        return refresh(self, dev)
    return wrapped


def _steps(cuda, prepass, monkeypatch, n=3, graph=False, fwd=True):
    from m3d import _lib
    from m3d import nn as mnn
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    monkeypatch.setattr(mnn, "WINO_V_PREPASS", prepass)
    monkeypatch.setattr(mnn, "WINO_V_PREPASS_MIN_VOXELS", 0)     # the test volume is small
    if not fwd:   # the data gradient's transforms alone on the pre-pass
        monkeypatch.setattr(mnn.WinoVPrep, "refresh", _dgrad_only_refresh(mnn.WinoVPrep.refresh))
    cfg = synthetic_rpn_config(64, depth=32, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=200)
    image = synthetic_volume(64, 32, seed=3).to(cuda)
    model = RPN(cfg, device=cuda, seed=7)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
    t = RPNTargets(match, bbox, cuda)
    losses = []
    if graph:
        step = model.graphed_train_step(image, t, proposals=False, warmup=2)
        for _ in range(n):
            losses.append(float(step()["loss"]))
    else:
        for _ in range(n):
            r = model.train_step(image, t, proposals=False)
            losses.append(float(r["loss"]))
    torch.cuda.synchronize()
    return losses, model.store.flat.clone()


@pytest.mark.parametrize("fwd", [True, False], ids=["fwd+dgrad", "dgrad"])
@pytest.mark.parametrize("graph", [False, True], ids=["eager", "graph"])
def test_wino_prepass_step_bitwise(cuda, monkeypatch, graph, fwd):
    from m3d import _lib
    from m3d import nn as mnn
    _lib.set_deterministic(True)
    try:
        l0, w0 = _steps(cuda, False, monkeypatch, graph=graph)
        g0 = mnn.WINO_V.gen
        l1, w1 = _steps(cuda, True, monkeypatch, graph=graph, fwd=fwd)
    finally:
        _lib.set_deterministic(False)
    assert mnn.WINO_V.gen > g0 and len(mnn.WINO_V.entries) > 0
    assert l0 == l1
    assert torch.equal(w0, w1)


def test_wino_v_entry_matches_inline_transform(cuda):
    """m3d_conv3d_fwd_wino_kv / _bwd_data_wino_xv with m3d_conv3d_wino_weight_v's
    buffers give the bits of the entries that transform inline."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(3)
    B, H, W, D, Cin, Cout = 1, 8, 8, 16, 64, 128
    x = torch.randn((B, H, W, D, Cin), device=cuda, generator=g)
    w = torch.randn((3, 3, 3, Cin, Cout), device=cuda, generator=g) * 0.05
    dz = torch.randn((B, H, W, D, Cout), device=cuda, generator=g)
    nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, Cin, Cout))
    ws = torch.empty(nb // 4 + 1, device=cuda)
    p = lambda t: t.data_ptr()   # noqa: E731
    st = _lib.stream()
    y0, y1 = torch.empty((B, H, W, D, Cout), device=cuda), torch.empty((B, H, W, D, Cout), device=cuda)
    _lib.check(L.m3d_conv3d_fwd_wino(p(x), B, H, W, D, Cin, p(w), Cout, D, 1, None, None, None, None, 1, None, p(y0),
                                     p(ws), nb, st))
    vb = int(L.m3d_conv3d_wino_v_bytes(Cin, Cout, 0, 0))
    v = torch.empty(vb // 4 + 1, device=cuda)
    _lib.check(L.m3d_conv3d_wino_weight_v(p(w), Cin, Cout, 0, 0, p(v), vb, st))
    _lib.check(L.m3d_conv3d_fwd_wino_kv(p(x), B, H, W, D, Cin, p(w), Cout, D, 1, None, None, None, None, 1, None,
                                        p(y1), None, p(v), p(ws), nb, st))
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    for ty in (0, 2, 4):
        dx0, dx1 = torch.empty_like(x), torch.empty_like(x)
        _lib.check(L.m3d_conv3d_bwd_data_wino_vy(p(dz), p(w), B, H, W, D, Cin, Cout, D, 1, p(dx0), 0, p(ws), nb, 0,
                                                 ty, st))
        vb = int(L.m3d_conv3d_wino_v_bytes(Cin, Cout, 1, ty))
        v = torch.empty(vb // 4 + 1, device=cuda)
        _lib.check(L.m3d_conv3d_wino_weight_v(p(w), Cin, Cout, 1, ty, p(v), vb, st))
        _lib.check(L.m3d_conv3d_bwd_data_wino_xv(p(dz), p(w), B, H, W, D, Cin, Cout, D, 1, p(dx1), 0, p(ws), nb,
                                                 p(v), ty, None, None, 0, st))
        torch.cuda.synchronize()
        assert torch.equal(dx0, dx1), ty
    # refused: a buffer too small, a bad tile
    assert L.m3d_conv3d_wino_weight_v(p(w), Cin, Cout, 0, 0, p(v), 16, st) != 0
    assert L.m3d_conv3d_wino_v_bytes(Cin, Cout, 1, 3) == 0
