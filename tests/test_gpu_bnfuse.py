"""Fused BN-ReLU backward in the data-gradient epilogues
(m3d_conv3d_bwd_data_bn / m3d_conv3d_bwd_data_wino_bn, nn.BNFuse).

C-ABI level: the fused call against the unfused pair it replaces (data
gradient, then m3d_bn_act_bwd on it): dz and dres bit for bit (same per-element
fp32 operations), the beta / gamma / bias sums within fp32 reassociation (the
partial rows are the GEMM's / Winograd's tiles instead of bn_act_bwd's blocks)
and against float64.  Model level: the RPN training graph with the fusion on
and off (M3D_BN_FUSE): same loss, kernel gradients bit for bit, BN / bias
gradients within 1e-5 of their scale, the fused run bitwise repeatable in
deterministic mode, and the bn_act_bwd launches actually gone."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu


def _bn_state(C, dev, g):
    gamma = torch.rand(C, generator=g) + 0.5
    beta = torch.randn(C, generator=g)
    mean = torch.randn(C, generator=g)
    var = torch.rand(C, generator=g) + 0.5
    rstd = 1.0 / torch.sqrt(var + 1e-3)
    scale = gamma * rstd
    shift = beta - mean * scale
    return [t.to(dev) for t in (mean, rstd, scale, shift)]


def _unfused(L, _lib, conv, x_shape, dx0, y, z, bn, relu, res, sums):
    from m3d import nn as mnn
    dx = dx0.clone() if dx0 is not None else torch.empty(x_shape, device=y.device)
    conv(dx, 1 if dx0 is not None else 0)
    C = x_shape[-1]
    M = dx.numel() // C
    mean, rstd, scale, _ = bn
    dz = torch.empty_like(dx)
    dres = torch.empty_like(dx) if res else None
    out = [torch.zeros(C, device=dx.device) if s else None for s in sums]
    mnn.bn_act_bwd(dx, y, z, M, C, relu, scale, mean, rstd, dz, dres, *out)
    return dz, dres, out


def _fused(L, _lib, conv_bn, x_shape, dx0, y, z, bn, relu, res, sums):
    mean, rstd, scale, _ = bn
    B, H, W, D, C = x_shape
    dx = dx0.clone() if dx0 is not None else torch.empty(x_shape, device=y.device)
    dres = torch.empty_like(dx) if res else None
    out = [torch.zeros(C, device=dx.device) if s else None for s in sums]
    nb = int(L.m3d_bn_bwd_fused_workspace_bytes(B, H, W, D, C))
    ws = torch.empty(nb // 4 + 1, device=dx.device)
    p = lambda t: None if t is None else t.data_ptr()        # noqa: E731
    d = _lib.BnBwd(p(y), p(z), p(scale), p(mean), p(rstd), 1 if relu else 0, p(dres), p(out[0]), p(out[1]),
                   p(out[2]))
    conv_bn(dx, 1 if dx0 is not None else 0, ctypes.addressof(d), ws.data_ptr(), nb)
    return dx, dres, out


CASES = [
    # (algorithm, k, Cin, Cout, B, H, W, D, accumulate, relu, with z, with dres)
    ("direct", 1, 64, 256, 1, 8, 8, 16, 0, True, True, False),      # 2c's input: 2b's unit
    ("direct", 1, 256, 64, 1, 8, 8, 16, 1, True, True, True),       # identity 2a after the residual park
    ("direct", 1, 512, 256, 2, 4, 4, 8, 0, False, False, True),     # no ReLU, no gamma sum
    ("direct", 3, 32, 64, 1, 6, 6, 8, 0, True, True, False),        # 3^3 implicit-GEMM data gradient
    ("direct", 1, 4, 32, 1, 5, 3, 7, 0, True, True, True),          # ragged rows, 4 channels
    ("wino", 3, 64, 64, 1, 8, 8, 16, 0, True, True, False),         # res2 2b: 4 tiles per block row
    ("wino", 3, 256, 256, 1, 6, 10, 12, 0, True, True, False),      # one tile per partial row
    ("wino", 3, 512, 512, 1, 4, 4, 8, 1, True, False, True),        # res5-like, accumulated
    ("wino", 3, 128, 64, 2, 5, 7, 9, 0, False, True, True),         # ragged grid, batch 2
    ("splitk4", 1, 2048, 512, 1, 4, 4, 16, 1, True, True, True),    # res5 identity 2a: 4 K-slices, accumulated
    ("splitk2", 1, 1024, 256, 1, 4, 4, 8, 0, True, True, False),    # 2 K-slices
    ("x3", 1, 512, 256, 1, 16, 16, 8, 0, True, True, False),         # rpn_conv_shared1 <- shared2 (bf16-split GEMM)
    ("x3", 1, 256, 512, 1, 10, 6, 9, 0, True, True, True),           # ragged last 256-row tile, dres
    ("x3", 1, 768, 1024, 2, 8, 8, 8, 0, False, False, True),         # no ReLU / gamma sum, 3 N-tiles
    ("x3", 1, 256, 64, 1, 16, 16, 8, 1, True, True, True),           # identity 2a: K = 64, accumulated (_bna)
    ("x3", 1, 512, 128, 1, 10, 6, 9, 1, True, True, False),          # ragged last tile, accumulated
]


@pytest.mark.parametrize("alg,k,cin,cout,B,H,W,D,acc,relu,withz,res", CASES)
def test_fused_matches_unfused(cuda, alg, k, cin, cout, B, H, W, D, acc, relu, withz, res):
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(11)
    x_shape = (B, H, W, D, cin)
    dz_in = torch.randn((B, H, W, D, cout), generator=g).to(cuda)
    w = (torch.randn((k, k, k, cin, cout), generator=g) * 0.05).to(cuda)
    bn = _bn_state(cin, cuda, g)
    zpre = torch.randn(x_shape, generator=g).to(cuda)
    y = zpre * bn[2] + bn[3]
    if relu:
        y = torch.relu(y)
    z = zpre if withz else None
    dx0 = torch.randn(x_shape, generator=g).to(cuda) if acc else None
    sums = (True, withz, True)
    st = _lib.stream()
    pad = (k - 1) // 2
    if alg == "wino":
        nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, cin, cout))
        ws = torch.empty(nb // 4 + 1, device=cuda)

        def conv(dx, a):
            _lib.check(L.m3d_conv3d_bwd_data_wino(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, cout, D, 1,
                                                  dx.data_ptr(), a, ws.data_ptr(), nb, st), "wino dgrad")

        def conv_bn(dx, a, d, bws, bwsb):
            _lib.check(L.m3d_conv3d_bwd_data_wino_bn(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, cout, D, 1,
                                                     dx.data_ptr(), a, ws.data_ptr(), nb, 0, d, bws, bwsb, st),
                       "wino dgrad bn")
    elif alg.startswith("splitk"):
        sp = int(alg[6:])
        wsk = torch.empty(sp * B * H * W * D * cin, device=cuda)

        def conv(dx, a):
            _lib.check(L.m3d_conv3d_bwd_data_splitk(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, cout, H, W, D,
                                                    1, 1, 1, dx.data_ptr(), a, sp, wsk.data_ptr(), wsk.numel() * 4,
                                                    st), "dgrad split-K")

        def conv_bn(dx, a, d, bws, bwsb):
            _lib.check(L.m3d_conv3d_bwd_data_splitk_bn(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, cout,
                                                       dx.data_ptr(), a, sp, wsk.data_ptr(), wsk.numel() * 4, d, bws,
                                                       bwsb, st), "dgrad split-K bn")
    elif alg == "x3":
        planes = torch.empty(3 * cin * cout, device=cuda, dtype=torch.int16)
        _lib.check(L.m3d_conv1_x3_planes(w.data_ptr(), cin, cout, 0, planes.data_ptr(), st), "planes")

        def conv(dx, a):
            # accumulate: the split GEMM into a temporary, then dx + t (one fp32 add,
            # the fused epilogue's t = acc + dx: IEEE addition commutes bit for bit)
            t = torch.empty_like(dx) if a else dx
            _lib.check(L.m3d_conv3d_bwd_data_x3(dz_in.data_ptr(), planes.data_ptr(), B, H, W, D, cin, cout,
                                                t.data_ptr(), st), "dgrad x3")
            if a:
                dx.add_(t)

        def conv_bn(dx, a, d, bws, bwsb):
            if a:
                _lib.check(L.m3d_conv3d_bwd_data_x3_bna(dz_in.data_ptr(), planes.data_ptr(), B, H, W, D, cin, cout,
                                                        dx.data_ptr(), a, d, bws, bwsb, st), "dgrad x3 bna")
            else:
                _lib.check(L.m3d_conv3d_bwd_data_x3_bn(dz_in.data_ptr(), planes.data_ptr(), B, H, W, D, cin, cout,
                                                       dx.data_ptr(), d, bws, bwsb, st), "dgrad x3 bn")
    else:
        def conv(dx, a):
            _lib.check(L.m3d_conv3d_bwd_data(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, k, k, k, cout, H, W,
                                             D, 1, 1, 1, pad, pad, pad, dx.data_ptr(), a, st), "dgrad")

        def conv_bn(dx, a, d, bws, bwsb):
            _lib.check(L.m3d_conv3d_bwd_data_bn(dz_in.data_ptr(), w.data_ptr(), B, H, W, D, cin, k, k, k, cout, H,
                                                W, D, 1, 1, 1, pad, pad, pad, dx.data_ptr(), a, d, bws, bwsb, st),
                       "dgrad bn")
    ref = _unfused(L, _lib, conv, x_shape, dx0, y, z, bn, relu, res, sums)
    got = _fused(L, _lib, conv_bn, x_shape, dx0, y, z, bn, relu, res, sums)
    torch.cuda.synchronize()
    assert torch.equal(got[0], ref[0]), float((got[0] - ref[0]).abs().max())
    if res:
        assert torch.equal(got[1], ref[1])
    # sums: fused vs unfused within fp32 reassociation, bounded per channel by
    # the sum of the terms' magnitudes (float64, from the bit-exact dz)
    mean, rstd, scale, _ = bn
    g64 = (ref[0].double() / scale.double()).reshape(-1, cin)
    xhat = ((zpre.double() - mean.double()) * rstd.double()).reshape(-1, cin)
    mags = [g64.abs().sum(0), (g64 * xhat).abs().sum(0), (g64 * scale.double()).abs().sum(0)]
    exact = [g64.sum(0), (g64 * xhat).sum(0), (g64 * scale.double()).sum(0)]
    for i, (a, b) in enumerate(zip(got[2], ref[2])):
        if b is None:
            continue
        bound = 1e-5 * mags[i] + 1e-30
        assert bool(((a.double() - b.double()).abs() <= bound).all()), i
        assert bool(((a.double() - exact[i]).abs() <= bound).all()), i


def test_fused_refuses_bad_descriptors(cuda):
    from m3d import _lib
    L = _lib.load()
    dz = torch.zeros((1, 4, 4, 4, 32), device=cuda)
    w = torch.zeros((1, 1, 1, 64, 32), device=cuda)
    dx = torch.zeros((1, 4, 4, 4, 64), device=cuda)
    y = torch.zeros_like(dx)
    s = torch.zeros(64, device=cuda)
    st = _lib.stream()
    args = (dz.data_ptr(), w.data_ptr(), 1, 4, 4, 4, 64, 1, 1, 1, 32, 4, 4, 4, 1, 1, 1, 0, 0, 0, dx.data_ptr(), 0)
    # relu without y
    d = _lib.BnBwd(None, None, None, None, None, 1, None, None, None, None)
    assert L.m3d_conv3d_bwd_data_bn(*args, ctypes.addressof(d), None, 0, st) != 0
    # sums without a workspace
    d = _lib.BnBwd(y.data_ptr(), None, None, None, None, 1, None, s.data_ptr(), None, None)
    assert L.m3d_conv3d_bwd_data_bn(*args, ctypes.addressof(d), None, 0, st) != 0
    # null descriptor
    assert L.m3d_conv3d_bwd_data_bn(*args, None, None, 0, st) != 0
    # strided data gradients have no fused form
    dzs = torch.zeros((1, 2, 2, 4, 32), device=cuda)
    d = _lib.BnBwd(y.data_ptr(), None, None, None, None, 1, None, None, None, None)
    assert L.m3d_conv3d_bwd_data_bn(dzs.data_ptr(), w.data_ptr(), 1, 4, 4, 4, 64, 1, 1, 1, 32, 2, 2, 4, 2, 2, 1,
                                    0, 0, 0, dx.data_ptr(), 0, ctypes.addressof(d), None, 0, st) != 0
    # Winograd: Cin must divide 256 or be a multiple of it
    assert L.m3d_conv3d_bwd_data_wino_bn(dz.data_ptr(), w.data_ptr(), 1, 4, 4, 4, 96, 32, 4, 1, dx.data_ptr(), 0,
                                         None, 0, 0, ctypes.addressof(d), None, 0, st) != 0


def _step(cuda, fuse, monkeypatch, log=None):
    from m3d import nn as mnn
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    monkeypatch.setattr(mnn, "BN_FUSE", fuse)
    cfg = synthetic_rpn_config(64, depth=16, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=200)
    image = synthetic_volume(64, 16, seed=3).to(cuda)
    model = RPN(cfg, device=cuda, seed=7)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
    monkeypatch.setattr(mnn, "LAYER_LOG", log)
    r = model.forward_backward(image, RPNTargets(match, bbox, cuda), proposals=False)
    monkeypatch.setattr(mnn, "LAYER_LOG", None)
    torch.cuda.synchronize()
    return r["loss"].clone(), model.store.grad_flat.clone(), [(p.name, p.grad.clone()) for p in model.store.params]


def test_model_fused_vs_unfused(cuda, monkeypatch):
    from m3d import _lib
    _lib.set_deterministic(True)
    try:
        log_on, log_off = [], []
        l_on, flat_on, g_on = _step(cuda, True, monkeypatch, log_on)
        l_on2, flat_on2, _ = _step(cuda, True, monkeypatch)
        l_off, _, g_off = _step(cuda, False, monkeypatch, log_off)
    finally:
        _lib.set_deterministic(False)
    n_on = sum(1 for r in log_on if r[0] == "bn_act_bwd")
    n_off = sum(1 for r in log_off if r[0] == "bn_act_bwd")
    # 16 blocks x (2a -> 2b, 2b -> 2c) + 12 block -> block inside the stages + the
    # RPN head's shared1 -> shared2 and shared2 -> class/bbox heads on 5 levels
    # (fewer where shared2's data gradient runs the x3 GEMM, which has no fused form)
    left = [r[5] for r in log_on if r[0] == "bn_act_bwd"]
    print("bn_act_bwd left with the fusion on:", n_on, "of", n_off, left)
    assert n_off - n_on >= 49, (n_on, n_off, left)
    assert torch.equal(l_on, l_on2)
    assert torch.equal(flat_on, flat_on2)
    assert abs(float(l_on) - float(l_off)) <= 1e-6 * abs(float(l_off))
    for (name, a), (_, b) in zip(g_on, g_off):
        scale = float(b.abs().max()) + 1e-30
        if name.endswith("/kernel:0"):
            assert torch.equal(a, b), name
        else:   # beta / gamma / bias: the sums' partial rows differ
            assert float((a - b).abs().max()) <= 1e-5 * scale, name
