"""Depth-slab kernels that read the neighbours' halo planes beside the slab
(m3d_maxpool3d_{fwd,bwd}_halo, m3d_conv3d_fwd_halo for the 7^3 stem,
m3d_conv3d_bwd_weight_halo for the direct weight gradient) against the same
kernels on the halo-extended copy of the slab (torch.cat of [lower halo, slab,
upper halo], the path they replace): forward values and argmax bit-identical,
the pool's slab / halo gradients bit-identical to the extended gradient's
planes, weight gradients equal up to the fp32 atomics' order.  Every
neighbour pattern: interior slab, lowest slab, highest slab."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NEIGHBOURS = [(1, 1), (0, 1), (1, 0)]


def _ext(x, halo, has_lo, has_hi, r):
    parts = ([halo[:, :, :, :r]] if has_lo else []) + [x] + ([halo[:, :, :, r:]] if has_hi else [])
    return torch.cat(parts, dim=3).contiguous()


@pytest.mark.parametrize("has_lo,has_hi", NEIGHBOURS)
def test_maxpool_halo_equals_extended(cuda, has_lo, has_hi):
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(5)
    B, H, W, D, C, r = 1, 10, 12, 6, 64, 1
    # quantised values: ties inside a window exercise the first-max rule
    x = torch.round(torch.randn((B, H, W, D, C), device=cuda, generator=g) * 4) / 4
    halo = torch.round(torch.randn((B, H, W, 2 * r, C), device=cuda, generator=g) * 4) / 4
    k, st, (py, px) = (3, 3, 3), (2, 2, 1), (0, 0)
    OH, OW, OD = (H + 1) // 2, (W + 1) // 2, D
    py = max((OH - 1) * 2 + 3 - H, 0) // 2
    px = max((OW - 1) * 2 + 3 - W, 0) // 2
    y = torch.empty((B, OH, OW, OD, C), device=cuda)
    am = torch.empty((B, OH, OW, OD, C), device=cuda, dtype=torch.uint8)
    _lib.check(L.m3d_maxpool3d_fwd_halo(x.data_ptr(), halo.data_ptr(), has_lo, has_hi, r, B, H, W, D, C, *k, *st,
                                        py, px, 1, OH, OW, OD, y.data_ptr(), am.data_ptr(), _lib.stream()))
    xe = _ext(x, halo, has_lo, has_hi, r)
    nlo = r if has_lo else 0
    ye = torch.empty_like(y)
    ame = torch.empty_like(am)
    _lib.check(L.m3d_maxpool3d_fwd(xe.data_ptr(), B, H, W, xe.shape[3], C, *k, *st, py, px, 1 - nlo, OH, OW, OD,
                                   ye.data_ptr(), ame.data_ptr(), _lib.stream()))
    assert torch.equal(y, ye) and torch.equal(am, ame)
    dy = torch.randn(y.shape, device=cuda, generator=g)
    dx = torch.empty_like(x)
    dh = torch.zeros_like(halo)
    _lib.check(L.m3d_maxpool3d_bwd_halo(dy.data_ptr(), am.data_ptr(), has_lo, has_hi, r, B, H, W, D, C, *k, *st,
                                        py, px, 1, OH, OW, OD, dx.data_ptr(), dh.data_ptr(), _lib.stream()))
    dxe = torch.empty_like(xe)
    _lib.check(L.m3d_maxpool3d_bwd(dy.data_ptr(), ame.data_ptr(), B, H, W, xe.shape[3], C, *k, *st, py, px,
                                   1 - nlo, OH, OW, OD, dxe.data_ptr(), _lib.stream()))
    assert torch.equal(dx, dxe[:, :, :, nlo:nlo + D])
    if has_lo:
        assert torch.equal(dh[:, :, :, :r], dxe[:, :, :, :r])
    if has_hi:
        assert torch.equal(dh[:, :, :, r:], dxe[:, :, :, nlo + D:])


def test_maxpool_halo_rejects_bad_geometry(cuda):
    from m3d import _lib
    L = _lib.load()
    x = torch.zeros((1, 4, 4, 4, 8), device=cuda)
    h = torch.zeros((1, 4, 4, 2, 8), device=cuda)
    y = torch.empty((1, 2, 2, 4, 8), device=cuda)
    am = torch.empty((1, 2, 2, 4, 8), device=cuda, dtype=torch.uint8)
    rc = L.m3d_maxpool3d_fwd_halo(x.data_ptr(), h.data_ptr(), 1, 1, 1, 1, 4, 4, 4, 8, 3, 3, 3, 2, 2, 2, 0, 0, 1,
                                  2, 2, 4, y.data_ptr(), am.data_ptr(), _lib.stream())
    assert rc != 0                                   # z-stride 2: not a 'same' slab window


def _stem_weights(cuda, g, cin, cout, k):
    return torch.randn((k, k, k, cin, cout), device=cuda, generator=g) / float(k ** 3 * cin) ** 0.5


@pytest.mark.parametrize("has_lo,has_hi", NEIGHBOURS)
def test_stem_halo_equals_extended(cuda, has_lo, has_hi):
    """conv1 (7^3, 1 -> 64, strides (2,2,1), ZeroPadding3D(3)) on a slab of 16
    planes with 3 halo planes per side: stem_fwd_kernel bit-identical, the
    direct weight gradient within the atomics' order."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(7)
    B, H, W, D, r = 1, 24, 20, 16, 3
    x = torch.tanh(0.5 * torch.randn((B, H, W, D, 1), device=cuda, generator=g))
    halo = torch.tanh(0.5 * torch.randn((B, H, W, 2 * r, 1), device=cuda, generator=g))
    w = _stem_weights(cuda, g, 1, 64, 7)
    bias = torch.randn(64, device=cuda, generator=g) * 0.1
    scale = 1 + 0.1 * torch.randn(64, device=cuda, generator=g)
    shift = 0.1 * torch.randn(64, device=cuda, generator=g)
    OH, OW, OD = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1, D
    y = torch.empty((B, OH, OW, OD, 64), device=cuda)
    z = torch.empty_like(y)
    _lib.check(L.m3d_conv3d_fwd_halo(x.data_ptr(), halo.data_ptr(), has_lo, has_hi, r, B, H, W, D, 1, w.data_ptr(),
                                     7, 7, 7, 64, OH, OW, OD, 2, 2, 1, 3, 3, 3, bias.data_ptr(), scale.data_ptr(),
                                     shift.data_ptr(), 1, z.data_ptr(), y.data_ptr(), _lib.stream()))
    xe = _ext(x, halo, has_lo, has_hi, r)
    nlo = r if has_lo else 0
    ye, ze = torch.empty_like(y), torch.empty_like(y)
    _lib.check(L.m3d_conv3d_fwd(xe.data_ptr(), B, H, W, xe.shape[3], 1, w.data_ptr(), 7, 7, 7, 64, OH, OW, OD,
                                2, 2, 1, 3, 3, 3 - nlo, bias.data_ptr(), scale.data_ptr(), shift.data_ptr(), None,
                                0, 1, ze.data_ptr(), ye.data_ptr(), 64, None, 0, 0, _lib.stream()))
    assert torch.equal(y, ye) and torch.equal(z, ze)
    dz = torch.randn(y.shape, device=cuda, generator=g)
    dw = torch.zeros_like(w)
    dwe = torch.zeros_like(w)
    _lib.check(L.m3d_conv3d_bwd_weight_halo(x.data_ptr(), halo.data_ptr(), has_lo, has_hi, r, dz.data_ptr(), B, H,
                                            W, D, 1, 7, 7, 7, 64, OH, OW, OD, 2, 2, 1, 3, 3, 3, dw.data_ptr(),
                                            _lib.stream()))
    _lib.check(L.m3d_conv3d_bwd_weight(xe.data_ptr(), dz.data_ptr(), B, H, W, xe.shape[3], 1, 7, 7, 7, 64, OH, OW,
                                       OD, 2, 2, 1, 3, 3, 3 - nlo, dwe.data_ptr(), _lib.stream()))
    torch.cuda.synchronize()
    assert float((dw - dwe).abs().max()) <= 1e-5 * float(dwe.abs().max())


@pytest.mark.parametrize("has_lo,has_hi", NEIGHBOURS)
def test_direct_wgrad_halo_equals_extended(cuda, has_lo, has_hi):
    """The 64-channel 3^3 convs of stage 2 (res2*_branch2b: Winograd forward,
    direct weight gradient) on a slab with one halo plane per side."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(9)
    B, H, W, D, C, r = 1, 8, 6, 12, 64, 1
    x = torch.randn((B, H, W, D, C), device=cuda, generator=g)
    halo = torch.randn((B, H, W, 2 * r, C), device=cuda, generator=g)
    dz = torch.randn((B, H, W, D, C), device=cuda, generator=g)
    dw = torch.zeros((3, 3, 3, C, C), device=cuda)
    dwe = torch.zeros_like(dw)
    _lib.check(L.m3d_conv3d_bwd_weight_halo(x.data_ptr(), halo.data_ptr(), has_lo, has_hi, r, dz.data_ptr(), B, H,
                                            W, D, C, 3, 3, 3, C, H, W, D, 1, 1, 1, 1, 1, 1, dw.data_ptr(),
                                            _lib.stream()))
    xe = _ext(x, halo, has_lo, has_hi, r)
    nlo = r if has_lo else 0
    _lib.check(L.m3d_conv3d_bwd_weight(xe.data_ptr(), dz.data_ptr(), B, H, W, xe.shape[3], C, 3, 3, 3, C, H, W, D,
                                       1, 1, 1, 1, 1, 1 - nlo, dwe.data_ptr(), _lib.stream()))
    torch.cuda.synchronize()
    assert float((dw - dwe).abs().max()) <= 1e-5 * float(dwe.abs().max())
    # and against float64 on the host
    xd = xe.double().cpu().permute(0, 4, 1, 2, 3)
    xd = torch.nn.functional.pad(xd, (1 - nlo, 1 - (r if has_hi else 0), 1, 1, 1, 1))
    dzd = dz.double().cpu().permute(0, 4, 1, 2, 3)
    ref = torch.nn.grad.conv3d_weight(xd, (C, C, 3, 3, 3), dzd)          # [Cout, Cin, kh, kw, kd]
    ref = ref.permute(2, 3, 4, 1, 0)
    assert float((dw.double().cpu() - ref).abs().max()) <= 1e-5 * float(ref.abs().max())


@pytest.mark.parametrize("has_lo,has_hi,Dl", [(1, 1, 16), (0, 1, 8), (1, 0, 4), (1, 1, 12)])
def test_wino_halo_phases_equal_one_launch(cuda, has_lo, has_hi, Dl):
    """m3d_conv3d_fwd_wino_halo_phase 1 (weights + interior z tiles, before the
    halo planes exist -- the buffer is filled only afterwards) then 2 (edge
    tiles, GEMM, output) == the one-launch m3d_conv3d_fwd_wino_halo, bit for
    bit; Dl = 4 has no interior tile."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(11)
    B, H, W, Cin, Cout = 1, 6, 10, 64, 128
    x = torch.randn((B, H, W, Dl, Cin), device=cuda, generator=g)
    halo_src = torch.randn((B, H, W, 2, Cin), device=cuda, generator=g)
    w = torch.randn((3, 3, 3, Cin, Cout), device=cuda, generator=g) / (27 * Cin) ** 0.5
    bias = torch.randn(Cout, device=cuda, generator=g) * 0.1
    res = torch.randn((B, H, W, Dl, Cout), device=cuda, generator=g)
    dext = Dl + has_lo + has_hi
    nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, dext, Dl, Cin, Cout))
    outs = []
    for phased in (False, True):
        ws = torch.full((nb // 4 + 1,), float("nan"), device=cuda)
        y = torch.empty((B, H, W, Dl, Cout), device=cuda)
        z = torch.empty_like(y)
        args = (B, H, W, Dl, Cin, w.data_ptr(), Cout, bias.data_ptr(), None, None, res.data_ptr(), 1,
                z.data_ptr(), y.data_ptr(), None, ws.data_ptr(), nb)
        if phased:
            halo = torch.full_like(halo_src, float("nan"))      # not yet arrived
            _lib.check(L.m3d_conv3d_fwd_wino_halo_phase(x.data_ptr(), None, has_lo, has_hi, *args, 1,
                                                        _lib.stream()))
            halo.copy_(halo_src)
            _lib.check(L.m3d_conv3d_fwd_wino_halo_phase(x.data_ptr(), halo.data_ptr(), has_lo, has_hi, *args, 2,
                                                        _lib.stream()))
        else:
            _lib.check(L.m3d_conv3d_fwd_wino_halo(x.data_ptr(), halo_src.data_ptr(), has_lo, has_hi, *args,
                                                  _lib.stream()))
        outs.append((y, z))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    assert torch.isfinite(outs[1][0]).all()
