"""GPU parity of the conv / pooling / optimizer kernels against the float64
PyTorch-CPU restatement of the Keras graph (oracle/model_ref.py).
Tolerance (north_star): fp32 results within 1e-4 relative to the output scale."""
import os
import zlib

import numpy as np
import pytest
import torch

from oracle import model_ref as MR

pytestmark = pytest.mark.gpu


def close(got, ref, rtol=1e-4):
    got = got.detach().double().cpu()
    ref = ref.detach().double().cpu()
    scale = float(ref.abs().max()) + 1e-12
    err = float((got - ref).abs().max())
    assert err <= rtol * scale, f"max err {err:.3e} vs scale {scale:.3e}"


def _join():
    """Weight gradients run on the side stream (m3d.nn.WGRAD_STREAM): join it
    before reading them, as RPNHead.finish_backward does in the model."""
    from m3d.nn import join_wgrad
    join_wgrad()


class _Layer:
    """Minimal stand-in of params.ConvLayer over explicit tensors."""

    class P:
        def __init__(self, data, grad):
            self.data, self.grad = data, grad

    def __init__(self, w, b):
        self.kernel = self.P(w, torch.zeros_like(w))
        self.bias = self.P(b, torch.zeros_like(b)) if b is not None else None
        self.k = tuple(w.shape[:3])

    def grad_dict(self, bn=None):
        g = {"kernel": self.kernel.grad, "bias": self.bias.grad if self.bias else None}
        if bn is not None:
            g["gamma"], g["beta"] = bn.gamma.grad, bn.beta.grad
        return g


class _BN:
    def __init__(self, c, dev, rng):
        self.gamma = _Layer.P(torch.tensor(rng.uniform(0.5, 1.5, c), dtype=torch.float32, device=dev),
                              torch.zeros(c, device=dev))
        self.beta = _Layer.P(torch.tensor(rng.normal(0, 0.1, c), dtype=torch.float32, device=dev),
                             torch.zeros(c, device=dev))
        self.moving_mean = torch.tensor(rng.normal(0, 0.2, c), dtype=torch.float32, device=dev)
        self.moving_variance = torch.tensor(rng.uniform(0.5, 2.0, c), dtype=torch.float32, device=dev)
        self.eps = 1e-3


CASES = [
    # (in spatial, Cin, Cout, k, stride, padding, bn, relu, residual)
    ((8, 8, 6), 64, 256, (1, 1, 1), (1, 1, 1), "valid", True, True, False),
    ((8, 8, 6), 256, 128, (1, 1, 1), (2, 2, 1), "valid", True, True, False),
    ((6, 6, 5), 64, 64, (3, 3, 3), (1, 1, 1), "same", True, True, False),
    ((4, 4, 7), 128, 96, (3, 3, 3), (1, 1, 1), "same", False, True, False),
    ((5, 5, 4), 256, 24, (1, 1, 1), (1, 1, 1), "valid", False, False, False),
    ((6, 6, 4), 64, 256, (1, 1, 1), (1, 1, 1), "valid", True, True, True),
    ((16, 16, 6), 1, 64, (7, 7, 7), (2, 2, 1), 3, True, True, False),
    ((14, 12, 40), 1, 64, (7, 7, 7), (2, 2, 1), 3, True, True, False),   # stem: two z tiles, a partial one
    ((64, 60, 8), 1, 64, (7, 7, 7), (2, 2, 1), 3, True, True, False),    # stem: several tiles per wave
    ((20, 18, 80), 1, 64, (7, 7, 7), (2, 2, 1), 3, True, True, False),   # stem: windows inside the volume
    ((3, 5, 9), 32, 160, (3, 3, 3), (1, 1, 1), "same", True, False, True),
    ((8, 8, 6), 256, 64, (1, 1, 1), (1, 1, 1), "valid", True, True, False),   # x3_wgrad64_kernel, 4 x 1 tiles
]


@pytest.mark.parametrize("wino", [True, False], ids=["wino", "direct"])
@pytest.mark.parametrize("case", CASES, ids=[str(i) for i in range(len(CASES))])
def test_conv_block_fwd_bwd(cuda, case, wino, monkeypatch):
    import m3d.nn as mnn
    from m3d.nn import conv_bn_act, conv_geom
    monkeypatch.setattr(mnn, "WINOGRAD", wino)
    monkeypatch.setattr(mnn, "WINO_MIN_C", 32)
    sp, cin, cout, k, stride, padding, use_bn, relu, use_res = case
    # stable per-case seed (Python's str hash is randomised per process)
    rng = np.random.default_rng(zlib.crc32(repr(case).encode()) + (0 if wino else 1 << 32))
    x = torch.tensor(rng.normal(size=(2, *sp, cin)), dtype=torch.float32)
    w = torch.tensor(rng.normal(0, 1.0 / np.sqrt(np.prod(k) * cin), (*k, cin, cout)), dtype=torch.float32)
    b = torch.tensor(rng.normal(0, 0.1, cout), dtype=torch.float32)
    geo = conv_geom(sp, k, stride, padding)
    res = torch.tensor(rng.normal(size=(2, *geo.out, cout)), dtype=torch.float32) if use_res else None
    layer = _Layer(w.to(cuda), b.to(cuda))
    bn = _BN(cout, cuda, rng) if use_bn else None
    xg = x.to(cuda).requires_grad_(cin != 1)
    rg = res.to(cuda).requires_grad_(True) if use_res else None
    # anchor tensor so the stem (input without grad) is still recorded
    layer.kernel.data.requires_grad_(True)
    y = conv_bn_act(xg, layer, geo, relu, residual=rg, res_mode=1 if use_res else 0, bn=bn,
                    need_dx=cin != 1)
    # float64 reference with autograd
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    yr = MR.conv3d(xr, wr, br, stride, padding)
    if use_bn:
        gr = bn.gamma.data.cpu().double().requires_grad_(True)
        ber = bn.beta.data.cpu().double().requires_grad_(True)
        yr = MR.batchnorm(yr, gr, ber, bn.moving_mean.cpu().double(), bn.moving_variance.cpu().double())
    rr = None
    if use_res:
        rr = res.double().requires_grad_(True)
        yr = yr + rr
    if relu:
        # the ReLU branch taken as the GPU forward took it: a pre-activation
        # within fp32 rounding of 0 may land on the other side in float64, and
        # one flipped element moves a weight gradient by O(x * dy)
        yr = yr * (y.detach().double().cpu() > 0)
    close(y, yr)
    g = torch.tensor(rng.normal(size=yr.shape), dtype=torch.float32)
    y.backward(g.to(cuda))
    _join()
    yr.backward(g.double())
    close(layer.kernel.grad, wr.grad)
    close(layer.bias.grad, br.grad)
    if cin != 1:
        close(xg.grad, xr.grad)
    if use_bn:
        close(bn.gamma.grad, gr.grad)
        close(bn.beta.grad, ber.grad)
    if use_res:
        close(rg.grad, rr.grad)


def test_fpn_upsample_residual(cuda):
    from m3d.nn import conv_bn_act, conv_geom
    rng = np.random.default_rng(11)
    c4 = torch.tensor(rng.normal(size=(1, 8, 8, 5, 64)), dtype=torch.float32)
    p5 = torch.tensor(rng.normal(size=(1, 4, 4, 5, 32)), dtype=torch.float32)
    w = torch.tensor(rng.normal(0, 0.1, (1, 1, 1, 64, 32)), dtype=torch.float32)
    b = torch.tensor(rng.normal(0, 0.1, 32), dtype=torch.float32)
    layer = _Layer(w.to(cuda).requires_grad_(True), b.to(cuda))
    x = c4.to(cuda).requires_grad_(True)
    r = p5.to(cuda).requires_grad_(True)
    y = conv_bn_act(x, layer, conv_geom((8, 8, 5), (1, 1, 1), (1, 1, 1), "valid"), False,
                    residual=r, res_mode=2)
    xr, rr = c4.double().requires_grad_(True), p5.double().requires_grad_(True)
    yr = MR.upsample221(rr) + MR.conv3d(xr, w.double(), b.double(), (1, 1, 1), "valid")
    close(y, yr)
    g = torch.randn(yr.shape)
    y.backward(g.to(cuda))
    _join()
    yr.backward(g.double())
    close(r.grad, rr.grad)
    close(x.grad, xr.grad)


@pytest.mark.parametrize("C", [8, 6])
def test_maxpool_same_and_subsample(cuda, C):
    """C = 8: the float4 kernels; C = 6: the generic per-element kernels."""
    from m3d.nn import max_pool3d, subsample221
    rng = np.random.default_rng(12)
    x = torch.tensor(rng.normal(size=(2, 10, 12, 7, C)), dtype=torch.float32)
    xg = x.to(cuda).requires_grad_(True)
    y = max_pool3d(xg, (3, 3, 3), (2, 2, 1), "same")
    xr = x.double().requires_grad_(True)
    yr = MR.maxpool3d_same(xr)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), yr.detach().float().numpy())
    g = torch.randn(yr.shape)
    y.backward(g.to(cuda))
    _join()
    yr.backward(g.double())
    close(xg.grad, xr.grad, rtol=1e-6)
    if C % 4:
        return                                   # subsample221 is float4-only
    s = subsample221(xg)
    np.testing.assert_array_equal(s.detach().cpu().numpy(), x[:, ::2, ::2].numpy())


@pytest.mark.parametrize("shape", [(1, 16, 16, 21, 64), (2, 9, 7, 8, 16), (1, 12, 10, 3, 32)])
def test_maxpool_333_specialised_equals_general(cuda, shape):
    """maxpool_fwd333 / bwd333 (the stem pool, (3,3,3) / (2,2,1) 'same') against
    the general z-run kernels they replace, run through the slab form with no
    neighbours (m3d_maxpool3d_*_halo: the general kernels on the same grid):
    values, argmax and input gradients bit-identical, odd / even H and W,
    ragged and single-run depths.  Ties are made likely (values on a coarse
    grid) so the first-maximum rule is exercised."""
    from m3d import _lib
    L = _lib.load()
    B, H, W, D, C = shape
    OH, OW = (H + 1) // 2, (W + 1) // 2
    py, px = (2 - (H - 1) % 2) // 2, (2 - (W - 1) % 2) // 2
    g = torch.Generator(device=cuda).manual_seed(4)
    x = torch.randint(-4, 5, shape, device=cuda, generator=g).float() * 0.25
    y1 = torch.empty((B, OH, OW, D, C), device=cuda)
    y2 = torch.empty_like(y1)
    a1 = torch.empty((B, OH, OW, D, C), device=cuda, dtype=torch.uint8)
    a2 = torch.empty_like(a1)
    halo = torch.zeros((B, H, W, 2, C), device=cuda)
    _lib.check(L.m3d_maxpool3d_fwd(x.data_ptr(), B, H, W, D, C, 3, 3, 3, 2, 2, 1, py, px, 1, OH, OW, D,
                                   y1.data_ptr(), a1.data_ptr(), _lib.stream()), "maxpool fwd")
    _lib.check(L.m3d_maxpool3d_fwd_halo(x.data_ptr(), halo.data_ptr(), 0, 0, 1, B, H, W, D, C, 3, 3, 3, 2, 2, 1,
                                        py, px, 1, OH, OW, D, y2.data_ptr(), a2.data_ptr(), _lib.stream()),
               "halo fwd")
    torch.cuda.synchronize()
    assert torch.equal(y1, y2) and torch.equal(a1, a2)
    dy = torch.randn((B, OH, OW, D, C), device=cuda, generator=g)
    d1 = torch.empty_like(x)
    d2 = torch.empty_like(x)
    dh = torch.zeros_like(halo)
    _lib.check(L.m3d_maxpool3d_bwd(dy.data_ptr(), a1.data_ptr(), B, H, W, D, C, 3, 3, 3, 2, 2, 1, py, px, 1, OH,
                                   OW, D, d1.data_ptr(), _lib.stream()), "maxpool bwd")
    _lib.check(L.m3d_maxpool3d_bwd_halo(dy.data_ptr(), a2.data_ptr(), 0, 0, 1, B, H, W, D, C, 3, 3, 3, 2, 2, 1,
                                        py, px, 1, OH, OW, D, d2.data_ptr(), dh.data_ptr(), _lib.stream()),
               "halo bwd")
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)


def test_sgd_keras_matches_formula(cuda):
    from m3d import _lib
    from m3d.params import ParamStore
    st = ParamStore()
    a = st.add("a/kernel:0", (3, 700), "glorot_uniform", True)
    bb = st.add("b/gamma:0", (5,), "ones", False)
    st.finalize(cuda, seed=3, weight_decay=0.01)
    w0 = st.flat.detach().clone()
    g = torch.zeros(st.total, device=cuda)      # padding of each segment stays zero
    for p in (a, bb):
        g[p.offset:p.offset + p.numel] = torch.randn(p.numel, device=cuda) * 3
    st.grad_flat.copy_(g)
    lr, mom, clip = 0.1, 0.9, 5.0
    L = _lib.load()
    _lib.check(L.m3d_sgd_keras(st.flat.data_ptr(), st.grad_flat.data_ptr(), st.moments.data_ptr(),
                               st.n_chunks, st.seg_of_chunk.data_ptr(), st.l2_coef.data_ptr(),
                               len(st.params), lr, mom, clip, st.norms.data_ptr(), _lib.stream()))
    for p, l2c in ((a, 0.01 / a.numel), (bb, 0.0)):
        sl = slice(p.offset, p.offset + p.numel)
        gt = g[sl] + l2c * w0[sl]
        gt = gt * clip / max(float(gt.norm()), clip)
        want = w0[sl] - lr * gt
        close(st.flat.detach()[sl], want, rtol=1e-6)


@pytest.mark.parametrize("nb,M,K,N,relu", [(3, 200, 64, 96, 0), (2, 130, 40, 36, 1), (64, 96, 256, 512, 0)])
def test_batched_gemm_f32(cuda, nb, M, K, N, relu):
    """m3d_gemm_f32 (the Winograd point-wise GEMM launch bench.py prices)
    against a float64 torch matmul, incl. ragged M/K/N tiles, bias, ReLU, accumulate."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(7)
    A = torch.randn((nb, M, K), generator=g)
    Bm = torch.randn((nb, K, N), generator=g)
    bias = torch.randn((N,), generator=g)
    C0 = torch.randn((nb, M, N), generator=g)
    ref = torch.bmm(A.double(), Bm.double()) + bias.double()
    if relu:
        ref = ref.clamp_min(0)
    ref = ref + C0.double()
    Ad, Bd, bd, Cd = (t.to(cuda).contiguous() for t in (A, Bm, bias, C0))
    _lib.check(L.m3d_gemm_f32(Ad.data_ptr(), Bd.data_ptr(), Cd.data_ptr(), nb, M, K, N, bd.data_ptr(),
                              relu, 1, _lib.stream()), "gemm")
    close(Cd, ref)


@pytest.mark.parametrize("D,OD,pz", [(6, 6, 1), (7, 6, 1), (7, 6, 0), (8, 6, 0), (5, 5, 1)])
def test_winograd_z_halo_geometry(cuda, D, OD, pz):
    """Winograd fwd / bwd-data / bwd-weight on a z-halo-extended depth slab
    (input depth D, output depth OD, z pad-before pz) vs float64 torch conv3d."""
    import torch.nn.functional as F
    from m3d import _lib
    L = _lib.load()
    H, W, Ci, Co = 6, 5, 128, 160
    g = torch.Generator().manual_seed(11)
    x = torch.randn((1, H, W, D, Ci), generator=g)
    w = torch.randn((3, 3, 3, Ci, Co), generator=g) * 0.05
    dy = torch.randn((1, H, W, OD, Co), generator=g)
    pz_hi = OD + 2 - pz - D
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    xc = F.pad(xr.permute(0, 4, 1, 2, 3), (pz, pz_hi, 1, 1, 1, 1))
    yr = F.conv3d(xc, wr.permute(4, 3, 0, 1, 2)).permute(0, 2, 3, 4, 1)
    (yr * dy.double()).sum().backward()
    xd, wd, dyd = x.to(cuda), w.to(cuda), dy.to(cuda)
    nb = int(L.m3d_conv3d_wino_workspace_bytes(1, H, W, D, OD, Ci, Co))
    ws = torch.empty(nb // 4 + 1, device=cuda)
    y = torch.empty((1, H, W, OD, Co), device=cuda)
    _lib.check(L.m3d_conv3d_fwd_wino(xd.data_ptr(), 1, H, W, D, Ci, wd.data_ptr(), Co, OD, pz, None, None,
                                     None, None, 0, None, y.data_ptr(), ws.data_ptr(), nb, _lib.stream()))
    dx = torch.empty((1, H, W, D, Ci), device=cuda)
    _lib.check(L.m3d_conv3d_bwd_data_wino(dyd.data_ptr(), wd.data_ptr(), 1, H, W, D, Ci, Co, OD, pz,
                                          dx.data_ptr(), 0, ws.data_ptr(), nb, _lib.stream()))
    dw = torch.zeros((3, 3, 3, Ci, Co), device=cuda)
    _lib.check(L.m3d_conv3d_bwd_weight_wino(xd.data_ptr(), dyd.data_ptr(), 1, H, W, D, Ci, Co, OD, pz,
                                            dw.data_ptr(), ws.data_ptr(), nb, _lib.stream()))
    close(y, yr)
    close(dx, xr.grad)
    close(dw, wr.grad)
    # training variants: the forward keeps U = B^T x B, the weight gradient reuses it
    # (only when the forward and weight-gradient tiles agree; u_bytes == 0 otherwise)
    ub = int(L.m3d_conv3d_wino_u_bytes(1, H, W, OD, Ci))
    u = torch.empty(max(ub, 4) // 4, device=cuda)
    y2 = torch.empty_like(y)
    keep = lambda: _lib.check(L.m3d_conv3d_fwd_wino_keep(  # noqa: E731
        xd.data_ptr(), 1, H, W, D, Ci, wd.data_ptr(), Co, OD, pz, None, None, None, None, 0, None,
        y2.data_ptr(), u.data_ptr(), ws.data_ptr(), nb, _lib.stream()))
    if ub == 0:
        with pytest.raises(ValueError):
            keep()
        return
    keep()
    dw2 = torch.zeros_like(dw)
    _lib.check(L.m3d_conv3d_bwd_weight_wino_u(u.data_ptr(), dyd.data_ptr(), 1, H, W, D, Ci, Co, OD, pz,
                                              dw2.data_ptr(), ws.data_ptr(), nb, _lib.stream()))
    assert torch.equal(y2, y)
    close(dw2, wr.grad)


@pytest.mark.parametrize("nb,M,K,N", [(3, 200, 64, 96), (2, 1000, 128, 36), (64, 512, 256, 512),
                                     (2, 1000, 320, 260), (1, 37, 192, 196), (3, 4099, 512, 256),
                                     (9, 4096, 256, 512), (5, 4000, 256, 256), (2, 1000, 64, 200),
                                     (1, 5000, 48, 136)])
def test_batched_wgrad_gemm_f32(cuda, nb, M, K, N):
    """m3d_gemm_wgrad_f32 (the Winograd weight-gradient GEMM launch bench.py
    prices): C[b] += A[b]^T B[b] against a float64 torch bmm, ragged M/K/N tiles.
    (9, 4096, ...) and (5, 4000, ...) cut tiles across stream-K workgroup ranges
    at odd steps (x3_wgrad_tr_kernel<0, true>: 18 and ~16 steps per workgroup);
    K <= 64 runs x3_wgrad64_kernel's 64x64 tiles, ragged K / N."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(11)
    A = torch.randn((nb, M, K), generator=g)
    Bm = torch.randn((nb, M, N), generator=g)
    C0 = torch.randn((nb, K, N), generator=g)
    ref = torch.bmm(A.double().transpose(1, 2), Bm.double()) + C0.double()
    Ad, Bd, Cd = (t.to(cuda).contiguous() for t in (A, Bm, C0))
    _lib.check(L.m3d_gemm_wgrad_f32(Ad.data_ptr(), Bd.data_ptr(), Cd.data_ptr(), nb, M, K, N, _lib.stream()),
               "gemm_wgrad")
    close(Cd, ref)


@pytest.mark.parametrize("nb,M,K,N", [(144, 4096, 256, 512), (40, 4096, 256, 512), (72, 2050, 256, 768),
                                     (300, 512, 256, 256)])
def test_wgrad_gemm_stream_k_shapes(cuda, nb, M, K, N):
    """x3_wgrad_tr_kernel's stream-K form (non-deterministic mode): whole tiles
    per workgroup with a plain add, the remainder tiles' step ranges added
    atomically -- 288 tiles on 256 CUs (one whole tile each + 1/8 of a
    remainder tile: the priced launch), 80 and 216 tiles (ranges only, a ragged
    last step), and 300 short tiles (the split grid with plain adds).  C += A^T
    B against float64 on the GPU, 1e-5 of the scale."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(13)
    A = torch.randn((nb, M, K), device=cuda, generator=g)
    Bm = torch.randn((nb, M, N), device=cuda, generator=g)
    C = torch.randn((nb, K, N), device=cuda, generator=g)
    ref = torch.baddbmm(C.double(), A.double().transpose(1, 2), Bm.double())
    _lib.check(L.m3d_gemm_wgrad_f32(A.data_ptr(), Bm.data_ptr(), C.data_ptr(), nb, M, K, N, _lib.stream()),
               "gemm_wgrad")
    err = float((C.double() - ref).abs().max()) / float(ref.abs().max())
    assert err < 1e-5, err


@pytest.mark.parametrize("nb,M,K,N", [(3, 300, 96, 160), (2, 300, 64, 256), (3, 1000, 256, 512),
                                     (1, 256, 128, 256), (2, 257, 512, 768), (96, 520, 256, 512),
                                     (3, 300, 64, 64), (144, 520, 64, 64)])
def test_split3_exact_and_gemm_x3(cuda, nb, M, K, N):
    """m3d_split3_f32: hi + mid + lo == x exactly (float64 sum of the bf16
    planes); m3d_gemm_x3 (the Winograd point-GEMM kernels: x3_gemm_kernel,
    its 128x64 tile for N == 64, and x3_gemm256_kernel for N % 256 == 0,
    M >= 256) against float64, ragged
    M tiles; m3d_gemm_x3_af (fp32 A) bit-identical to it."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator().manual_seed(13)
    A = torch.randn((nb, M, K), generator=g) * torch.exp(torch.randn((nb, M, K), generator=g) * 4)
    Bt = torch.randn((nb, N, K), generator=g)
    Ad, Bd = A.to(cuda), Bt.to(cuda)
    A3 = torch.empty(3 * A.numel(), dtype=torch.int16, device=cuda)
    B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device=cuda)
    _lib.check(L.m3d_split3_f32(Ad.data_ptr(), A.numel(), A3.data_ptr(), _lib.stream()), "split3")
    _lib.check(L.m3d_split3_f32(Bd.data_ptr(), Bt.numel(), B3.data_ptr(), _lib.stream()), "split3")
    planes = (A3.cpu().view(3, -1).to(torch.int32) & 0xFFFF) << 16
    parts = planes.view(torch.float32).double()
    assert torch.equal(parts.sum(0), A.reshape(-1).double())
    C = torch.empty((nb, M, N), device=cuda)
    _lib.check(L.m3d_gemm_x3(A3.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, M, K, N, _lib.stream()), "gemm_x3")
    close(C, torch.bmm(A.double(), Bt.double().transpose(1, 2)))
    # the step's form: A in fp32, split inside the GEMM (x3_gemm256_af_kernel /
    # x3_gemm_kernel<AF32>): the same split and MFMA order, bit-identical
    C2 = torch.full((nb, M, N), float("nan"), device=cuda)
    _lib.check(L.m3d_gemm_x3_af(Ad.data_ptr(), B3.data_ptr(), C2.data_ptr(), nb, M, K, N, _lib.stream()),
               "gemm_x3_af")
    assert torch.equal(C, C2)


def test_batch_items_past_operand_bound(tmp_path):
    """Every conv entry point with a batch whose tensors pass the loaders'
    32-bit operand bound runs one batch item at a time (M3D_OPERAND_LIMIT
    lowers the 4 GiB bound to 500 KB so a 3 x 262 KB batch crosses it): the
    forward and data gradients are bit-identical to the whole-batch launch,
    the weight gradients (summed per item) both within 1e-5 of the float64
    weight gradient (of its largest element; 2e-5 for the Winograd F(4x2x4)
    weight gradients), and the Winograd workspace
    shrinks to one item's."""
    import subprocess
    import sys
    worker = os.path.join(os.path.dirname(__file__), "operand_limit_worker.py")
    res = {}
    for tag, lim in (("whole", None), ("items", "500000")):
        env = dict(os.environ)
        env.pop("M3D_OPERAND_LIMIT", None)
        if lim:
            env["M3D_OPERAND_LIMIT"] = lim
        out = str(tmp_path / f"{tag}.npz")
        p = subprocess.run([sys.executable, worker, out], env=env, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        res[tag] = np.load(out)
    a, b = res["whole"], res["items"]
    assert (b["ws_bytes"] < a["ws_bytes"]).all()
    for k in a.files:
        if k == "ws_bytes" or k.startswith("ref_"):
            continue
        if k.endswith("dw"):
            # the per-item sums reassociate the fp32 tile sums: each form against
            # float64.  The Winograd weight gradients (F(4x2x4) tiles, w_ / h_) pass
            # the point GEMMs' fp32 tile sums through G^T, whose F(4,3) rows (4, 8/3)
            # amplify their rounding: measured 1.35e-5 here (C = 32, 192 tiles)
            ref = a["ref_" + k]
            scale = float(np.abs(ref).max())
            tol = 2e-5 if k[0] in "wh" else 1e-5
            for tag, got in (("whole", a[k]), ("items", b[k])):
                err = float(np.abs(got - ref).max()) / scale
                assert err <= tol, (k, tag, err)
        else:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, True)])
def test_bn_act_bwd_modes(relu, res):
    """m3d_bn_act_bwd against the float64 formulas (include/m3d.h), and its
    elementwise-only (no sums, no workspace) and sums-only (no dz / dres)
    calls equal to the fused one bit for bit."""
    from m3d import nn as mnn
    torch.manual_seed(5)
    dev = torch.device("cuda")
    M, C = 3000, 96
    dy, z = torch.randn(M, C, device=dev), torch.randn(M, C, device=dev)
    gamma, beta = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev)
    mean, var = torch.randn(C, device=dev), torch.rand(C, device=dev) + 0.5
    rstd = 1.0 / torch.sqrt(var + 1e-3)
    scale, shift = gamma * rstd, beta - mean * gamma * rstd
    y = z * scale + shift
    if relu:
        y = torch.relu(y)

    def run(with_dz, with_sums):
        dz = torch.full_like(dy, 7.0) if with_dz else None
        dres = torch.full_like(dy, 7.0) if with_dz and res else None
        sums = [torch.zeros(C, device=dev) for _ in range(3)] if with_sums else [None] * 3
        mnn.bn_act_bwd(dy, y, z, M, C, relu, scale, mean, rstd, dz, dres, *sums)
        torch.cuda.synchronize()
        return dz, dres, sums

    dz, dres, sums = run(True, True)
    g = dy.double() * ((y > 0).double() if relu else 1.0)
    xhat = (z.double() - mean.double()) * rstd.double()
    close(dz, g * scale.double())
    if res:
        close(dres, g)
    close(sums[0], g.sum(0))
    close(sums[1], (g * xhat).sum(0))
    close(sums[2], (g * scale.double()).sum(0))
    dz1, dres1, _ = run(True, False)
    _, _, sums2 = run(False, True)
    assert torch.equal(dz1, dz) and (not res or torch.equal(dres1, dres))
    assert all(torch.equal(a, b) for a, b in zip(sums2, sums))


@pytest.mark.parametrize("shape,cout,stride,res,acc", [
    ((1, 4, 4, 16, 1024), 512, (1, 1, 1), True, 0),      # res5-like: 32 rows of tiles, K = 1024
    ((1, 8, 8, 16, 512), 256, (2, 2, 1), False, 1),      # strided shortcut, accumulated dgrad
])
def test_splitk_1x1_matches_one_pass(cuda, shape, cout, stride, res, acc):
    """m3d_conv3d_fwd_splitk / _bwd_data_splitk (K-slices summed in slice order,
    then the full epilogue: bias, z, BN, residual, ReLU; strided and accumulated
    stores) against the one-pass kernels, within the f32 summation-order bound."""
    from m3d import _lib
    L = _lib.load()
    torch.manual_seed(3)
    assert L.m3d_conv3d_splitk_count(1 << 20, 1024, 512) == 1     # enough tiles: one pass
    B, H, W, D, Cin = shape
    OH, OW, OD = -(-H // stride[0]), -(-W // stride[1]), -(-D // stride[2])
    M = B * OH * OW * OD
    sp = L.m3d_conv3d_splitk_count(M, Cin, cout)
    assert sp > 1, "shape expected to take the split-K path"
    x = torch.randn(shape, device=cuda)
    w = torch.randn((1, 1, 1, Cin, cout), device=cuda) / Cin ** 0.5
    b, sc, sh = torch.randn(cout, device=cuda), torch.rand(cout, device=cuda) + 0.5, torch.randn(cout, device=cuda)
    r = torch.randn((B, OH, OW, OD, cout), device=cuda) if res else None
    outs = []
    for split in (False, True):
        y = torch.empty((B, OH, OW, OD, cout), device=cuda)
        z = torch.empty_like(y)
        p = _lib.ptr
        if split:
            ws = torch.empty(sp * M * cout, device=cuda)
            _lib.check(L.m3d_conv3d_fwd_splitk(p(x), *shape, p(w), cout, OH, OW, OD, *stride, p(b), p(sc), p(sh),
                                               p(r), 1 if res else 0, 1, p(z), p(y), sp, p(ws), ws.numel() * 4,
                                               _lib.stream()), "fwd")
        else:
            _lib.check(L.m3d_conv3d_fwd(p(x), *shape, p(w), 1, 1, 1, cout, OH, OW, OD, *stride, 0, 0, 0, p(b),
                                        p(sc), p(sh), p(r), 1 if res else 0, 1, p(z), p(y), cout, None, 0, 0,
                                        _lib.stream()), "fwd")
        outs.append((y, z))
    close(outs[1][0], outs[0][0], 1e-5)
    close(outs[1][1], outs[0][1], 1e-5)
    # data gradient: dx (+)= conv^T dz, strided scatter / accumulate
    dz = torch.randn((B, OH, OW, OD, cout), device=cuda)
    spd = L.m3d_conv3d_splitk_count(M, cout, Cin)
    dxs = []
    for split in (False, True):
        dx = torch.randn(shape, device=cuda) if acc else torch.zeros(shape, device=cuda)
        if acc:
            torch.manual_seed(9)
            dx = torch.randn(shape, device=cuda)
        p = _lib.ptr
        if split and spd > 1:
            ws = torch.empty(spd * M * Cin, device=cuda)
            _lib.check(L.m3d_conv3d_bwd_data_splitk(p(dz), p(w), B, H, W, D, Cin, cout, OH, OW, OD, *stride, p(dx),
                                                    acc, spd, p(ws), ws.numel() * 4, _lib.stream()), "bwd_data")
        else:
            _lib.check(L.m3d_conv3d_bwd_data(p(dz), p(w), B, H, W, D, Cin, 1, 1, 1, cout, OH, OW, OD, *stride,
                                             0, 0, 0, p(dx), acc, _lib.stream()), "bwd_data")
        dxs.append(dx)
    close(dxs[1], dxs[0], 1e-5)


@pytest.mark.parametrize("res_mode", [0, 1, 2])
def test_conv1_x3_matches_direct(cuda, res_mode):
    """1x1x1 stride-1 convs on the bf16-split GEMM (m3d_conv3d_fwd_x3 with the
    conv epilogue: bias, z, BN, residual same-shape / (2,2,1)-upsampled, ReLU;
    m3d_conv3d_bwd_data_x3) against the f32 direct
    kernels and a float64 evaluation."""
    from m3d import _lib
    L = _lib.load()
    p = _lib.ptr
    torch.manual_seed(11 + res_mode)
    B, H, W, D, Cin, Cout = 1, 16, 16, 64, 512, 256
    x = torch.randn((B, H, W, D, Cin), device=cuda)
    w = torch.randn((Cin, Cout), device=cuda) / Cin ** 0.5
    b, sc, sh = torch.randn(Cout, device=cuda), torch.rand(Cout, device=cuda) + 0.5, torch.randn(Cout, device=cuda)
    rshape = (B, H // 2, W // 2, D, Cout) if res_mode == 2 else (B, H, W, D, Cout)
    r = torch.randn(rshape, device=cuda) if res_mode else None
    planes = torch.empty(3 * Cin * Cout, device=cuda, dtype=torch.int16)
    _lib.check(L.m3d_conv1_x3_planes(p(w), Cin, Cout, 1, p(planes), _lib.stream()), "planes")
    y1, z1 = torch.empty((B, H, W, D, Cout), device=cuda), torch.empty((B, H, W, D, Cout), device=cuda)
    _lib.check(L.m3d_conv3d_fwd_x3(p(x), B, H, W, D, Cin, p(planes), Cout, p(b), p(sc), p(sh), p(r), res_mode, 1,
                                   p(z1), p(y1), _lib.stream()), "fwd_x3")
    y0, z0 = torch.empty_like(y1), torch.empty_like(z1)
    _lib.check(L.m3d_conv3d_fwd(p(x), B, H, W, D, Cin, p(w), 1, 1, 1, Cout, H, W, D, 1, 1, 1, 0, 0, 0, p(b), p(sc),
                                p(sh), p(r), res_mode, 1, p(z0), p(y0), Cout, None, 0, 0, _lib.stream()), "fwd")
    zr = x.double().reshape(-1, Cin) @ w.double() + b.double()
    yr = zr * sc.double() + sh.double()
    if res_mode == 1:
        yr = yr + r.double().reshape(-1, Cout)
    elif res_mode == 2:
        up = r.double().repeat_interleave(2, 1).repeat_interleave(2, 2)
        yr = yr + up.reshape(-1, Cout)
    yr = torch.relu(yr)
    close(z1.reshape(-1, Cout), zr)
    close(y1.reshape(-1, Cout), yr)
    close(y1, y0, 1e-5)
    # data gradient: N = Cin, K = Cout
    dz = torch.randn((B, H, W, D, Cout), device=cuda)
    _lib.check(L.m3d_conv1_x3_planes(p(w), Cin, Cout, 0, p(planes), _lib.stream()), "planes_t")
    d1, d0 = torch.full((B, H, W, D, Cin), 7.0, device=cuda), torch.empty((B, H, W, D, Cin), device=cuda)
    _lib.check(L.m3d_conv3d_bwd_data_x3(p(dz), p(planes), B, H, W, D, Cin, Cout, p(d1), _lib.stream()), "bwd_x3")
    _lib.check(L.m3d_conv3d_bwd_data(p(dz), p(w), B, H, W, D, Cin, 1, 1, 1, Cout, H, W, D, 1, 1, 1, 0, 0, 0,
                                     p(d0), 0, _lib.stream()), "bwd")
    close(d1.reshape(-1, Cin), dz.double().reshape(-1, Cout) @ w.double().t())
    close(d1, d0, 1e-5)


def test_wino_shared_weight_transform_bit_identical(cuda):
    """m3d_conv3d_fwd_wino_v / _bwd_data_wino_v with v_ready = 1 (the RPN
    head's shared kernel on several levels: the weight transform of the first
    call reused from the workspace) give the same bits as a fresh transform."""
    from m3d import _lib
    L = _lib.load()
    p = _lib.ptr
    torch.manual_seed(21)
    Cin, Cout = 128, 256
    w = torch.randn((3, 3, 3, Cin, Cout), device=cuda) / (27 * Cin) ** 0.5
    b = torch.randn(Cout, device=cuda)
    shapes = [(1, 8, 8, 16), (1, 4, 4, 8), (1, 2, 2, 4)]
    nbs = [L.m3d_conv3d_wino_workspace_bytes(*s, s[3], Cin, Cout) for s in shapes]
    shared = torch.empty(max(nbs) // 4 + 1, device=cuda)
    for i, s in enumerate(shapes):
        x = torch.randn((*s, Cin), device=cuda)
        dz = torch.randn((*s, Cout), device=cuda)
        outs = []
        for reuse in (False, True):
            ws = shared if reuse else torch.empty(nbs[i] // 4 + 1, device=cuda)
            nb = shared.numel() * 4 if reuse else nbs[i]
            v = 1 if (reuse and i > 0) else 0
            y = torch.empty((*s, Cout), device=cuda)
            _lib.check(L.m3d_conv3d_fwd_wino_v(p(x), *s, Cin, p(w), Cout, s[3], 1, p(b), None, None, None, 1, None,
                                               p(y), p(ws), nb, v, _lib.stream()), "fwd_v")
            outs.append(y)
        assert torch.equal(outs[0], outs[1])
    for i, s in enumerate(shapes):          # the data gradient, its own shared workspace
        dz = torch.randn((*s, Cout), device=cuda)
        outs = []
        for reuse in (False, True):
            ws = shared if reuse else torch.empty(nbs[i] // 4 + 1, device=cuda)
            nb = shared.numel() * 4 if reuse else nbs[i]
            v = 1 if (reuse and i > 0) else 0
            dx = torch.empty((*s, Cin), device=cuda)
            _lib.check(L.m3d_conv3d_bwd_data_wino_v(p(dz), p(w), *s, Cin, Cout, s[3], 1, p(dx), 0, p(ws), nb, v,
                                                    _lib.stream()), "bwd_v")
            outs.append(dx)
        assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("cin,cout", [(128, 128), (256, 512), (64, 64), (64, 128)])
def test_wino_weight_gradient_accuracy(cuda, cin, cout):
    """The Winograd weight gradient (the step's 3^3 convs with >= 64 channels;
    64 -> 64 runs x3_wgrad64_kernel, 64 -> 128 x3_wgrad_kernel,
    F(2x2x4) tiles by default, M3D_WINO_WGRAD_NZ=2 for F(2x2x2)) against
    float64: the fp32 summation over the tiles passes through G^T, whose F(4,3)
    rows amplify it -- held to 2e-5 of the gradient's scale (the direct fp32
    weight gradient's own error is ~1e-6 here), with the measured value printed."""
    from m3d import _lib
    L = _lib.load()
    g = torch.Generator(device=cuda).manual_seed(cin + cout)
    B, H, W, D = 1, 16, 16, 32
    x = torch.randn((B, H, W, D, cin), device=cuda, generator=g)
    dz = torch.randn((B, H, W, D, cout), device=cuda, generator=g)
    dw = torch.zeros((3, 3, 3, cin, cout), device=cuda)
    nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, cin, cout))
    ws = torch.empty(nb // 4 + 1, device=cuda)
    _lib.check(L.m3d_conv3d_bwd_weight_wino(x.data_ptr(), dz.data_ptr(), B, H, W, D, cin, cout, D, 1,
                                            dw.data_ptr(), ws.data_ptr(), nb, _lib.stream()))
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv3d_weight(x.double().cpu().permute(0, 4, 1, 2, 3), (cout, cin, 3, 3, 3),
                                      dz.double().cpu().permute(0, 4, 1, 2, 3), padding=1).permute(2, 3, 4, 1, 0)
    err = float((dw.double().cpu() - ref).abs().max() / ref.abs().max())
    print(f"winograd weight gradient {cin}->{cout}: rel err {err:.2e}")
    assert err <= 2e-5


def test_bn_affine_batched_matches_per_layer(cuda):
    """ParamStore.bn_affine_refresh (one m3d_bn_affine_batched launch for every
    BN layer) writes the same bits as m3d_bn_affine per layer, and a backbone
    forward with the batched affines equals one with the per-call affines."""
    from m3d import _lib
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    L = _lib.load()
    model = RPN(synthetic_rpn_config(64), device=cuda, seed=3)
    st = model.store
    g = torch.Generator().manual_seed(5)
    with torch.no_grad():
        for bn in st.bns:                   # non-trivial statistics and affine parameters
            bn.moving_mean.copy_(torch.randn(bn.c, generator=g))
            bn.moving_variance.copy_(torch.rand(bn.c, generator=g) + 0.5)
            bn.gamma.data.copy_(torch.randn(bn.c, generator=g))
            bn.beta.data.copy_(torch.randn(bn.c, generator=g))
    st.bn_affine_refresh()
    torch.cuda.synchronize()
    for bn in st.bns:
        ref = torch.empty((3, bn.c), device=cuda)
        _lib.check(L.m3d_bn_affine(bn.gamma.data.data_ptr(), bn.beta.data.data_ptr(), bn.moving_mean.data_ptr(),
                                   bn.moving_variance.data_ptr(), float(bn.eps), bn.c, ref[1].data_ptr(),
                                   ref[2].data_ptr(), ref[0].data_ptr(), _lib.stream()), "bn_affine")
        assert torch.equal(ref, bn.aff), bn.name
    image = synthetic_volume(64, seed=7).to(cuda)
    with torch.no_grad():
        a = model.backbone(image)
        refresh = st.bn_affine_refresh
        st.bn_affine_refresh = lambda: None          # per-call affines (bn_aff_live stays False)
        st.bn_aff_live = False
        try:
            import m3d.backbone as mb
            orig = mb.ResNet3D.__call__

            def per_call(self, image):
                return self._forward(image)
            mb.ResNet3D.__call__ = per_call
            b = model.backbone(image)
        finally:
            mb.ResNet3D.__call__ = orig
            st.bn_affine_refresh = refresh
    for x, y in zip(a, b):
        if x is not None:
            assert torch.equal(x, y)


def test_col_sums_batched_matches_per_unit(cuda):
    """m3d_col_sums_batched (the bias-only units' bias gradients, nn.BiasSums):
    every item's column sums are bit-identical to the per-unit m3d_bn_act_bwd
    (relu 0, no BN, sum_dz), added (+=) into out, across the shapes the model
    feeds it (one-row to 32^3-row matrices, 4 to 256 channels); float64 within
    1e-5 of scale; a shared out / bad C is rejected."""
    import ctypes

    from m3d import _lib, nn
    L = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(11)
    shapes = [(32768, 256), (4096, 256), (1, 4), (333, 32), (513, 128), (12345, 64), (7, 256)]
    xs = [torch.randn(m, c, generator=g).to(cuda) for m, c in shapes]
    base = [torch.randn(c, generator=g).to(cuda) for _, c in shapes]
    ref = [b.clone() for b in base]
    for x, r, (m, c) in zip(xs, ref, shapes):
        nn.bn_act_bwd(x, None, None, m, c, False, None, None, None, None, None, None, None, r)
    out = [b.clone() for b in base]
    n_max = _lib.COL_SUMS_MAX
    for i0 in range(0, len(shapes), n_max):                 # batches of at most M3D_COL_SUMS_MAX items
        sl = slice(i0, i0 + n_max)
        arr = (_lib.ColSumsItem * len(shapes[sl]))(*[_lib.ColSumsItem(x.data_ptr(), m, c, o.data_ptr())
                                                     for x, o, (m, c) in zip(xs[sl], out[sl], shapes[sl])])
        wsb = int(L.m3d_col_sums_batched_workspace_bytes(arr, len(arr)))
        ws = torch.empty(wsb // 4 + 1, device=cuda)
        _lib.check(L.m3d_col_sums_batched(arr, len(arr), ws.data_ptr(), wsb, _lib.stream()), "col_sums_batched")
    torch.cuda.synchronize()
    over = (_lib.ColSumsItem * (n_max + 1))(*[_lib.ColSumsItem(xs[1].data_ptr(), 4, 256, o.data_ptr())
                                             for o in [torch.empty(256, device=cuda) for _ in range(n_max + 1)]])
    with pytest.raises(ValueError):
        _lib.check(L.m3d_col_sums_batched(over, n_max + 1, ws.data_ptr(), wsb, _lib.stream()), "col_sums_batched")
    for x, o, r, b in zip(xs, out, ref, base):
        assert torch.equal(o, r)
        want = b.double() + x.double().sum(0)
        assert float((o.double() - want).abs().max()) <= 1e-5 * max(1.0, float(want.abs().max()))
    bad = (_lib.ColSumsItem * 2)(_lib.ColSumsItem(xs[0].data_ptr(), 4, 256, out[0].data_ptr()),
                                 _lib.ColSumsItem(xs[1].data_ptr(), 4, 256, out[0].data_ptr()))
    with pytest.raises(ValueError):
        _lib.check(L.m3d_col_sums_batched(bad, 2, ws.data_ptr(), wsb, _lib.stream()), "col_sums_batched")
    bad1 = (_lib.ColSumsItem * 1)(_lib.ColSumsItem(xs[0].data_ptr(), 4, 6, out[0].data_ptr()))
    with pytest.raises(ValueError):
        _lib.check(L.m3d_col_sums_batched(bad1, 1, ws.data_ptr(), wsb, _lib.stream()), "col_sums_batched")
    assert ctypes.sizeof(_lib.ColSumsItem) == 32


def test_bias_batch_model_step_matches_inline(cuda):
    """The RPN training step with the bias-only units' gradients batched
    (nn.BIAS_BATCHED, flushed in RPNHead.finish_backward) gives the same
    gradients as inline per-unit reductions (the FPN units bit for bit; the RPN
    heads' bias sums all levels at once instead of level by level)."""
    from m3d import _lib, nn
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    _lib.set_deterministic(True)              # weight gradients without arrival-order atomics
    cfg = synthetic_rpn_config(64, depth=32, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
    image = synthetic_volume(64, 32, seed=0).to(cuda)
    grads = []
    for batched in (True, False):
        model = RPN(cfg, device=cuda, seed=5)
        match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
        targets = RPNTargets(match, bbox, cuda)
        old = nn.BIAS_BATCHED
        nn.BIAS_BATCHED = batched
        try:
            model.forward_backward(image, targets, proposals=False)
        finally:
            nn.BIAS_BATCHED = old
            torch.cuda.synchronize()
        grads.append({p.name: p.grad.detach().clone() for p in model.store.params if p.grad is not None})
    _lib.set_deterministic(False)
    a, b = grads
    assert a.keys() == b.keys()
    for k in a:
        if "rpn_class_raw/bias" in k or "rpn_bbox_pred/bias" in k:
            s = float(b[k].abs().max())
            assert float((a[k] - b[k]).abs().max()) <= 1e-5 * max(s, 1e-6), k
        else:
            assert torch.equal(a[k], b[k]), k


def test_x3_planes_batched_matches_per_kernel(cuda):
    """m3d_conv1_x3_planes_batched (nn.X3Planes: one launch per model forward
    for every split-GEMM 1x1x1 kernel) writes the same bits as
    m3d_conv1_x3_planes per kernel and orientation; in a model's second
    training pass every split-GEMM 1x1x1 conv takes the refreshed planes (no
    per-conv split), and its gradients equal a pass with per-conv splits."""
    import ctypes

    from m3d import _lib, nn
    L = _lib.load()
    g = torch.Generator(device="cpu").manual_seed(3)
    shapes = [(64, 256), (2048, 512), (32, 256), (256, 1024)]
    ws = [torch.randn(ci, co, generator=g).to(cuda) for ci, co in shapes]
    fw = [torch.empty(3 * ci * co, device=cuda, dtype=torch.int16) for ci, co in shapes]
    bw = [torch.empty(3 * ci * co, device=cuda, dtype=torch.int16) for ci, co in shapes]
    items = (_lib.X3PlanesItem * len(shapes))(*[_lib.X3PlanesItem(w.data_ptr(), f.data_ptr(), b.data_ptr(), ci, co)
                                                for w, f, b, (ci, co) in zip(ws, fw, bw, shapes)])
    tab = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8).to(cuda)
    _lib.check(L.m3d_conv1_x3_planes_batched(tab.data_ptr(), len(shapes), max(a * b for a, b in shapes),
                                             _lib.stream()), "planes_batched")
    for w, f, b, (ci, co) in zip(ws, fw, bw, shapes):
        for t, got in ((1, f), (0, b)):
            ref = torch.empty_like(got)
            _lib.check(L.m3d_conv1_x3_planes(w.data_ptr(), ci, co, t, ref.data_ptr(), _lib.stream()), "planes")
            assert torch.equal(ref, got)
    with pytest.raises(ValueError):
        _lib.check(L.m3d_conv1_x3_planes_batched(tab.data_ptr(), 0, 16, _lib.stream()), "planes_batched")
    assert ctypes.sizeof(_lib.X3PlanesItem) == 32

    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    _lib.set_deterministic(True)
    try:
        cfg = synthetic_rpn_config(64, depth=32, PRE_NMS_LIMIT=2000, POST_NMS_ROIS_TRAINING=500)
        image = synthetic_volume(64, 32, seed=0).to(cuda)
        grads = []
        for batched in (True, False):
            model = RPN(cfg, device=cuda, seed=5)
            match, bbox = synthetic_rpn_targets(model.anchors.shape[1], 256, seed=2)
            targets = RPNTargets(match, bbox, cuda)
            old = nn.X3_PLANES_BATCHED, nn.CONV1_X3_FWD_TILES, nn.CONV1_X3_DGRAD_TILES
            # every eligible 1x1x1 conv and data gradient on the split GEMM at this small size
            nn.X3_PLANES_BATCHED, nn.CONV1_X3_FWD_TILES, nn.CONV1_X3_DGRAD_TILES = batched, 1, 1
            try:
                model.forward_backward(image, targets, proposals=False)        # registers the kernels
                model.forward_backward(image, targets, proposals=False)        # zero_grad + the same pass again
                if batched:
                    h0, m0 = nn.X3_PLANES.hits, nn.X3_PLANES.misses
                    model.forward_backward(image, targets, proposals=False)
                    assert nn.X3_PLANES.hits > h0 and nn.X3_PLANES.misses == m0
            finally:
                nn.X3_PLANES_BATCHED, nn.CONV1_X3_FWD_TILES, nn.CONV1_X3_DGRAD_TILES = old
                torch.cuda.synchronize()
            grads.append(model.store.grad_flat.detach().clone())
        assert torch.equal(grads[0], grads[1])
    finally:
        _lib.set_deterministic(False)
