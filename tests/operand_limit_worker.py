"""Worker of tests/test_gpu_conv.py::test_batch_items_past_operand_bound: runs the
conv entry points (direct fwd with BN / residual / upsampled residual, direct
bwd-data / bwd-weight, Winograd fwd / bwd-data / bwd-weight and their
depth-slab halo forms) on a batch of 3 and saves the outputs to OUT.npz.  Run
once with M3D_OPERAND_LIMIT below the batch's tensor sizes (every entry point
then runs one batch item at a time) and once without."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    out = sys.argv[1]
    from m3d import _lib
    L = _lib.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    B, H, W, D, C = 3, 16, 16, 8, 32

    def rnd(*shape, s=1.0):
        return (torch.randn(shape, generator=g) * s).to(dev)

    x = rnd(B, H, W, D, C)
    w3 = rnd(3, 3, 3, C, C, s=0.05)
    w1 = rnd(1, 1, 1, C, C, s=0.1)
    bias, scale, shift = rnd(C, s=0.1), rnd(C, s=0.2) + 1.0, rnd(C, s=0.1)
    res = rnd(B, H, W, D, C)
    res_up = rnd(B, H // 2, W // 2, D, C)
    dz = rnd(B, H, W, D, C)
    dz_s = rnd(B, H // 2, W // 2, D, C)
    s = _lib.stream()
    r = {}

    def fwd(name, wt, k, stride, pad, OH, OW, resid, mode):
        y = torch.empty((B, OH, OW, D, C), device=dev)
        z = torch.empty_like(y)
        _lib.check(L.m3d_conv3d_fwd(x.data_ptr(), B, H, W, D, C, wt.data_ptr(), k, k, k, C, OH, OW, D,
                                    *stride, pad, pad, pad, bias.data_ptr(), scale.data_ptr(), shift.data_ptr(),
                                    _lib.ptr(resid), mode, 1, z.data_ptr(), y.data_ptr(), C, None, 0, 0, s), name)
        r[name + "_y"], r[name + "_z"] = y, z

    fwd("d3", w3, 3, (1, 1, 1), 1, H, W, res, 1)
    fwd("d3up", w3, 3, (1, 1, 1), 1, H, W, res_up, 2)
    fwd("d1s", w1, 1, (2, 2, 1), 0, H // 2, W // 2, None, 0)
    dx = torch.empty_like(x)
    _lib.check(L.m3d_conv3d_bwd_data(dz.data_ptr(), w3.data_ptr(), B, H, W, D, C, 3, 3, 3, C, H, W, D, 1, 1, 1,
                                     1, 1, 1, dx.data_ptr(), 0, s), "bwd_data 3")
    dxs = torch.zeros_like(x)
    _lib.check(L.m3d_conv3d_bwd_data(dz_s.data_ptr(), w1.data_ptr(), B, H, W, D, C, 1, 1, 1, C, H // 2, W // 2, D,
                                     2, 2, 1, 0, 0, 0, dxs.data_ptr(), 1, s), "bwd_data 1 strided")
    dw = torch.zeros_like(w3)
    _lib.check(L.m3d_conv3d_bwd_weight(x.data_ptr(), dz.data_ptr(), B, H, W, D, C, 3, 3, 3, C, H, W, D, 1, 1, 1,
                                       1, 1, 1, dw.data_ptr(), s), "bwd_weight 3")
    r.update(d3_dx=dx, d1s_dx=dxs, d3_dw=dw)
    # Winograd, whole volume
    nb = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, C, C))
    ws = torch.empty(nb // 4 + 1, device=dev)
    y = torch.empty_like(x)
    _lib.check(L.m3d_conv3d_fwd_wino(x.data_ptr(), B, H, W, D, C, w3.data_ptr(), C, D, 1, bias.data_ptr(),
                                     scale.data_ptr(), shift.data_ptr(), res.data_ptr(), 1, None, y.data_ptr(),
                                     ws.data_ptr(), nb, s), "wino fwd")
    wdx = torch.empty_like(x)
    _lib.check(L.m3d_conv3d_bwd_data_wino(dz.data_ptr(), w3.data_ptr(), B, H, W, D, C, C, D, 1, wdx.data_ptr(), 0,
                                          ws.data_ptr(), nb, s), "wino bwd_data")
    wdw = torch.zeros_like(w3)
    _lib.check(L.m3d_conv3d_bwd_weight_wino(x.data_ptr(), dz.data_ptr(), B, H, W, D, C, C, D, 1, wdw.data_ptr(),
                                            ws.data_ptr(), nb, s), "wino bwd_weight")
    r.update(w_y=y, w_dx=wdx, w_dw=wdw)
    # Winograd depth-slab forms: both neighbours present
    halo = rnd(B, H, W, 2, C)
    nbh = int(L.m3d_conv3d_wino_workspace_bytes(B, H, W, D + 2, D, C, C))
    wsh = torch.empty(nbh // 4 + 1, device=dev)
    hy = torch.empty_like(x)
    _lib.check(L.m3d_conv3d_fwd_wino_halo(x.data_ptr(), halo.data_ptr(), 1, 1, B, H, W, D, C, w3.data_ptr(), C,
                                          bias.data_ptr(), None, None, None, 1, None, hy.data_ptr(), None,
                                          wsh.data_ptr(), nbh, s), "wino fwd halo")
    hdx, hdh = torch.empty_like(x), torch.empty_like(halo)
    _lib.check(L.m3d_conv3d_bwd_data_wino_halo(dz.data_ptr(), w3.data_ptr(), 1, 1, B, H, W, D, C, C, hdx.data_ptr(),
                                               hdh.data_ptr(), 0, wsh.data_ptr(), nbh, s), "wino bwd_data halo")
    hdw = torch.zeros_like(w3)
    _lib.check(L.m3d_conv3d_bwd_weight_wino_halo(x.data_ptr(), halo.data_ptr(), 1, 1, dz.data_ptr(), B, H, W, D, C,
                                                 C, hdw.data_ptr(), wsh.data_ptr(), nbh, s), "wino bwd_weight halo")
    r.update(h_y=hy, h_dx=hdx, h_dhalo=hdh, h_dw=hdw)
    torch.cuda.synchronize()
    # float64 weight gradients (the anchor of the dw comparisons)
    def wgrad64(xin, dzz, pad):
        xi = xin.cpu().double().permute(0, 4, 1, 2, 3)
        gi = dzz.cpu().double().permute(0, 4, 1, 2, 3)
        gw = torch.nn.grad.conv3d_weight(xi, (C, C, 3, 3, 3), gi, padding=pad)
        return gw.permute(2, 3, 4, 1, 0).contiguous()
    r["ref_d3_dw"] = wgrad64(x, dz, 1)
    r["ref_w_dw"] = r["ref_d3_dw"]
    x_ext = torch.cat([halo[:, :, :, 0:1], x, halo[:, :, :, 1:2]], dim=3)
    r["ref_h_dw"] = wgrad64(x_ext, dz, (1, 1, 0))
    np.savez(out, ws_bytes=np.array([nb, nbh]), **{k: v.cpu().numpy() for k, v in r.items()})


if __name__ == "__main__":
    main()
