"""Depth-slab sharding (m3d/slab.py) on the CPU with gloo, world sizes 2 and 3.

The HIP kernels need a GPU, so the z-windowed op in these tests is a plain
torch-CPU conv3d on the halo-extended slab with the slab geometry m3d.nn
hands the kernels (z padding only where the volume ends).  What is checked is
the sharding itself: halo exchange forward/backward, the per-slab z padding,
the global anchor index map and the loss partition -- the slab results must
equal the single-volume ones."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_parallel import run


def _conv_z(x_ext, w, pz_lo, pz_hi, pad_yx):
    """channels-last x [1,H,W,D,C], w [k,k,k,Cin,Cout] -> 'same' in y/x, z padded (pz_lo, pz_hi)."""
    xc = x_ext.permute(0, 4, 1, 2, 3)                      # N C H W D
    xc = F.pad(xc, (pz_lo, pz_hi, pad_yx, pad_yx, pad_yx, pad_yx))
    y = F.conv3d(xc, w.permute(4, 3, 0, 1, 2))
    return y.permute(0, 2, 3, 4, 1)


def _halo_conv(rank, world, D=12, k=3):
    import torch.distributed as dist  # noqa: F401
    from m3d import slab
    g = torch.Generator().manual_seed(0)
    x = torch.randn((1, 5, 4, D, 3), generator=g, dtype=torch.float64)
    w = torch.randn((k, k, k, 3, 2), generator=g, dtype=torch.float64)
    gy = torch.randn((1, 5, 4, D, 2), generator=g, dtype=torch.float64)
    r = (k - 1) // 2
    # single volume
    xf = x.clone().requires_grad_(True)
    yf = _conv_z(xf, w, r, r, r)
    (yf * gy).sum().backward()
    # slab
    sg = slab.SlabGroup(D, rank, world)
    xs = x[:, :, :, sg.z0:sg.z1].clone().requires_grad_(True)
    with slab.active(sg):
        xe, nlo = slab.halo_z(xs, r)
    nhi = xe.shape[3] - sg.Dl - nlo
    ys = _conv_z(xe, w, r - nlo, r - nhi, r)
    (ys * gy[:, :, :, sg.z0:sg.z1]).sum().backward()
    ok_y = torch.allclose(ys, yf[:, :, :, sg.z0:sg.z1], rtol=0, atol=1e-12)
    ok_g = torch.allclose(xs.grad, xf.grad[:, :, :, sg.z0:sg.z1], rtol=0, atol=1e-12)
    return [ok_y, ok_g, sg.z0, sg.z1, nlo, nhi]


@pytest.mark.parametrize("world", [2, 3])
def test_halo_conv_equals_single_volume(world):
    out = run(_halo_conv, world)
    for rank, (ok_y, ok_g, z0, z1, nlo, nhi) in out.items():
        assert ok_y and ok_g, (rank, z0, z1)
        assert nlo == (1 if rank > 0 else 0) and nhi == (1 if rank < world - 1 else 0)


def _halo_planes_conv(rank, world, D=12):
    """The Winograd slab form: halo_planes() hands the kernels the neighbours'
    planes beside the slab (emulated here by a conv over [halo_lo, x, halo_hi]);
    the data gradient comes back as (interior dx, dhalo) and return_halo_grads
    routes dhalo to its owners -- equal to the single-volume conv."""
    from m3d import slab
    g = torch.Generator().manual_seed(0)
    x = torch.randn((1, 5, 4, D, 3), generator=g, dtype=torch.float64)
    w = torch.randn((3, 3, 3, 3, 2), generator=g, dtype=torch.float64)
    gy = torch.randn((1, 5, 4, D, 2), generator=g, dtype=torch.float64)
    xf = x.clone().requires_grad_(True)
    yf = _conv_z(xf, w, 1, 1, 1)
    (yf * gy).sum().backward()
    sg = slab.SlabGroup(D, rank, world)
    xs = x[:, :, :, sg.z0:sg.z1].clone()
    with slab.active(sg):
        halo, hlo, hhi = slab.halo_planes(xs, 1)
        xe = torch.cat(([halo[:, :, :, :1]] if hlo else []) + [xs] + ([halo[:, :, :, 1:]] if hhi else []), 3)
        xe.requires_grad_(True)
        ys = _conv_z(xe, w, 1 - hlo, 1 - hhi, 1)
        (ys * gy[:, :, :, sg.z0:sg.z1]).sum().backward()
        dx = xe.grad[:, :, :, hlo:hlo + sg.Dl].clone()
        dh = torch.zeros_like(halo)
        if hlo:
            dh[:, :, :, :1] = xe.grad[:, :, :, :1]
        if hhi:
            dh[:, :, :, 1:] = xe.grad[:, :, :, -1:]
        slab.return_halo_grads(dx, dh)
    ok_y = torch.allclose(ys, yf[:, :, :, sg.z0:sg.z1], rtol=0, atol=1e-12)
    ok_g = torch.allclose(dx, xf.grad[:, :, :, sg.z0:sg.z1], rtol=0, atol=1e-12)
    return [ok_y, ok_g, hlo, hhi]


@pytest.mark.parametrize("world", [2, 3])
def test_halo_planes_equal_single_volume(world):
    out = run(_halo_planes_conv, world)
    for rank, (ok_y, ok_g, hlo, hhi) in out.items():
        assert ok_y and ok_g, rank
        assert hlo == (1 if rank > 0 else 0) and hhi == (1 if rank < world - 1 else 0)


def _stem_halo(rank, world):
    return _halo_conv(rank, world, D=16, k=7)


def test_stem_sized_halo():
    for ok_y, ok_g, *_ in run(_stem_halo, 2).values():
        assert ok_y and ok_g


def _exchange_collectives(rank, world):
    from m3d import slab
    sg = slab.SlabGroup(8, rank, world)
    t = torch.full((3,), float(rank))
    gathered = sg.all_gather(t)
    s = torch.arange(5, dtype=torch.float32) * (rank + 1)
    sg.all_reduce_sum_(s, bucket=2)
    return [gathered.tolist(), s.tolist()]


def test_slab_collectives():
    out = run(_exchange_collectives, 2)
    for g, s in out.values():
        assert g == [[0.0] * 3, [1.0] * 3]
        assert s == [0.0, 3.0, 6.0, 9.0, 12.0]


def test_slab_bounds_aligned_and_covering():
    from m3d.slab import slab_bounds
    for D, n in [(256, 8), (128, 8), (10, 3), (64, 4), (7, 2)]:
        b = slab_bounds(D, n)
        assert b[0][0] == 0 and b[-1][1] == D
        assert all(b[i][1] == b[i + 1][0] for i in range(n - 1))
        assert all(z0 % 4 == 0 for z0, _ in b)
    with pytest.raises(ValueError):
        slab_bounds(6, 4)


def test_local_anchor_index_partitions_global_order():
    """The slabs' index maps partition [0, A) and follow the (y,x,z,a) order of
    the level-concatenated RPN outputs (core/models.py:3250-3263)."""
    from m3d.slab import SlabGroup
    hw, D, apl = [(4, 4), (2, 2), (1, 1)], 12, 3
    full = np.concatenate([SlabGroup(D, 0, 1).local_anchor_index(hw, apl)])
    assert np.array_equal(full, np.arange(sum(h * w for h, w in hw) * D * apl))
    parts = [SlabGroup(D, r, 3).local_anchor_index(hw, apl) for r in range(3)]
    allidx = np.sort(np.concatenate(parts))
    assert np.array_equal(allidx, full)
    # a local row (level 1, y=1, x=0, zl=1, a=2) of rank 1 (z0 = 4)
    sg = SlabGroup(D, 1, 3)
    off0 = 16 * sg.Dl * apl
    row = off0 + ((1 * 2 + 0) * sg.Dl + 1) * apl + 2
    assert parts[1][row] == 16 * D * apl + ((1 * 2 + 0) * D + 5) * apl + 2


def test_slab_losses_sum_to_single_volume_loss():
    """Per-slab focal CE / Huber partial sums over global counts add up to the
    single-volume RPN losses, and so do their logit gradients."""
    from m3d.model import RPNTargets, rpn_bbox_loss, rpn_class_loss, synthetic_rpn_targets
    from m3d.slab import SlabGroup
    hw, D, apl = [(8, 8), (4, 4), (2, 2), (1, 1), (1, 1)], 8, 3
    A = sum(h * w for h, w in hw) * D * apl
    match, bbox = synthetic_rpn_targets(A, 256, seed=4)
    g = torch.Generator().manual_seed(1)
    logits = torch.randn((1, A, 2), generator=g, dtype=torch.float64)
    deltas = torch.randn((1, A, 6), generator=g, dtype=torch.float64)
    t = RPNTargets(match, bbox, "cpu")
    t.gt_bbox = t.gt_bbox.double()
    lf, df = logits.clone().requires_grad_(True), deltas.clone().requires_grad_(True)
    ref = rpn_class_loss(t, lf) + 1.5 * rpn_bbox_loss(t, df)
    ref.backward()
    tot = 0.0
    gl, gd = torch.zeros_like(logits), torch.zeros_like(deltas)
    for r in range(2):
        gi = SlabGroup(D, r, 2).local_anchor_index(hw, apl)
        ts = RPNTargets.for_slab(match, bbox, gi, "cpu")
        ts.gt_bbox = ts.gt_bbox.double()
        ll = logits[:, gi].clone().requires_grad_(True)
        ld = deltas[:, gi].clone().requires_grad_(True)
        loss = rpn_class_loss(ts, ll) + 1.5 * rpn_bbox_loss(ts, ld)
        loss.backward()
        tot += float(loss)
        gl[:, gi] = ll.grad
        gd[:, gi] = ld.grad
    assert abs(tot - float(ref)) < 1e-12 * max(1.0, abs(float(ref)))
    torch.testing.assert_close(gl, lf.grad, rtol=0, atol=1e-15)
    torch.testing.assert_close(gd, df.grad, rtol=0, atol=1e-15)
