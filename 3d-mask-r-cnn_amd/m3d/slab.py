"""Depth-slab sharding of ONE volume over the GPUs of a node.

Depth is never strided in the reference network (all strides (2,2,1):
core/models.py:242,245,212-225, FPN upsample (2,2,1) 3193, P6 3211), so the
z-slab [z0, z1) of the input maps to the same [z0, z1) on every level C1..P6
and on the RPN's (y, x, z, a)-ordered anchors.  Each rank holds one slab of
every activation.  The only data-path exchange is a z-halo: before every op
whose window spans z (the 7^3 stem, the 3^3 max-pool, every 3^3 conv) a rank
receives the r = (kd-1)/2 boundary planes of its neighbours (point-to-point
over RCCL/xGMI) and runs the op on the extended slab with the z padding only
where the volume really ends; in backward the halo planes' gradients travel
back to their owners and are added there.  The result is the single-volume
computation: identical per-voxel arithmetic (slab bounds are multiples of 4, so the
Winograd 2x2x4 tiles coincide with the unsharded ones).

Losses are partial sums over each rank's anchors divided by the global
counts; weight gradients are all-reduced with SUM; the ProposalLayer merges
per-slab top-k candidates (all-gather) into the global top-k and every rank
runs the same NMS.  The reference's only multi-GPU mode is batch-split tower
replication (core/parallel_model.py:15-90); that is m3d.parallel's data
parallel mode.
"""
from __future__ import annotations

from contextlib import contextmanager

import numpy as np
import torch
import torch.distributed as dist

_ACTIVE = None


Z_ALIGN = 4   # the Winograd output tile along z (F(2x2x4)): slab starts are multiples of it


def slab_bounds(depth, world):
    """Near-equal split of [0, depth) into `world` slabs starting at multiples
    of Z_ALIGN, so every slab's Winograd z tiles coincide with the whole
    volume's (the sharded forward is then bit-identical)."""
    units = (depth + Z_ALIGN - 1) // Z_ALIGN
    if units < world:
        raise ValueError(f"depth {depth} too small for {world} slabs")
    per, rem = divmod(units, world)
    out, z = [], 0
    for r in range(world):
        n = Z_ALIGN * (per + (1 if r < rem else 0))
        out.append((z, min(z + n, depth)))
        z += n
    return out


class SlabGroup:
    """This rank's slab [z0, z1) of a depth-D volume and its two neighbours.

    host_staging: route exchanged tensors through host memory (the gloo
    backend, used by the CPU tests and the single-GPU multi-process test);
    RCCL ("nccl") moves device buffers directly."""

    MAX_HALO = 3          # the 7^3 stem

    def __init__(self, depth, rank=None, world=None, host_staging=None):
        self.world = world if world is not None else (dist.get_world_size() if dist.is_initialized() else 1)
        self.rank = rank if rank is not None else (dist.get_rank() if dist.is_initialized() else 0)
        self.D = int(depth)
        self.bounds = slab_bounds(self.D, self.world)
        self.z0, self.z1 = self.bounds[self.rank]
        if self.world > 1 and min(b - a for a, b in self.bounds) < self.MAX_HALO:
            raise ValueError(f"depth slabs of {self.D}/{self.world} are thinner than the {self.MAX_HALO}-plane halo")
        self.lo = self.rank - 1 if self.rank > 0 else None
        self.hi = self.rank + 1 if self.rank < self.world - 1 else None
        if host_staging is None:
            host_staging = self.world > 1 and dist.is_initialized() and dist.get_backend() == "gloo"
        self.host_staging = host_staging
        # Own communicators (collective: every rank builds its SlabGroup): the
        # halo P2P of the backward never queues behind the gradient buckets the
        # overlapped all-reduce (default group) has in flight, and the proposal
        # candidates' all-gather (launched on a side stream beside the backward)
        # never sits between a halo exchange and its partner.
        self.halo_group = self.coll_group = None
        if self.world > 1 and dist.is_initialized():
            ranks = list(range(self.world))
            self.halo_group = dist.new_group(ranks)
            self.coll_group = dist.new_group(ranks)

    @property
    def Dl(self):
        return self.z1 - self.z0

    # -- communication ----------------------------------------------------
    def _out(self, t):
        t = t.contiguous()
        return t.cpu() if self.host_staging and t.is_cuda else t

    def _buf(self, shape, like):
        dev = "cpu" if self.host_staging else like.device
        return torch.empty(shape, dtype=like.dtype, device=dev)

    def exchange_start(self, to_lo, to_hi, shape):
        """Post the exchange of exchange() and return at once; the returned
        finish() waits for it (on RCCL: makes the current stream wait for the
        communicator's stream -- no host sync) and returns (from_lo, from_hi).
        Work enqueued in between overlaps the transfer."""
        like = to_lo if to_lo is not None else to_hi
        ops, recv = [], [None, None]
        if self.lo is not None:
            recv[0] = self._buf(shape, like)
            ops += [dist.P2POp(dist.isend, self._out(to_lo), self.lo, self.halo_group),
                    dist.P2POp(dist.irecv, recv[0], self.lo, self.halo_group)]
        if self.hi is not None:
            recv[1] = self._buf(shape, like)
            ops += [dist.P2POp(dist.isend, self._out(to_hi), self.hi, self.halo_group),
                    dist.P2POp(dist.irecv, recv[1], self.hi, self.halo_group)]
        works = dist.batch_isend_irecv(ops) if ops else []

        def finish():
            for req in works:
                req.wait()
            r = recv
            if self.host_staging and like.is_cuda:
                r = [None if t is None else t.to(like.device, non_blocking=False) for t in recv]
            ops.clear()                    # the send buffers lived until here
            return r[0], r[1]
        return finish

    def exchange(self, to_lo, to_hi, shape):
        """Send to_lo to the lower / to_hi to the upper neighbour; receive a
        `shape` tensor from each neighbour present.  Returns (from_lo, from_hi)."""
        return self.exchange_start(to_lo, to_hi, shape)()

    def all_gather(self, t):
        """[world, *t.shape] stack of every rank's t."""
        if self.world == 1:
            return t[None]
        src = self._out(t)
        parts = [torch.empty_like(src) for _ in range(self.world)]
        dist.all_gather(parts, src, group=self.coll_group)
        out = torch.stack(parts)
        return out.to(t.device) if out.device != t.device else out

    def all_reduce_sum_(self, t, bucket=16 * 1024 * 1024):
        if self.world == 1:
            return t
        for s in range(0, t.numel(), bucket):
            chunk = t[s:s + bucket]
            if self.host_staging and t.is_cuda:
                h = chunk.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.SUM)
                chunk.copy_(h)
            else:
                dist.all_reduce(chunk, op=dist.ReduceOp.SUM)
        return t

    # -- anchors ------------------------------------------------------------
    def local_anchor_index(self, level_hw, apl):
        """int64 [A_local]: global (y,x,z,a)-order index of each local RPN
        output row (levels concatenated as core/models.py:3250-3263)."""
        out, off = [], 0
        zs = np.arange(self.z0, self.z1, dtype=np.int64)
        a = np.arange(apl, dtype=np.int64)
        for H, W in level_hw:
            yx = np.arange(H * W, dtype=np.int64)
            g = ((yx[:, None, None] * self.D + zs[None, :, None]) * apl + a[None, None, :]).reshape(-1)
            out.append(off + g)
            off += H * W * self.D * apl
        return np.concatenate(out)


@contextmanager
def active(sg):
    """Run the enclosed forward (and its backward) sharded over `sg`."""
    global _ACTIVE
    prev = _ACTIVE
    _ACTIVE = sg if (sg is not None and sg.world > 1) else None
    try:
        yield sg
    finally:
        _ACTIVE = prev


def current():
    return _ACTIVE


class _HaloZ(torch.autograd.Function):
    """x [B,H,W,Dl,C] -> [B,H,W,Dl+nlo+nhi,C] with the neighbours' r boundary
    planes; backward returns the halo gradients to their owners."""

    @staticmethod
    def forward(ctx, x, r, sg):
        B, H, W, D, C = x.shape
        shape = (B, H, W, r, C)
        from_lo, from_hi = sg.exchange(x[:, :, :, :r] if sg.lo is not None else None,
                                       x[:, :, :, D - r:] if sg.hi is not None else None, shape)
        ctx.sg, ctx.r, ctx.D = sg, r, D
        ctx.nlo = r if from_lo is not None else 0
        parts = [p for p in (from_lo, x, from_hi) if p is not None]
        return torch.cat(parts, dim=3)

    @staticmethod
    def backward(ctx, g):
        sg, r, D, nlo = ctx.sg, ctx.r, ctx.D, ctx.nlo
        B, H, W, _, C = g.shape
        gx = g[:, :, :, nlo:nlo + D].contiguous()
        from_lo, from_hi = sg.exchange(g[:, :, :, :nlo] if sg.lo is not None else None,
                                       g[:, :, :, nlo + D:] if sg.hi is not None else None,
                                       (B, H, W, r, C))
        if from_lo is not None:
            gx[:, :, :, :r] += from_lo
        if from_hi is not None:
            gx[:, :, :, D - r:] += from_hi
        return gx, None, None


def halo_planes(x, r=1):
    """The neighbours' r boundary planes of slab x [B,H,W,Dl,C] without
    building the halo-extended slab: (halo [B,H,W,2r,C] -- planes [0, r) from
    the lower rank, [r, 2r) from the upper --, has_lo, has_hi).  The Winograd
    kernels read them beside x (m3d_conv3d_*_wino_halo); a rank at the volume's
    end has no plane there (its padding is zero)."""
    sg = _ACTIVE
    B, H, W, D, C = x.shape
    if r > D:
        raise ValueError(f"z-halo of {r} planes exceeds the slab")
    from_lo, from_hi = sg.exchange(x[:, :, :, :r] if sg.lo is not None else None,
                                   x[:, :, :, D - r:] if sg.hi is not None else None, (B, H, W, r, C))
    halo = torch.empty((B, H, W, 2 * r, C), device=x.device, dtype=x.dtype)
    if from_lo is not None:
        halo[:, :, :, :r] = from_lo
    if from_hi is not None:
        halo[:, :, :, r:] = from_hi
    return halo, int(from_lo is not None), int(from_hi is not None)


class PendingHalo:
    """halo_planes() whose exchange is in flight (halo_planes_start): has_lo /
    has_hi are known at once; result() waits and returns halo_planes()'s tuple."""

    def __init__(self, finish, has_lo, has_hi):
        self._finish, self._res = finish, None
        self.has_lo, self.has_hi = has_lo, has_hi

    def result(self):
        if self._res is None:
            self._res = self._finish()
            self._finish = None
        return self._res


def halo_planes_start(x, r=1):
    """halo_planes() split around the transfer: posts the exchange and returns
    a PendingHalo, so the caller can enqueue the work that does not read the
    halo planes (the Winograd conv's weight transform and interior z tiles,
    m3d_conv3d_fwd_wino_halo_phase) before waiting for it."""
    sg = _ACTIVE
    B, H, W, D, C = x.shape
    if r > D:
        raise ValueError(f"z-halo of {r} planes exceeds the slab")
    fin = sg.exchange_start(x[:, :, :, :r] if sg.lo is not None else None,
                            x[:, :, :, D - r:] if sg.hi is not None else None, (B, H, W, r, C))

    def finish():
        from_lo, from_hi = fin()
        halo = torch.empty((B, H, W, 2 * r, C), device=x.device, dtype=x.dtype)
        if from_lo is not None:
            halo[:, :, :, :r] = from_lo
        if from_hi is not None:
            halo[:, :, :, r:] = from_hi
        return halo, int(from_lo is not None), int(from_hi is not None)
    return PendingHalo(finish, int(sg.lo is not None), int(sg.hi is not None))


def return_halo_grads(dx, dhalo, r=1):
    """Backward of halo_planes: send the gradient of each neighbour's planes
    (dhalo [B,H,W,2r,C]) to it and add what the neighbours send for this
    rank's boundary planes into dx [B,H,W,Dl,C] in place."""
    sg = _ACTIVE
    B, H, W, D, C = dx.shape
    from_lo, from_hi = sg.exchange(dhalo[:, :, :, :r] if sg.lo is not None else None,
                                   dhalo[:, :, :, r:] if sg.hi is not None else None, (B, H, W, r, C))
    if from_lo is not None:
        dx[:, :, :, :r] += from_lo
    if from_hi is not None:
        dx[:, :, :, D - r:] += from_hi
    return dx


def halo_z(x, r):
    """(x_ext, n_lower_halo_planes) under the active slab group (identity when
    not sharded or r == 0)."""
    sg = _ACTIVE
    if sg is None or r == 0:
        return x, 0
    if r > sg.MAX_HALO or r > x.shape[3]:
        raise ValueError(f"z-halo of {r} planes exceeds the slab")
    xe = _HaloZ.apply(x, int(r), sg)
    return xe, (r if sg.lo is not None else 0)
