"""Multi-GPU data parallelism over RCCL (torch.distributed backend "nccl").

One process per GPU.  Every rank runs the full RPN step on its own volume
(weak scaling: per-GPU work is fixed as N grows) and the gradients, which
live in ONE flat buffer (params.ParamStore.grad_flat), are averaged with a
single bucketed all-reduce before the fused SGD kernel -- the reference's
equivalent is ParallelModel's in-graph tower replication
(core/parallel_model.py:15-90).  Buckets are contiguous slices of the flat
buffer, so no packing copies are needed.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

BUCKET_FLOATS = 16 * 1024 * 1024        # 64 MiB per all-reduce


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/...)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def allreduce_mean_(flat: torch.Tensor, world: int, bucket=BUCKET_FLOATS):
    """In-place average of a flat gradient buffer across ranks, in buckets."""
    if world <= 1:
        return flat
    n = flat.numel()
    for s in range(0, n, bucket):
        dist.all_reduce(flat[s:s + bucket], op=dist.ReduceOp.SUM)
    flat.mul_(1.0 / world)
    return flat


def data_parallel_train_step(model, image, targets, world, proposals=True):
    """model.train_step with the gradient average inserted before SGD."""
    model.store.zero_grad()
    out = model.forward(image, proposals=proposals)
    lc, lb = model.losses(out, targets)
    total = lc * model.LOSS_WEIGHTS["rpn_class_loss"] + lb * model.LOSS_WEIGHTS["rpn_bbox_loss"]
    total.backward()
    model.rpn.finish_backward()
    allreduce_mean_(model.store.grad_flat, world)
    model.sgd_step()
    return {"loss": total.detach(), "rpn_class_loss": lc.detach(), "rpn_bbox_loss": lb.detach(),
            "rpn_rois": out["rpn_rois"]}
