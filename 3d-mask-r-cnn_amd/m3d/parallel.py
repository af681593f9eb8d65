"""Multi-GPU data parallelism over RCCL (torch.distributed backend "nccl").

One process per GPU.  Every rank runs the full RPN step on its own volume
(weak scaling: per-GPU work is fixed as N grows) and the gradients, which
live in ONE flat buffer (params.ParamStore.grad_flat), are averaged with
bucketed all-reduces that start during the backward as soon as a bucket's
gradients are final (OverlappedAllReduce), before the fused SGD kernel -- the reference's
equivalent is ParallelModel's in-graph tower replication
(core/parallel_model.py:15-90).  Buckets are contiguous slices of the flat
buffer, so no packing copies are needed.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

BUCKET_FLOATS = 16 * 1024 * 1024        # 64 MiB per all-reduce


def init_from_env(backend=None, timeout_s=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/...).
    Collectives time out after ``timeout_s`` (M3D_DIST_TIMEOUT, default 600 s),
    so a deadlocked halo exchange or all-reduce ends the process with an error
    instead of hanging the node."""
    import datetime
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if ws <= 1:
        return 0, 1
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        to = datetime.timedelta(seconds=float(timeout_s or os.environ.get("M3D_DIST_TIMEOUT", "600")))
        if backend == "nccl":
            # bind this rank to its GPU before the communicator exists (eager
            # RCCL init on that device; barriers need not guess the device)
            local = torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
            torch.cuda.set_device(local)
            dist.init_process_group(backend=backend, device_id=local, timeout=to)
        else:
            dist.init_process_group(backend=backend, timeout=to)
    return dist.get_rank(), dist.get_world_size()


# ---------------------------------------------------------------------------
# self-validation of a multi-rank run (bench.py N > 1)
# ---------------------------------------------------------------------------
_INT_OF_WIDTH = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def tensor_digest(t: torch.Tensor) -> torch.Tensor:
    """Bit-level digest of a tensor: int64 [3] = (element count, sum of its raw
    words, sum of word * (i mod 65521 + 1)), the words being the elements' bytes
    read as an integer of the element's width (bf16 / fp16 as int16, fp64 as
    int64: no value conversion, so tensors that differ in any bit differ in
    their words) -- equal digests for bit-identical tensors; any single changed
    word changes both sums (int64 sums wrap, identically on every rank)."""
    w = t.detach().contiguous().reshape(-1)
    if w.dtype == torch.bool:
        w = w.view(torch.uint8)
    if w.is_floating_point() or w.is_complex():
        if w.is_complex():
            w = torch.view_as_real(w).reshape(-1)
        it = _INT_OF_WIDTH.get(w.element_size())
        if it is None:
            raise TypeError(f"tensor_digest: no integer type of width {w.element_size()} for {t.dtype}")
        w = w.view(it)
    w = w.to(torch.int64)
    idx = (torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521) + 1
    return torch.stack([torch.tensor(w.numel(), device=w.device, dtype=torch.int64), w.sum(), (w * idx).sum()])


def ranks_identical(tensors: dict, group=None) -> dict:
    """For each named tensor: is it bit-identical on every rank of ``group``?
    One all_gather of the digests; under gloo (which gathers host tensors only)
    the digests are moved to the host first."""
    names = sorted(tensors)
    if not names:
        return {}
    d = torch.stack([tensor_digest(tensors[n]) for n in names])
    if dist.get_backend(group) == "gloo":
        d = d.cpu()
    world = dist.get_world_size(group)
    out = [torch.empty_like(d) for _ in range(world)]
    dist.all_gather(out, d, group=group)
    return {n: bool(all(torch.equal(o[i], out[0][i]) for o in out)) for i, n in enumerate(names)}


def validate_replicas(named: dict, group=None) -> dict:
    """{"ok", "identical": {name: bool}}: the replicated state of a multi-rank
    step (weights after the all-reduce + optimizer; the merged proposals and
    the all-reduced loss of a depth-slab step) must agree bit for bit."""
    same = ranks_identical(named, group)
    return {"ok": all(same.values()), "identical": same}


def rel_close(a: float, b: float, rtol: float) -> bool:
    return abs(a - b) <= rtol * max(abs(a), abs(b), 1e-30)


def allreduce_mean_(flat: torch.Tensor, world: int, bucket=BUCKET_FLOATS):
    """In-place average of a flat gradient buffer across ranks, in buckets."""
    if world <= 1:
        return flat
    n = flat.numel()
    for s in range(0, n, bucket):
        dist.all_reduce(flat[s:s + bucket], op=dist.ReduceOp.SUM)
    flat.mul_(1.0 / world)
    return flat


class OverlappedAllReduce:
    """Bucketed SUM all-reduce of the flat gradient buffer, overlapped with the
    backward pass (the MI355X/RCCL counterpart of DDP's gradient buckets).

    Buckets are contiguous slices of ``grad_flat`` (no packing copies).  In
    forward every conv unit registers the gradient views it will write
    (``use``, via m3d.nn.GRAD_HOOK); its backward reports them final
    (``done``) right after enqueuing their kernels, and a bucket whose every
    intersecting parameter is final is all-reduced at once with
    ``async_op=True``: RCCL's stream waits for the compute stream at that
    point and then runs concurrently with the rest of the backward.  The
    backward finalises the flat buffer from its end (RPN head, FPN, stage 5,
    ...) to its start (stem), so buckets launch tail-first.  Parameters that
    no unit registers (the fused RPN class/bbox head, folded in by
    finish_backward) keep their buckets until ``finish``, which launches the
    rest, waits for all, and averages."""

    def __init__(self, store, world, bucket=BUCKET_FLOATS, average=True, group=None):
        self.store, self.world = store, world
        self.average, self.group = average, group
        flat = store.grad_flat
        self.base = flat.data_ptr()
        self.esize = flat.element_size()
        n = flat.numel()
        self.bounds = [(s, min(s + bucket, n)) for s in range(0, n, bucket)]
        self.param_of = {}
        self.param_buckets = []
        for i, p in enumerate(store.params):
            self.param_of[p.offset] = i
            b0, b1 = p.offset // bucket, (p.offset + max(p.numel, 1) - 1) // bucket
            self.param_buckets.append(list(range(b0, b1 + 1)))
        self.bucket = bucket
        self._pending0 = [0] * len(self.bounds)
        for pb in self.param_buckets:
            for b in pb:
                self._pending0[b] += 1
        self.reset()

    def reset(self):
        self.pending_params = list(self._pending0)
        self.param_left = {}                  # param index -> outstanding uses
        self.key_params = {}
        self.key_uses = {}
        self.finished = set()
        self.launched = [None] * len(self.bounds)
        self.order = []

    def _param(self, t):
        off = (t.data_ptr() - self.base) // self.esize
        return self.param_of[off]

    def use(self, key, tensors):
        if key not in self.key_params:
            self.key_params[key] = [self._param(t) for t in tensors]
        self.key_uses[key] = self.key_uses.get(key, 0) + 1

    def done(self, key):
        self.key_uses[key] -= 1
        if self.key_uses[key] > 0:
            return
        for pi in self.key_params[key]:
            if pi in self.finished:
                continue
            self.finished.add(pi)
            for b in self.param_buckets[pi]:
                self.pending_params[b] -= 1
                if self.pending_params[b] == 0:
                    self._launch(b)

    def _launch(self, b):
        if self.launched[b] is None:
            s, e = self.bounds[b]
            self.launched[b] = dist.all_reduce(self.store.grad_flat[s:e], op=dist.ReduceOp.SUM,
                                               group=self.group, async_op=True)
            self.order.append(b)

    def finish(self):
        self.n_early = len(self.order)        # buckets launched during the backward
        for b in range(len(self.bounds)):
            self._launch(b)
        for w in self.launched:
            w.wait()
        if self.average:
            self.store.grad_flat.mul_(1.0 / self.world)


def data_parallel_train_step(model, image, targets, world, proposals=True, overlap=True, force_hook=False):
    """model.train_step with the gradient average inserted before SGD; with
    ``overlap`` the buckets are all-reduced during the backward (``force_hook``:
    also for a one-rank group, to exercise the collective path)."""
    from . import nn as mnn
    model.store.zero_grad()
    hook = None
    if (world > 1 or force_hook) and overlap:
        hook = getattr(model, "_dp_hook", None)
        if hook is None or hook.world != world:
            hook = model._dp_hook = OverlappedAllReduce(model.store, world)
        hook.reset()
        mnn.GRAD_HOOK = hook
    try:
        out = model.forward(image, proposals=False)
        join = model.proposals_async(out)[1] if proposals else None   # overlaps the backward
        total, lc, lb = model.loss_total(out, targets)
        total.backward()
    finally:
        mnn.GRAD_HOOK = None
    model.rpn.finish_backward()
    if hook is not None:
        hook.finish()
    else:
        allreduce_mean_(model.store.grad_flat, world)
    model.optimizer_step()
    return {"loss": total.detach(), "rpn_class_loss": lc.detach(), "rpn_bbox_loss": lb.detach(),
            "rpn_rois": join() if join is not None else None}


# ---------------------------------------------------------------------------
# depth-slab sharding of one volume (BASELINE configs[4])
# ---------------------------------------------------------------------------
def level_hw(model):
    """(H_l, W_l) of P2..P6 for the model's IMAGE_SHAPE (strides (4,8,16,32,64) in y/x)."""
    from .anchors import compute_backbone_shapes
    shapes = compute_backbone_shapes(model.config, model.config.IMAGE_SHAPE)
    return [(int(h), int(w)) for h, w, _ in shapes]


class SlabRPN:
    """One RPN training step on a volume split into depth slabs, one per rank.

    Every rank holds the full (replicated) parameters, the slab [z0,z1) of the
    input volume and of every activation; halo planes move point-to-point
    (m3d.slab), the loss is the global one (partial sums / global counts), the
    weight gradients are SUM-all-reduced (they are partial sums of one
    gradient), SGD runs replicated, proposals are merged globally."""

    def __init__(self, model, sg, rpn_match, rpn_bbox):
        from .model import RPNTargets
        from .slab import SlabGroup  # noqa: F401
        self.model, self.sg = model, sg
        apl = model.rpn.apl
        gi = sg.local_anchor_index(level_hw(model), apl)
        self.local_index = torch.from_numpy(gi).to(model.device)
        self.targets = RPNTargets.for_slab(rpn_match, rpn_bbox, gi, model.device)

    def slice(self, volume):
        """The rank's slab of a whole [B,H,W,D,C] volume."""
        return volume[:, :, :, self.sg.z0:self.sg.z1].contiguous()

    def forward(self, image_slab, proposals=True):
        from . import slab
        m = self.model
        with slab.active(self.sg):
            fmaps = m.features(image_slab)
            logits, probs, bbox = m.rpn(fmaps)
        rois = None
        if proposals:
            rois = m.proposal_layer.call_slab([probs, bbox, m.anchors], self.sg, self.local_index)
        return {"rpn_class_logits": logits, "rpn_class": probs, "rpn_bbox": bbox, "rpn_rois": rois,
                "feature_maps": fmaps}

    def _proposals_async(self, out):
        """The slab ProposalLayer (local top-k, candidate all-gather on the
        group's own communicator, decode, 3-D NMS) launched right after the
        forward on a side HIP stream, as RPN.proposals_async does for one
        volume: it overlaps the backward.  Returns join() -> rpn_rois on the
        current stream.  Host-staged (gloo) groups run it in line."""
        m = self.model
        probs, bbox = out["rpn_class"].detach(), out["rpn_bbox"].detach()
        args = ([probs, bbox, m.anchors], self.sg, self.local_index)
        if not probs.is_cuda or self.sg.host_staging:
            rois = m.proposal_layer.call_slab(*args)
            return lambda: rois
        main = torch.cuda.current_stream(probs.device)
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(probs.device)
        side = self._side
        side.wait_stream(main)
        with torch.cuda.stream(side):
            rois = m.proposal_layer.call_slab(*args)
        probs.record_stream(side)
        bbox.record_stream(side)

        def join():
            main.wait_stream(side)
            rois.record_stream(main)
            return rois
        return join

    def train_step(self, image_slab, proposals=True, apply=True, overlap=True, force_hook=False):
        """One sharded step.  The weight gradients (partial sums of one
        gradient) are SUM-all-reduced in buckets DURING the backward
        (OverlappedAllReduce, as the data-parallel path) -- the halo exchanges
        and the bucket all-reduces then share the backward.  apply=False stops
        before the optimizer (tests compare the reduced gradient); force_hook:
        the overlapped all-reduce also for a one-rank group (exercises the
        collective path on one GPU)."""
        from . import nn as mnn
        from . import slab
        m = self.model
        m.store.zero_grad()
        hook = None
        if (self.sg.world > 1 or force_hook) and overlap:
            hook = getattr(self, "_hook", None)
            if hook is None:
                hook = self._hook = OverlappedAllReduce(m.store, self.sg.world, average=False)
            hook.reset()
            mnn.GRAD_HOOK = hook
        try:
            out = self.forward(image_slab, proposals=False)
            join = self._proposals_async(out) if proposals else None     # overlaps the backward
            total, lc, lb = m.loss_total(out, self.targets)
            with slab.active(self.sg):          # halo gradients flow during backward
                total.backward()
        finally:
            mnn.GRAD_HOOK = None
        m.rpn.finish_backward()
        if hook is not None:
            hook.finish()
        else:
            self.sg.all_reduce_sum_(m.store.grad_flat)
        if join is not None:
            out["rpn_rois"] = join()
        if apply:
            m.optimizer_step()
        parts = torch.stack([total.detach(), lc.detach(), lb.detach()])
        self.sg.all_reduce_sum_(parts)
        return {"loss": parts[0], "rpn_class_loss": parts[1], "rpn_bbox_loss": parts[2],
                "rpn_rois": out["rpn_rois"], "outputs": out}
