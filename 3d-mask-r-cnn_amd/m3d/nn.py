"""Autograd functions of the backbone / FPN / RPN graph over libm3d.so.

Parameters live in a flat ``ParamStore`` (see params.py); every function here
accumulates its weight / bias / BN gradients straight into the parameter's
gradient view with the kernels' atomics, so autograd only carries activation
gradients.  Layout is channels-last [B,H,W,D,C] throughout, as the reference.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import weakref
from dataclasses import dataclass

import torch

from . import _lib, slab
from ._lib import check, ptr, stream


# Per-layer work records for the roofline accounting of bench.py: when set to
# a list, every conv / pool / subsample forward appends
# (kind, direct_flops, executed_flops, compulsory_bytes).  executed_flops is
# the MFMA work of the algorithm actually run (the 64 batched GEMMs for a
# Winograd layer); compulsory bytes = input + weights + residual + output.
LAYER_LOG = None
# with LAYER_LOG: also bracket every logged launch group with HIP events
# (bench.py step_roofline: measured time per layer beside its roofline time)
LAYER_TIMING = False


# ReLU branch record for parity tests: when set to a dict, every conv unit
# with a ReLU appends its output's sign mask (y > 0, on the host) under its
# Keras layer name, in call order.  The float64 restatement can then take the
# branches the GPU forward took (oracle/model_ref.RefRPN relu_masks): a
# pre-activation within fp32 rounding of 0 otherwise flips the branch and moves
# every gradient upstream of it.
RELU_CAPTURE = None


# Gradient-ready hook of the data-parallel path (m3d.parallel.OverlappedAllReduce):
# when set, every conv unit registers its gradient tensors in forward
# (use(key, tensors)) and reports them final once its backward has enqueued
# the weight/BN gradient kernels (done(key)), so finished buckets of the flat
# gradient buffer are all-reduced while the rest of the backward runs.
GRAD_HOOK = None


# Weight gradients run on a side HIP stream, concurrently with the data-
# gradient chain of the backward (the next layer's backward needs dx, never
# dW): the many small, under-filled launches of the deep stages then overlap.
# The side stream waits for the compute stream before each weight gradient
# (dz ready), and join_wgrad() -- called by RPNHead.finish_backward, i.e.
# before anything reads the gradients -- makes the compute stream wait for it.
# False runs them in line (bench.py --wgrad-inline: serialized kernel traces).
WGRAD_STREAM = True
# Enqueue order inside a conv unit's backward: True launches the weight
# gradient (side stream) after the data gradient (compute stream), False before
# it.  The GPU work and its dependencies are the same either way (eager 128^3
# step 26.23 vs 26.25 ms), but a HIP-graph replay puts a node's first-captured
# successor on the node's own queue: with the weight gradient first, the
# compute path hopped onto the weight-gradient queue behind its backlog and the
# replay ran 28.7 ms; data gradient first, 26.04 ms (scripts/archive/gpu_r05_graph3.sh).
WGRAD_LAST = True
_SIDE = {}
_SIDE_USED = set()


# Host throttle of the side stream under memory pressure: the tensors a
# weight gradient reads (x, dz) are record_stream'ed to the side stream, so
# the caching allocator can reuse their blocks only once the host sees the side
# stream's events complete -- with the host enqueueing the whole backward far
# ahead of the GPU (a 256^3 step is ~200 ms of GPU work) none are, every later
# allocation takes new device memory, and reservations reach the device's
# capacity (263-306 GB reserved for 115-141 GB allocated at 256^3) where the
# allocator frees and re-allocates segments inside the step.  When more than
# this fraction of the device is reserved, the host waits for the side stream
# every WGRAD_THROTTLE_EVERY weight gradients (0: off).
WGRAD_THROTTLE = 0.5
WGRAD_THROTTLE_EVERY = 4
_THROTTLE = {}


def _throttle(key, side):
    if WGRAD_THROTTLE <= 0:
        return
    if torch.cuda.is_current_stream_capturing():
        # a host wait on a stream under graph capture is illegal (it would
        # invalidate the capture); a replayed graph allocates nothing anyway
        return
    st = _THROTTLE.setdefault(key, {"total": torch.cuda.get_device_properties(key).total_memory, "n": 0})
    st["n"] += 1
    if st["n"] % max(1, WGRAD_THROTTLE_EVERY) == 0 and \
            torch.cuda.memory_reserved(key) > WGRAD_THROTTLE * st["total"]:
        side.synchronize()


# Fork / join events of the weight-gradient stream (m3d_stream_fork): "2" no
# system-scope fence (default; both streams are on one device, agent scope is
# all the consumer needs: on gfx950 an agent-scope release writes back every
# XCD's L2 to the device-coherent level, and each kernel's completion signal
# carries its own agent-scope release, so the consumer's acquire sees the
# producer's stores -- the system-scope part only adds visibility to the host
# and peer devices, which no consumer of these events needs), "1" device-scope
# release, "0" plain event, "torch":
# Stream.wait_stream.  The fork showed as a ~7.5 us compute-queue bubble per
# layer in the 128^3 kernel trace; A/B (scripts/archive/gpu_r03x.sh, same box): mode 2
# 29.80 / 29.90 ms per step, torch / 0 / 1 30.05-30.10 ms.
FORK_EVENT = "2"


_EV_RING = 64
_FORK_EVENTS = {}       # (device, mode) -> [events, next]: the caller-owned events of m3d_stream_fork


def fork_event(dev_index, mode):
    """Next event of the (device, mode) ring (m3d_fork_event_create): an event
    is recorded again only after 63 later forks were enqueued, long after the
    wait that used it."""
    key = (dev_index, mode)
    ring = _FORK_EVENTS.get(key)
    if ring is None:
        L = _lib.load()
        evs = []
        with torch.cuda.device(dev_index):
            for _ in range(_EV_RING):
                ev = ctypes.c_void_p()
                check(L.m3d_fork_event_create(mode, ctypes.byref(ev)), "fork_event_create")
                evs.append(ev.value)
        ring = _FORK_EVENTS[key] = [evs, 0]
    ev = ring[0][ring[1]]
    ring[1] = (ring[1] + 1) % _EV_RING
    return ev


def _fork(src, dst):
    """dst waits for the work enqueued on src so far."""
    if FORK_EVENT == "torch":
        dst.wait_stream(src)
        return
    ev = fork_event(src.device.index if src.device.index is not None else torch.cuda.current_device(),
                    int(FORK_EVENT))
    check(_lib.load().m3d_stream_fork(src.cuda_stream, dst.cuda_stream, ev), "stream_fork")


def _wgrad_stream(dev):
    if not WGRAD_STREAM:
        return None
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(dev)
    _SIDE_USED.add(key)
    side = _SIDE[key]
    _throttle(key, side)
    _fork(torch.cuda.current_stream(dev), side)
    return side


def join_wgrad(dev=None):
    """Make the current stream wait for the weight gradients launched on the side stream."""
    for key in list(_SIDE_USED):
        if dev is None or key == (dev.index if dev.index is not None else torch.cuda.current_device()):
            _fork(_SIDE[key], torch.cuda.current_stream(torch.device("cuda", key)))
            _SIDE_USED.discard(key)


def _grad_done(grads, side=None):
    h = grads.get("_hook") if grads else None
    if h is not None:
        if side is not None:
            # the bucket all-reduce must follow this layer's weight gradients
            # (side) and its BN/bias gradients (compute stream)
            _fork(torch.cuda.current_stream(), side)
            with torch.cuda.stream(side):
                h[0].done(h[1])
        else:
            h[0].done(h[1])


def _span():
    """Start event of a logged launch group (LAYER_TIMING): recorded on the
    current stream before the group's first launch; None when not timing."""
    if LAYER_LOG is None or not LAYER_TIMING:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _log(kind, direct_flops, exec_flops, nbytes, phase="fwd", name="", t0=None, engine="f32"):
    """Append (kind, direct_flops, executed_flops, compulsory_bytes, phase, name,
    start_event, end_event, engine) to LAYER_LOG; the end event is recorded on
    the current stream right after the group's launches (both None when not
    timing).  engine: the MFMA form the group's GEMM ran on -- "x3" (fp32 as six
    bf16 MFMAs on the exact split: ceiling bf16 peak / 6) or "f32"
    (v_mfma_f32_32x32x2_f32) -- so the step roofline prices it at the ceiling of
    the kernel that ran it."""
    if LAYER_LOG is not None:
        t1 = None
        if t0 is not None:
            t1 = torch.cuda.Event(enable_timing=True)
            t1.record()
        LAYER_LOG.append((kind, float(direct_flops), float(exec_flops), float(nbytes), phase, name, t0, t1,
                          engine))


# (2,2,1)-strided 1x1x1 convs' weight gradients (the stage-first blocks' 2a and
# shortcut) as subsample + the stride-1 split-GEMM gradient instead of the f32
# implicit-GEMM gradient (round 6; same box: 256^3 146.35 -> 145.93 ms, 128^3
# 23.89 vs 23.94 ms, profiles/r06_wgrad1_strided_ab.txt)
WGRAD1_STRIDED_X3 = True


def _wgrad1_x3(geo, cin, cout, in_sp):
    """Does m3d_conv3d_bwd_weight run this conv's weight gradient on the x3
    GEMM?  (1x1x1 stride-1 convs with Cin % 4 == 0 and Cout >= 65:
    csrc/conv3d.hip, m3d_conv3d_bwd_weight.)"""
    return (geo.k == (1, 1, 1) and geo.stride == (1, 1, 1) and geo.pad == (0, 0, 0)
            and tuple(geo.out) == tuple(in_sp) and cin % 4 == 0 and cout >= 65)


def _wino_exec(B, OH, OW, OD, cin, cout, nz, ny=None):
    """MFMA FLOPs of the Winograd point GEMMs, F(ny x 2 x nz): (ny+2)*4*(nz+2)
    points (ny: the forward's y tile unless given)."""
    if ny is None:
        ny = int(_L().m3d_conv3d_wino_tile_y())
    tiles = B * -(-OH // ny) * -(-OW // 2) * -(-OD // nz)
    return 2.0 * (ny + 2) * 4 * (nz + 2) * tiles * cin * cout


def _L():
    return _lib.load()


# depth-slab sharding: the Winograd convs read the neighbours' halo planes beside
# the slab (m3d_conv3d_*_wino_halo); M3D_SLAB_HALO_PLANES=0 builds the
# halo-extended copy of every z-window input instead (torch.cat, the old path)
SLAB_HALO_PLANES = True

# ... and post the exchange before the Winograd conv's first launch phase
# (m3d_conv3d_fwd_wino_halo_phase 1: weights + interior z tiles), waiting only
# before phase 2 (False: exchange, then the one-launch conv)
SLAB_OVERLAP = True

# big-K 1x1x1 stride-1 convs on the bf16-split GEMM (False: the f32 direct kernel)
CONV1_X3 = True
# split-K 1x1x1 convs where the output tiles do not fill the chip (False: one pass)
SPLITK = True
# largest transformed input U a Winograd conv keeps from its forward for its
# weight gradient (per layer; at 256^3 the P2 layers' U is 6.4 GB each).  With
# the side-stream throttle below holding the allocator's reservations down,
# keeping them is 4 ms faster per 256^3 step (177.6 vs 181.8 ms, 141 vs 133 GB
# peak, r03r); above the cap the weight gradient re-transforms x
WINO_KEEP_MAX_BYTES = 8 * 2**30
# largest Winograd workspace a shared kernel keeps across its calls
SHARE_WINO_MAX_BYTES = 6 * 2**30

# Winograd F(4x2x4, 3^3) for stride-1 'same' 3x3x3 convs (False disables)
WINOGRAD = True
WINO_MIN_C = 64
# below this channel count the weight gradient runs as a direct implicit GEMM.
# Round 2 kept the 64-channel res2*_branch2b on the direct kernel (its own
# F(2x2x2) input transform cost more than it saved: 0.35 vs 0.33 ms); with the
# weight gradient on the forward's kept F(2x2x4) U there is no input transform
# left to pay, and 64 is faster: step 29.8 -> 29.5 ms (same-box A/B, r03n)
WINO_WGRAD_MIN_C = 64


# Layers whose Winograd data gradient runs on F(4x2x4) tiles instead of the
# library's F(2x2x4) ('+'-separated layer names, "*" = all; round 5 moved every
# data gradient to F(2x2x4) for gradient accuracy).  Round 6: the
# three 64-channel res2 branch2b convs, the last data gradients of the backward
# chain (their rounding reaches only res2a / the stem): 256^3 step 151.6 ->
# 150.2 ms, configs[1] gradient median 2.05e-6 unchanged (profiles/r06_res2_dgrad_y4.txt)
WINO_DGRAD_Y4 = "res2a_branch2b+res2b_branch2b+res2c_branch2b"


def _dgrad_tile_y(name):
    if not WINO_DGRAD_Y4:
        return 0
    return 4 if WINO_DGRAD_Y4 == "*" or name in WINO_DGRAD_Y4.split("+") else 0


def use_winograd(geo, cin, cout, in_sp):
    """'same' 3x3x3 stride-1 convs, or their z-halo-extended depth-slab form
    (z pad 0/1, input depth = output depth + halo planes)."""
    # below 64 channels the (bandwidth-bound) transforms cost more than the
    # 4.5x MFMA saving of F(2x2x4)
    return (WINOGRAD and geo.k == (3, 3, 3) and geo.stride == (1, 1, 1) and geo.pad[:2] == (1, 1)
            and tuple(geo.out[:2]) == tuple(in_sp[:2]) and geo.pad[2] in (0, 1)
            and 0 <= in_sp[2] - geo.out[2] <= 2
            and cin % 32 == 0 and cout % 32 == 0 and min(cin, cout) >= WINO_MIN_C)


def _splitk(xshape, geo, cin, cout, bwd_data):
    """K-slices of the split-K form of a 1x1x1 conv (m3d_conv3d_splitk_count; 1: one pass).
    Under depth-slab sharding the count is the whole volume's (depth is never
    strided), so every slab sums its K slices exactly as the unsharded run."""
    if geo.k != (1, 1, 1) or geo.pad != (0, 0, 0) or not SPLITK:
        return 1
    B, (OH, OW, OD) = xshape[0], geo.out
    sg = slab.current()
    if sg is not None:
        OD = sg.D
    K, N = (cout, cin) if bwd_data else (cin, cout)
    return int(_L().m3d_conv3d_splitk_count(B * OH * OW * OD, K, N))


# Fewest 256x256 output tiles for which a 1x1x1 conv runs as one bf16-split
# GEMM (m3d_conv3d_fwd_x3 / _bwd_data_x3) instead of the implicit GEMM or its
# split-K form, per direction.  Round 5 (scripts/conv1_paths.py,
# profiles/r05_conv1_paths.txt): at >= 128 tiles the split GEMM's forward wins
# at every K (64 -> 256 at 256^3: 0.56 vs 0.82 ms; 128 -> 512: 0.36 vs 0.55;
# 2048 -> 512 at 8x8x256: 0.27 vs 0.34), at 64 tiles it loses to split-K
# (2048 -> 256 at 8x8x256: 0.24 vs 0.17 ms).  Both forms give the same bits
# as the implicit GEMM on the split (no split-K).  The data gradient alone is
# faster from 256 tiles at short K too (256 -> 64: 0.37 vs 0.49 ms), but
# inside the 256^3 step (fused BN-ReLU backward epilogues) it is not: slab step
# 159.1 / 159.7 ms with the round-4 rule (K >= 256) for the data gradient vs
# 160.2 / 167.8 with K >= 32 (scripts/archive/gpu_r05_slab_ab.sh), so that rule stays.
CONV1_X3_FWD_TILES = 128
CONV1_X3_DGRAD_TILES = 256
CONV1_X3_MIN_K = 32             # forward; round 4: 256 (and 256 tiles)
CONV1_X3_DGRAD_MIN_K = 256
# the data gradient with the producer's BN-ReLU backward fused into the split
# GEMM (m3d_conv3d_bwd_data_x3_bna): its own K floor, and whether it also takes
# the accumulating (identity blocks' 2a) gradients.  Round 6 A/B of K >= 32 with
# accumulate against the round-5 rule (K >= 256, no accumulate), same box
# (scripts/r06/gpu_bna.sh, profiles/r06_x3_bna_ab.txt): 128^3 24.58 vs 24.50 ms,
# 256^3 148.4 vs 148.9 ms -- neutral, so the round-5 rule stays.
CONV1_X3_DGRAD_FUSED_MIN_K = 256
X3_BN_FUSE_ACC = False


def _conv1_x3(xshape, geo, K, N, bwd_data=False, fused=False):
    """Run a 1x1x1 stride-1 conv (forward: K = Cin, N = Cout; data gradient:
    K = Cout, N = Cin) as one GEMM on the exact bf16 split (m3d_conv3d_fwd_x3 /
    _bwd_data_x3)?  When N is a multiple of 256 and its 256x256 tiles number
    at least CONV1_X3_FWD_TILES / CONV1_X3_DGRAD_TILES.  The choice uses the
    whole volume's depth under depth-slab sharding, so every slab runs the same
    kernel as the unsharded volume."""
    if not CONV1_X3 or geo.k != (1, 1, 1) or geo.stride != (1, 1, 1) or geo.pad != (0, 0, 0):
        return False
    B, H, W, D = xshape[:4]
    kmin = (CONV1_X3_DGRAD_FUSED_MIN_K if fused else CONV1_X3_DGRAD_MIN_K) if bwd_data else CONV1_X3_MIN_K
    if tuple(geo.out) != (H, W, D) or K % 32 or N % 256 or K < kmin:
        return False
    sg = slab.current()
    Dg = sg.D if sg is not None else D
    return -(-B * H * W * Dg // 256) * (N // 256) >= (CONV1_X3_DGRAD_TILES if bwd_data else CONV1_X3_FWD_TILES)


def _check_generations(ctx):
    """Ordering contract of the batched per-forward buffers (ParamStore's BN
    affine, X3Planes): a conv unit's backward reads the affine / split planes
    its forward used, which live in buffers the NEXT model forward refreshes in
    place.  A backward that runs after another forward (retain_graph double
    backward, accumulation across an update) would silently use the newer
    values, so it raises instead."""
    g = ctx.aff_gen
    if g is not None and g[0].bn_gen != g[1]:
        raise RuntimeError("conv backward after another model forward: the batched BN affine this unit's "
                           "forward used was refreshed (run each backward before the next forward)")
    if ctx.x3_gen is not None and X3_PLANES.gen != ctx.x3_gen:
        raise RuntimeError("conv backward after another model forward: the split planes this unit's "
                           "forward used were refreshed (run each backward before the next forward)")


class X3Planes:
    """The bf16-split planes of the 1x1x1 kernels that run on the split GEMM
    (m3d_conv1_x3_planes), refreshed for all of them by ONE launch per model
    forward (m3d_conv1_x3_planes_batched: both orientations, the data
    gradient's too) instead of one launch per conv and per data gradient.

    A kernel is registered the first time a conv asks for its planes (that call
    splits it alone); each RPN.forward refreshes the registered kernels first
    (``refresh``) and its convs take the cached planes while ``live``, i.e.
    during that forward only (``invalidate`` at its end): a conv unit's forward
    hands the data-gradient planes to its backward through ctx, so no cached
    plane outlives the weights it was split from (optimizer steps, weight
    loads and in-place edits all happen outside a forward).  Entries are keyed
    by the kernel tensor's storage pointer and element count and hold a weak
    reference to it (the model's persistent kernel view, kept by the
    ParamStore: while it lives no other tensor can have its storage; a dead
    entry is dropped at the next refresh)."""

    def __init__(self):
        self.entries = {}            # (ptr, numel) -> [weakref(w), cin, cout, fwd, bwd, valid]
        self.tables = {}             # device -> (device item table, n, max_el, key)
        self.live = False
        self.gen = 0                 # refreshes that rewrote the planes (_check_generations)
        self.hits = self.misses = 0  # refreshed planes taken / per-conv splits while live (tests)

    @staticmethod
    def _dev(dev):
        dev = torch.device(dev)
        return torch.device("cuda", torch.cuda.current_device() if dev.index is None else dev.index)

    def _alive(self, dev):
        for k in [k for k, e in self.entries.items() if e[0]() is None]:
            del self.entries[k]
        return [e for e in self.entries.values() if e[0]().device == dev]

    def refresh(self, dev):
        """Split every registered kernel on ``dev`` (current stream) and go live."""
        dev = self._dev(dev)
        capturing = torch.cuda.is_current_stream_capturing()
        es = self._alive(dev)
        if es:
            key = tuple((ptr(e[0]()), ptr(e[3]), ptr(e[4])) for e in es)
            t = self.tables.get(dev)
            if capturing and (t is None or t[3] != key):
                # the table would need a host-to-device copy, illegal under graph
                # capture: this pass splits per conv instead (correct, unbatched)
                self.live = False
                return
            if t is None or t[3] != key:
                items = (_lib.X3PlanesItem * len(es))(*[_lib.X3PlanesItem(ptr(e[0]()), ptr(e[3]), ptr(e[4]), e[1], e[2])
                                                        for e in es])
                host = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8)
                t = self.tables[dev] = (host.to(dev), len(es), max(e[1] * e[2] for e in es), key)
            check(_L().m3d_conv1_x3_planes_batched(ptr(t[0]), t[1], t[2], stream()), "conv1_x3_planes_batched")
            self.gen += 1
            for e in es:
                e[5] = True
        self.live = True

    def invalidate(self):
        self.live = False

    def cached(self, w, transpose):
        """The refreshed planes of w (None when not live / not registered yet)."""
        if not self.live:
            return None
        e = self.entries.get((w.data_ptr(), w.numel()))
        if e is None or not e[5] or e[0]() is None:
            return None
        self.hits += 1
        return e[3] if transpose else e[4]

    def ensure(self, w, cin, cout):
        """Register w (the caller's persistent kernel tensor) for the next refresh."""
        key = (w.data_ptr(), w.numel())
        e = self.entries.get(key)
        if (X3_PLANES_BATCHED and (e is None or e[0]() is None)
                and not torch.cuda.is_current_stream_capturing()):
            self.entries[key] = [weakref.ref(w), cin, cout,
                                 torch.empty(3 * cin * cout, device=w.device, dtype=torch.int16),
                                 torch.empty(3 * cin * cout, device=w.device, dtype=torch.int16), False]

    def get(self, w, cin, cout, transpose):
        p = self.cached(w, transpose)
        if p is not None:
            return p
        if self.live:
            self.misses += 1         # a split GEMM's planes not covered by this forward's refresh
        planes = torch.empty(3 * cin * cout, device=w.device, dtype=torch.int16)
        check(_L().m3d_conv1_x3_planes(ptr(w), cin, cout, 1 if transpose else 0, ptr(planes), stream()),
              "conv1_x3_planes")
        return planes


# one launch per model forward for every split-GEMM 1x1x1 kernel's planes
# (False: one m3d_conv1_x3_planes per conv call and per data gradient)
X3_PLANES_BATCHED = True
X3_PLANES = X3Planes()


class WinoVPrep:
    """The Winograd-domain weights of every 3x3x3 conv (the forward's and the
    data gradient's transform, m3d_conv3d_wino_weight_v), produced at the start
    of each model forward on a side stream instead of inside each conv on the
    compute stream.  They depend on the kernel only, so the ~75 small transform
    launches of a step (x3_wt_kernel + wino_weight_kernel per conv and data
    gradient) leave the critical path and overlap the stem / early layers.

    Registration and lifetime follow X3Planes: a conv registers its kernel (and
    the data-gradient tile it will use) the first time it runs, transforming
    inline that time; each RPN.forward refreshes every registered kernel
    (``refresh``: the side stream first waits for the compute stream, so the
    previous step's optimizer update and data gradients are ordered before the
    overwrite) and the convs of that forward take the buffers while ``live``,
    each after waiting for its own entry's event.  A unit's forward hands the
    data-gradient buffer, its event and the refresh generation to its backward
    (checked: a backward after another forward raises).  Buffers persist per
    kernel (~3 GB for the RPN's 3x3x3 convs)."""

    def __init__(self):
        self.entries = {}            # key -> [weakref(w), cin, cout, dgrad, ty, buf, nbytes, event, valid]
        self.live = False
        self.active_fwd = False      # this forward registers / takes the forward transforms (RPN.forward:
                                     # volumes >= WINO_V_PREPASS_MIN_VOXELS) ...
        self.active_dgrad = False    # ... and the data-gradient ones (every training forward)
        self.gen = 0
        self.streams = {}
        self.pending = set()         # devices whose pre-pass stream the next join() waits for

    def refresh(self, dev):
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.device(dev).index is None \
            else torch.device(dev)
        for k in [k for k, e in self.entries.items() if e[0]() is None]:
            del self.entries[k]
        es = [e for e in self.entries.values() if e[0]().device == dev
              and (self.active_dgrad if e[3] else self.active_fwd)]
        if not es:
            self.live = True
            return
        side = self.streams.get(dev)
        if side is None:
            side = self.streams[dev] = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        L = _L()
        with torch.cuda.stream(side):
            for e in es:
                check(L.m3d_conv3d_wino_weight_v(ptr(e[0]()), e[1], e[2], e[3], e[4], ptr(e[5]), e[6], stream()),
                      "conv3d_wino_weight_v")
                e[7].record(side)
                e[8] = True
        self.pending.add(dev)
        self.gen += 1
        self.live = True

    def invalidate(self):
        self.live = False

    def join(self):
        """The compute stream waits for the pre-pass stream (every entry a
        backward did not take is then ordered too; a HIP-graph capture needs the
        side stream joined before it ends)."""
        for dev in self.pending:
            torch.cuda.current_stream(dev).wait_stream(self.streams[dev])
        self.pending = set()

    def ensure(self, w, cin, cout, dgrad, ty):
        key = (w.data_ptr(), w.numel(), dgrad, ty)
        e = self.entries.get(key)
        if (e is None or e[0]() is None) and not torch.cuda.is_current_stream_capturing():
            nb = int(_L().m3d_conv3d_wino_v_bytes(cin, cout, dgrad, ty))
            if nb > 0:
                self.entries[key] = [weakref.ref(w), cin, cout, dgrad, ty,
                                     torch.empty(nb // 4 + 1, device=w.device, dtype=torch.float32), nb,
                                     torch.cuda.Event(), False]

    def take(self, w, dgrad, ty):
        """(buffer, event, gen) of w's refreshed transform, None when not live /
        not registered yet.  The caller waits on the event before using it."""
        if not self.live:
            return None
        e = self.entries.get((w.data_ptr(), w.numel(), dgrad, ty))
        if e is None or not e[8] or e[0]() is None:
            return None
        return e[5], e[7], self.gen


# (the RPN's) Winograd weight transforms on a side stream at the start of the
# forward, for volumes of at least WINO_V_PREPASS_MIN_VOXELS voxels.  Same box
# (scripts/r06/gpu_prepass.sh, gpu_prepass256.sh, gpu_prepass2.sh,
# profiles/r06_wino_prepass_ab.txt): 128^3 graph step 24.52 -> 24.25 and 24.39
# -> 24.10 ms, 256^3 147.4 -> 146.9 ms; at 64^3 the replay is slower with the
# side stream in the graph -- 9.92 -> 10.40 ms with both transforms on it, 9.88
# -> 10.76 ms with the data gradient's alone (configs[0] 10.6 -> 11.4 ms) -- so
# smaller volumes transform inline.  (active_fwd / active_dgrad stay separate
# switches for such A/Bs.)
WINO_V_PREPASS = True
WINO_V_PREPASS_MIN_VOXELS = 128 ** 3
WINO_V = WinoVPrep()


def _x3_planes(w, cin, cout, transpose):
    return X3_PLANES.get(w, cin, cout, transpose)


def _shared_wino_ws(wshare, role, ws, wsb, tag=None):
    """Workspace of a Winograd conv whose kernel is shared across calls
    (``wshare``: one dict per shared kernel and forward pass, e.g. the RPN
    head's rpn_conv_shared1 on P2..P6).  The first call of a role ("fwd" /
    "bwd") transforms the weights into its workspace, sized for the largest
    level, and keeps it; later calls of that role reuse the workspace with
    v_ready = 1 (no weight transform).  ``tag`` (weight pointer, Cin, Cout)
    guards the reuse: a held workspace transformed from other weights is never
    passed with v_ready = 1.  Returns (ws, ws_bytes, v_ready)."""
    if wshare is None:
        return ws, wsb, 0
    if role == "fwd":
        wshare["max_bytes"] = max(wshare.get("max_bytes", 0), wsb)
    if wshare.get("max_bytes", wsb) > SHARE_WINO_MAX_BYTES:
        # a held workspace this large (32 GB for P2 at 256^3) outlives the
        # level that needs it and crowds the caching allocator: per-level
        # workspaces as before (measured 204 -> 306 ms/step at 256^3 held)
        return ws, wsb, 0
    held = wshare.get(role)
    if held is not None and held[1] >= wsb and held[2] == tag:
        return held[0], held[1], 1
    nb = max(wsb, wshare.get("max_bytes", 0))
    if nb > wsb:
        ws = torch.empty(nb // 4 + 1, device=ws.device, dtype=torch.float32)
        wsb = nb
    wshare[role] = (ws, wsb, tag)
    return ws, wsb, 0


def _shared_wino_release(wshare):
    """After a shared kernel's data-gradient call: the last pending call of
    the pass drops the held 'bwd' workspace (it would otherwise live until the
    autograd graph is destroyed, through the rest of the backbone backward)."""
    if wshare is None or "pending_bwd" not in wshare:
        return
    wshare["pending_bwd"] -= 1
    if wshare["pending_bwd"] <= 0:
        wshare.pop("bwd", None)
        wshare.pop("pending_bwd", None)


def _wino_ws(B, H, W, D, OD, cin, cout, dev, dedicated=False):
    """(workspace, bytes) of one Winograd conv call, from the caching allocator.
    (A per-stream arena grown to the largest conv measured no better at 256^3 --
    216-940 ms before the side-stream throttle, DESIGN.md 5 -- and was removed.)"""
    n = int(_L().m3d_conv3d_wino_workspace_bytes(B, H, W, D, OD, cin, cout))
    return torch.empty(n // 4 + 1, device=dev, dtype=torch.float32), n


def release_wino_arena():
    """Kept for callers of the removed arena (bench.py): nothing is held."""
    return None


def same_out_pad(n, k, s):
    """TF 'SAME': out = ceil(n/s), pad_before = floor(max((out-1)s+k-n, 0)/2)."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2


def valid_out(n, k, s):
    return (n - k) // s + 1


def bn_act_bwd(dy, y, z, M, C, relu, scale, mean, rstd, dz, dres, sum_dpre, sum_xhat, sum_dz):
    """m3d_bn_act_bwd with its deterministic-reduction workspace."""
    L = _L()
    need = sum_dpre is not None or sum_xhat is not None or sum_dz is not None
    wsb = int(L.m3d_bn_act_bwd_workspace_bytes(M, C)) if need else 0
    ws = torch.empty(max(wsb // 4, 1), device=dy.device, dtype=torch.float32) if need else None
    check(L.m3d_bn_act_bwd(ptr(dy), ptr(y), ptr(z), M, C, 1 if relu else 0, ptr(scale), ptr(mean),
                           ptr(rstd), ptr(dz), ptr(dres), 0, ptr(sum_dpre), ptr(sum_xhat),
                           ptr(sum_dz), ptr(ws), wsb, stream()), "bn_act_bwd")


class BiasSums:
    """The bias gradients of the bias-only units of one forward (the FPN's
    fpn_c*p* / fpn_p* convs and the RPN class/bbox heads: out += column sums of
    the output gradient, tf.nn.bias_add's gradient), collected during the
    backward and reduced by two launches in ``flush`` (m3d_col_sums_batched,
    bit-identical per item to the per-unit m3d_bn_act_bwd) instead of two per
    unit.  Armed by RPN.forward for its training graph (BIAS_BATCH), flushed by
    RPNHead.finish_backward, i.e. before the weight-gradient join and before
    anything reads the gradients.  The output gradients stay referenced until
    the flush (same stream: no record_stream needed)."""

    def __init__(self):
        self.items = []           # (x, M, C, out)

    def add(self, x, M, C, out):
        if any(o is out or o.data_ptr() == out.data_ptr() for _, _, _, o in self.items) \
                or len(self.items) >= min(_lib.COL_SUMS_MAX, BIAS_BATCH_MAX):
            self.flush()
        self.items.append((x, M, C, out))

    def flush(self):
        items, self.items = self.items, []
        if not items:
            return
        L = _L()
        arr = (_lib.ColSumsItem * len(items))(*[_lib.ColSumsItem(ptr(x), M, C, ptr(o)) for x, M, C, o in items])
        wsb = int(L.m3d_col_sums_batched_workspace_bytes(arr, len(items)))
        if wsb <= 0:
            raise ValueError("col_sums_batched: " + L.m3d_last_error().decode())
        ws = torch.empty(wsb // 4 + 1, device=items[0][0].device, dtype=torch.float32)
        t0 = _span()
        check(L.m3d_col_sums_batched(arr, len(items), ptr(ws), wsb, stream()), "col_sums_batched")
        if LAYER_LOG is not None:
            _log("bias_sums", 0, 0, 4.0 * sum(x.numel() for x, _, _, _ in items), "bwd_bn",
                 f"{len(items)} bias-only units", t0)


# The BiasSums of the training forward being built (RPN.forward sets and
# clears it); None: every bias-only unit reduces its own bias gradient inline.
BIAS_BATCH = None
# Batch the bias-only units' reductions (True) or launch one per unit (False,
# default).  Measured at 128^3 (scripts/archive/gpu_r05_bias.sh, same box): eager
# neutral (26.34 vs 26.32 ms, 655 vs 679 launches per step), but the HIP-graph
# replay of the step slows from 26.0-26.2 to 30.6-30.7 ms with it on; under
# rocprofv3 the batched replay shows no such loss (its queue assignment is the
# clean one, r05gtrace2), so the cause is not found -- off until it is.  Ruled
# out (scripts/archive/gpu_r05_bias2.sh / _bias3.sh): where the flushes land (batches of
# 2 / 4 / 16: all 30.1-30.2 ms), the item table's kernel-argument size (a
# 4-item build: 30.1 ms) and which units are deferred (the FPN's alone, or the
# RPN heads' one sum alone: 29.9-30.0 ms) -- one reduction moved from the
# backward to finish_backward is enough.
BIAS_BATCHED = False
# most items per batched launch (flushed when full; A/B of where the flushes land)
BIAS_BATCH_MAX = 16
# which bias-only units join the batch: the FPN convs ("fpn") and / or the RPN
# class / bbox heads ("rpn")
BIAS_BATCH_UNITS = "fpn+rpn"


def bias_grad(dy, M, C, out, grads=None, batch=None):
    """out += column sums of dy [M, C]: batched when ``batch`` is armed and the
    unit has no bucket hook (a DP all-reduce may start as soon as the unit's
    gradients are signalled done), inline otherwise."""
    if batch is not None and BIAS_BATCHED and not (grads and grads.get("_hook") is not None):
        batch.add(dy, M, C, out)
    else:
        bn_act_bwd(dy, None, None, M, C, False, None, None, None, None, None, None, None, out)


@dataclass
class ConvGeom:
    k: tuple
    stride: tuple
    pad: tuple        # pad-before per axis
    out: tuple        # output spatial (OH, OW, OD)


def conv_geom(in_sp, k, stride, padding):
    """padding: 'same' | 'valid' | int (explicit symmetric zero padding, ZeroPadding3D)."""
    k = tuple(k)
    stride = tuple(stride)
    if padding == "same":
        op = [same_out_pad(n, kk, s) for n, kk, s in zip(in_sp, k, stride)]
        return ConvGeom(k, stride, tuple(p for _, p in op), tuple(o for o, _ in op))
    if padding == "valid":
        return ConvGeom(k, stride, (0, 0, 0), tuple(valid_out(n, kk, s) for n, kk, s in zip(in_sp, k, stride)))
    p = int(padding)
    return ConvGeom(k, stride, (p, p, p),
                    tuple(valid_out(n + 2 * p, kk, s) for n, kk, s in zip(in_sp, k, stride)))


class GradLink:
    """Lets the bwd-data kernel accumulate one consumer's gradient of a tensor
    into another's (accumulate=1) instead of autograd adding two full tensors.

    mode "res" -- identity_block (core/models.py:157-189): x is both conv 2a's
    input and conv 2c's residual; 2c's backward always runs before 2a's (2a ->
    2b -> 2c), so 2c parks dres in ``buf`` and returns no residual gradient.
    mode "dx2" -- conv_block (core/models.py:192-232): x is the input of both
    the shortcut conv and conv 2a, whose backward order is not fixed: the
    first to run parks its dx and returns none, the second accumulates into
    the parked buffer and returns the sum.

    A link is bound to the tensor x it carries the gradient of (its storage
    pointer and shape): a parked buffer is only handed to that tensor's
    consumer.  ``registry`` (a list owned by the model's forward) collects the
    links; check_links() after the backward raises if a parked gradient was
    never consumed (a partner backward that did not run, e.g. autograd.grad on
    an intermediate), instead of silently dropping it."""
    __slots__ = ("buf", "mode", "key")

    def __init__(self, mode="res", x=None, registry=None):
        self.buf = None
        self.mode = mode
        self.key = None if x is None else (x.data_ptr(), tuple(x.shape))
        if registry is not None:
            registry.append(self)


def check_links(links):
    """Raise if any GradLink still holds a parked gradient (see GradLink)."""
    bad = [l for l in links if l.buf is not None]
    if bad:
        raise RuntimeError(f"{len(bad)} parked residual/shortcut gradient(s) were never consumed: "
                           "both consumers of a linked tensor must run their backward in the same pass")


def _link_take(link, x):
    """(parked gradient of x, 1) if the link holds one for x, else (None, 0)."""
    if link is not None and link.buf is not None and link.buf.shape == x.shape and (
            link.key is None or link.key == (x.data_ptr(), tuple(x.shape))):
        buf, link.buf = link.buf, None
        return buf, 1
    return None, 0


def _link_park(link, dx, acc):
    """mode dx2, first consumer: park dx and return no gradient."""
    if link is not None and link.mode == "dx2" and not acc and dx is not None:
        link.buf = dx
        return None
    return dx


# Fused BN-ReLU backward (m3d_conv3d_bwd_data_bn / _wino_bn): the data
# gradient of a unit's sole consumer applies the unit's frozen-BN + ReLU backward
# in its epilogue (dz and dres stored, the beta / gamma / bias sums reduced from
# per-tile partials), so the unit's own backward skips bn_act_bwd -- one
# read-modify-write pass over the activation gradient less per fused unit.
# BN_FUSE = False runs bn_act_bwd everywhere (A/B; tests/test_gpu_bnfuse.py).
BN_FUSE = True
# ... and in the bf16-split 1x1x1 data gradient (m3d_conv3d_bwd_data_x3_bn;
# False: that GEMM's plain store, then the producer's bn_act_bwd).  Round 5
# had it off (the epilogue spilled: 25.49 vs 25.05 ms at 128^3); round 6's
# spill-free x3_gemm256_af_kernel<2> (per-wave LDS staging, float4 rows):
# 128^3 24.54 vs 24.60 ms, 256^3 148.1 vs 148.8 ms, same box
# (scripts/r06/gpu_fuse.sh, profiles/r06_x3_bn_fuse_ab.txt).
X3_BN_FUSE = True


class BNFuse:
    """Hand-off of one unit's BN-ReLU backward to its consumer's data gradient.

    The model wires it where the graph guarantees the consumer's data gradient
    is the last contribution to the unit's output gradient: a block's 2a -> 2b
    and 2b -> 2c, an identity block's input conv (whose GradLink already holds
    the residual gradient), the RPN head's shared1 -> shared2.  The producer
    arms it in forward; the consumer fuses when its data-gradient kernel has the
    fused form and its result is final, and marks it ``done``; the producer's
    backward then takes the incoming gradient as its dz (checked to be the
    consumer's buffer: any other contribution raises instead of being lost).

    While ``done`` is set, the consumer has already written the unit's dz (not
    dL/dy) into the gradient it returns, and added the unit's beta / gamma /
    bias sums: a hook on the unit's output, or autograd.grad stopping at it,
    sees dz.  ``registry`` (a list owned by the model's forward) collects the
    records; check_fuses() after the backward raises if one was applied by its
    consumer but never consumed by its producer's backward (a partial backward),
    as check_links() does for a parked GradLink."""
    __slots__ = ("armed", "done", "y", "z", "bn", "relu", "need_res", "grads", "buf", "dres", "name")

    def __init__(self, registry=None):
        self.armed = self.done = False
        self.y = self.z = self.bn = self.grads = self.buf = self.dres = None
        self.relu = self.need_res = False
        self.name = ""
        if registry is not None:
            registry.append(self)

    def arm(self, y, z, bn, relu, need_res, grads, name):
        self.armed, self.done = True, False
        self.y, self.z, self.bn, self.relu, self.need_res, self.grads, self.name = \
            y, z, bn, relu, need_res, grads, name
        self.buf = self.dres = None

    def clear(self):
        self.armed = self.done = False
        self.y = self.z = self.bn = self.grads = self.buf = self.dres = None

    def descriptor(self, dres, item=None):
        """The m3d_bn_bwd_t of the fused entry points (the tensors stay held by
        this record and the caller's dres); ``item``: batch item b's rows only."""
        g = self.grads or {}
        mean = rstd = scale = None
        if self.bn is not None:
            mean, rstd, scale = self.bn
        y, z = self.y, self.z
        if item is not None:
            y = y[item:item + 1]
            z = z[item:item + 1] if z is not None else None
            dres = dres[item:item + 1] if dres is not None else None
        d = _lib.BnBwd(ptr(y), ptr(z), ptr(scale), ptr(mean), ptr(rstd), 1 if self.relu else 0,
                       ptr(dres), ptr(g.get("beta")), ptr(g.get("gamma") if z is not None else None),
                       ptr(g.get("bias")))
        return d


def check_fuses(records):
    """Raise if a BNFuse record was applied by its consumer's data gradient but
    its producer's backward never took it (see BNFuse)."""
    bad = [r.name for r in records if r.done]
    if bad:
        raise RuntimeError(f"fused BN-ReLU backward of {bad[:4]} was applied by the consumer's data gradient, "
                           "but the producing unit's backward never ran in this pass (its BN sums are already "
                           "accumulated and its output gradient holds dz, not dL/dy)")


def _per_item(B, vin, cin, vout, cout):
    """csrc/conv3d.hip per_item(): batches whose operands pass the 32-bit bound
    run one item at a time (the fused forms refuse those)."""
    lim = int(os.environ.get("M3D_OPERAND_LIMIT", "0") or 0)
    lim = (lim if 0 < lim < 0xFFFFFFF0 else 0xFFFFFFF0) // 4
    return B > 1 and (B * vin * cin >= lim or B * vout * cout >= lim or B * vin > 0x7FFFFFFF
                      or B * vout > 0x7FFFFFFF)


def _fuse_final(link, x, acc):
    """Is this data gradient the last contribution to x's gradient?  A linked x
    (GradLink keyed by x) is final once the parked partner gradient was taken
    (acc = 1); an unlinked one is final on its own (the model wires BNFuse only
    to sole consumers)."""
    linked = link is not None and link.key == (x.data_ptr(), tuple(x.shape))
    return acc == 1 if linked else acc == 0


def _bn_fuse_ws(rec, B, H, W, D, C, dev):
    g = rec.grads or {}
    if g.get("beta") is None and g.get("bias") is None and (g.get("gamma") is None or rec.z is None):
        return None, 0
    n = int(_L().m3d_bn_bwd_fused_workspace_bytes(B, H, W, D, C))
    return torch.empty(n // 4 + 1, device=dev, dtype=torch.float32), n


class _ConvBNAct(torch.autograd.Function):
    """y = act(BN_frozen(conv(x, w) + b) [+ residual]).

    res_mode 1: residual has y's shape; 2: residual is the (2,2,1)-nearest
    source of y (FPN top-down add, core/models.py:3193-3204)."""

    @staticmethod
    def forward(ctx, x, residual, w, b, bn, geo, relu, res_mode, grads, need_dx, link=None, halo=None,
                wshare=None, name="", fuse=None, fuse_in=None):
        t0 = _span()
        ctx.name = name
        B, H, W, D, Cin = x.shape
        # depth slab (m3d.slab): halo = (planes [B,H,W,2,C], has_lo, has_hi) read by the
        # Winograd kernels beside x instead of a halo-extended copy of x; a
        # slab.PendingHalo (exchange still in flight) is resolved between the two
        # launch phases of the Winograd conv below
        pending = halo if isinstance(halo, slab.PendingHalo) else None
        if pending is not None:
            halo = (None, pending.has_lo, pending.has_hi)
        ctx.halo = halo
        kh, kw, kd = geo.k
        Cout = w.shape[-1]
        OH, OW, OD = geo.out
        y = torch.empty((B, OH, OW, OD, Cout), device=x.device, dtype=torch.float32)
        z = None
        scale = shift = None
        if bn is not None:
            gamma, beta, mean, var, eps = bn[:5]
            aff = bn[5] if len(bn) > 5 else None
            # the batched affine is a view into the store's shared buffer: the next
            # refresh overwrites it (checked in backward, _check_generations)
            ctx.aff_gen = bn[6] if len(bn) > 6 else None
            if aff is None:
                aff = torch.empty((3, Cout), device=x.device, dtype=torch.float32)
                check(_L().m3d_bn_affine(ptr(gamma), ptr(beta), ptr(mean), ptr(var), float(eps), Cout,
                                         ptr(aff[1]), ptr(aff[2]), ptr(aff[0]), stream()), "bn_affine")
            rstd, scale, shift = aff[0], aff[1], aff[2]
            if grads is not None and grads.get("gamma") is not None:
                z = torch.empty_like(y)
            ctx.bn = (mean, rstd, scale)
        else:
            ctx.bn = None
            ctx.aff_gen = None
        ctx.wino = use_winograd(geo, Cin, Cout, (H, W, D)) and res_mode != 2
        ctx.vd = None
        if halo is not None and not ctx.wino and not _stem_halo(geo, Cin, Cout, res_mode):
            raise ValueError("halo planes are read by the Winograd kernels and the stem only")
        ctx.u = None
        if halo is not None and not ctx.wino:
            # the 7^3 stem on a depth slab: the neighbours' 3 planes beside the slab
            r = halo[0].shape[3] // 2
            check(_L().m3d_conv3d_fwd_halo(ptr(x), ptr(halo[0]), halo[1], halo[2], r, B, H, W, D, Cin, ptr(w),
                                           kh, kw, kd, Cout, OH, OW, OD, *geo.stride, *geo.pad, ptr(b),
                                           ptr(scale), ptr(shift), 1 if relu else 0, ptr(z), ptr(y), stream()),
                  "conv3d_fwd_halo")
        elif ctx.wino:
            dext = D + (halo[1] + halo[2] if halo is not None else 0)
            ws, wsb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device)
            # training: keep the transformed input U for the weight gradient when
            # the forward and weight-gradient tiles agree (u_bytes > 0)
            nu = int(_L().m3d_conv3d_wino_u_bytes(B, H, W, OD, Cin)) // 4 \
                if grads is not None and grads.get("kernel") is not None \
                and min(Cin, Cout) >= WINO_WGRAD_MIN_C else 0
            if nu * 4 > WINO_KEEP_MAX_BYTES:
                nu = 0          # too large to hold until the backward: the weight gradient re-transforms x
            vf = None
            ctx.vd = None
            if WINO_V_PREPASS and halo is None:
                if WINO_V.active_fwd:
                    WINO_V.ensure(w, Cin, Cout, 0, 0)
                    vf = WINO_V.take(w, 0, 0)
                    if vf is not None:
                        torch.cuda.current_stream().wait_event(vf[1])
                if need_dx and WINO_V.active_dgrad:
                    ty = _dgrad_tile_y(name)
                    WINO_V.ensure(w, Cin, Cout, 1, ty)
                    ctx.vd = WINO_V.take(w, 1, ty)      # waited on in the backward
            if pending is not None:
                # phase 1 (weights + interior z tiles) overlaps the halo transfer
                ctx.u = torch.empty(nu, device=x.device, dtype=torch.float32) if nu > 0 else None
                args = (B, H, W, D, Cin, ptr(w), Cout, ptr(b), ptr(scale), ptr(shift), ptr(residual),
                        1 if relu else 0, ptr(z), ptr(y), ptr(ctx.u), ptr(ws), wsb)
                check(_L().m3d_conv3d_fwd_wino_halo_phase(ptr(x), None, halo[1], halo[2], *args, 1, stream()),
                      "conv3d_fwd_wino_halo_phase1")
                halo = ctx.halo = pending.result()
                check(_L().m3d_conv3d_fwd_wino_halo_phase(ptr(x), ptr(halo[0]), halo[1], halo[2], *args, 2,
                                                          stream()), "conv3d_fwd_wino_halo_phase2")
            elif halo is not None:
                ctx.u = torch.empty(nu, device=x.device, dtype=torch.float32) if nu > 0 else None
                check(_L().m3d_conv3d_fwd_wino_halo(ptr(x), ptr(halo[0]), halo[1], halo[2], B, H, W, D, Cin,
                                                    ptr(w), Cout, ptr(b), ptr(scale), ptr(shift), ptr(residual),
                                                    1 if relu else 0, ptr(z), ptr(y), ptr(ctx.u), ptr(ws), wsb,
                                                    stream()), "conv3d_fwd_wino_halo")
            elif vf is not None:
                # the transformed weights from this forward's side-stream pre-pass (WinoVPrep)
                ctx.u = torch.empty(nu, device=x.device, dtype=torch.float32) if nu > 0 else None
                check(_L().m3d_conv3d_fwd_wino_kv(ptr(x), B, H, W, D, Cin, ptr(w), Cout, OD, geo.pad[2],
                                                  ptr(b), ptr(scale), ptr(shift), ptr(residual), 1 if relu else 0,
                                                  ptr(z), ptr(y), ptr(ctx.u), ptr(vf[0]), ptr(ws), wsb, stream()),
                      "conv3d_fwd_wino_kv")
            elif nu > 0:
                ctx.u = torch.empty(nu, device=x.device, dtype=torch.float32)
                check(_L().m3d_conv3d_fwd_wino_keep(ptr(x), B, H, W, D, Cin, ptr(w), Cout, OD, geo.pad[2],
                                                    ptr(b), ptr(scale), ptr(shift), ptr(residual),
                                                    1 if relu else 0, ptr(z), ptr(y), ptr(ctx.u),
                                                    ptr(ws), wsb, stream()), "conv3d_fwd_wino_keep")
            else:
                if wshare is not None:          # may be held across calls: not the arena
                    ws, wsb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device, dedicated=True)
                ws, wsb, v_ready = _shared_wino_ws(wshare, "fwd", ws, wsb, (w.data_ptr(), Cin, Cout))
                check(_L().m3d_conv3d_fwd_wino_v(ptr(x), B, H, W, D, Cin, ptr(w), Cout, OD, geo.pad[2],
                                                 ptr(b), ptr(scale), ptr(shift), ptr(residual), 1 if relu else 0,
                                                 ptr(z), ptr(y), ptr(ws), wsb, v_ready, stream()),
                      "conv3d_fwd_wino")
        elif res_mode <= 2 and _conv1_x3(x.shape, geo, Cin, Cout):
            planes = _x3_planes(w, Cin, Cout, True)
            X3_PLANES.ensure(w, Cin, Cout)
            check(_L().m3d_conv3d_fwd_x3(ptr(x), B, H, W, D, Cin, ptr(planes), Cout, ptr(b), ptr(scale),
                                         ptr(shift), ptr(residual), res_mode, 1 if relu else 0, ptr(z), ptr(y),
                                         stream()), "conv3d_fwd_x3")
        else:
            nsk = _splitk(x.shape, geo, Cin, Cout, 0)
            if nsk > 1:
                wsk = torch.empty((nsk, y.numel()), device=x.device, dtype=torch.float32)
                check(_L().m3d_conv3d_fwd_splitk(ptr(x), *x.shape, ptr(w), Cout, OH, OW, OD, *geo.stride,
                                                 ptr(b), ptr(scale), ptr(shift), ptr(residual), res_mode,
                                                 1 if relu else 0, ptr(z), ptr(y), nsk, ptr(wsk),
                                                 wsk.numel() * 4, stream()), "conv3d_fwd_splitk")
            else:
                check(_L().m3d_conv3d_fwd(ptr(x), *x.shape, ptr(w), *geo.k, Cout, OH, OW, OD,
                                          *geo.stride, *geo.pad, ptr(b), ptr(scale), ptr(shift),
                                          ptr(residual), res_mode, 1 if relu else 0, ptr(z), ptr(y), Cout,
                                          None, 0, 0, stream()), "conv3d_fwd")
        if LAYER_LOG is not None:
            direct = 2.0 * (y.numel() // Cout) * kh * kw * kd * Cin * Cout
            exe = direct
            if ctx.wino:
                exe = _wino_exec(B, OH, OW, OD, Cin, Cout, int(_L().m3d_conv3d_wino_tile_z()))
            nb = 4.0 * (x.numel() + w.numel() + y.numel() + (residual.numel() if residual is not None else 0))
            x3 = ctx.wino or (res_mode <= 2 and halo is None and _conv1_x3(x.shape, geo, Cin, Cout))
            _log("wino" if ctx.wino else f"conv{kh}", direct, exe, nb, "fwd", name, t0, "x3" if x3 else "f32")
        ctx.save_for_backward(x, w, y, z)
        ctx.wshare = wshare
        if wshare is not None and ctx.wino and halo is None and need_dx:
            # data-gradient calls still to come: the last one releases the held workspace
            wshare["pending_bwd"] = wshare.get("pending_bwd", 0) + 1
        ctx.geo, ctx.relu, ctx.res_mode, ctx.grads, ctx.need_dx = geo, relu, res_mode, grads, need_dx
        # the data gradient's split planes of this forward's refresh (X3Planes), if any
        ctx.x3_bwd = None
        if (geo.k == (1, 1, 1) and need_dx and halo is None
                and _conv1_x3(x.shape, geo, Cout, Cin, bwd_data=True, fused=X3_BN_FUSE)):
            ctx.x3_bwd = X3_PLANES.cached(w, False)
            if ctx.x3_bwd is None:
                X3_PLANES.ensure(w, Cin, Cout)
        ctx.x3_gen = X3_PLANES.gen if ctx.x3_bwd is not None else None
        ctx.bias_batch = BIAS_BATCH if grads is not None else None
        ctx.link = link
        ctx.res_shape = None if residual is None else tuple(residual.shape)
        # this unit's BN-ReLU backward handed to its consumer (BNFuse)
        ctx.fuse = None
        # (res_mode 2, the FPN's upsampled residual, has no fused form: its residual
        # gradient needs the upsample adjoint, so such a unit is never armed)
        if (fuse is not None and BN_FUSE and grads is not None and (bn is not None or relu)
                and Cout % 4 == 0 and res_mode in (0, 1)):
            fuse.arm(y, z, ctx.bn, relu, res_mode != 0, grads, name)
            ctx.fuse = fuse
        # ... and the producer's, applied in this unit's data gradient
        ctx.fuse_in = None
        if (fuse_in is not None and fuse_in.armed and need_dx and halo is None and wshare is None
                and fuse_in.y is not None and fuse_in.y.data_ptr() == x.data_ptr()
                and fuse_in.y.shape == x.shape):
            ctx.fuse_in = fuse_in
        return y

    @staticmethod
    def backward(ctx, dy):
        _check_generations(ctx)
        x, w, y, z = ctx.saved_tensors
        dy = dy.contiguous()
        geo, grads = ctx.geo, ctx.grads or {}
        B, H, W, D, Cin = x.shape
        kh, kw, kd = geo.k
        Cout = w.shape[-1]
        OH, OW, OD = geo.out
        M = B * OH * OW * OD
        L = _L()
        need_res = ctx.res_mode != 0
        trivial = ctx.bn is None and not ctx.relu
        logging = LAYER_LOG is not None
        direct = 2.0 * M * kh * kw * kd * Cin * Cout
        t0 = _span()
        rec = ctx.fuse
        ctx.fuse = None
        fused_bn = rec is not None and rec.done
        if fused_bn:
            # the consumer's data gradient already applied this unit's BN-ReLU
            # backward: dy is its dz buffer, dres and the BN / bias sums are written
            if rec.buf is None or dy.data_ptr() != rec.buf.data_ptr() or dy.shape != rec.buf.shape:
                raise RuntimeError(f"{ctx.name}: fused BN-ReLU backward was applied by its consumer, but the "
                                   "output gradient has another contribution (the unit is not the consumer's "
                                   "sole producer-consumer pair; see nn.BNFuse)")
            dz = dy
            dres = rec.dres
            rec.clear()
        elif trivial:
            if rec is not None:
                rec.clear()
            dz = dy
            dres = dy if need_res else None
            if grads.get("bias") is not None:
                bias_grad(dy, M, Cout, grads["bias"], grads,
                          ctx.bias_batch if "fpn" in BIAS_BATCH_UNITS.split("+") else None)
        else:
            if rec is not None:
                rec.clear()
            dz = torch.empty_like(dy)
            dres = torch.empty_like(dy) if need_res else None
            mean = rstd = scale = None
            if ctx.bn is not None:
                mean, rstd, scale = ctx.bn
            bn_act_bwd(dy, y, z, M, Cout, ctx.relu, scale, mean, rstd, dz, dres, grads.get("beta"),
                       grads.get("gamma") if z is not None else None, grads.get("bias"))
        if logging and not fused_bn and not (trivial and ctx.bias_batch is not None and BIAS_BATCHED
                                             and grads.get("_hook") is None):
            nel = dy.numel() * (1 + (0 if trivial else 1 + (ctx.relu or ctx.bn is not None) +
                                     (z is not None) + (dres is not None and not trivial)))
            _log("bn_act_bwd", 0, 0, 4.0 * nel, "bwd_bn", ctx.name, t0)
        side = _wgrad_stream(x.device) if grads.get("kernel") is not None else None
        if side is not None:
            dz.record_stream(side)
            x.record_stream(side)
        halo = ctx.halo
        dext = D + (halo[1] + halo[2] if halo is not None else 0)
        if halo is not None and side is not None:
            halo[0].record_stream(side)
        if ctx.wino:
            def wgrad():
                with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                    tw = _span()
                    if min(Cin, Cout) < WINO_WGRAD_MIN_C and halo is not None:
                        # the direct kernel reads the neighbours' planes beside the slab
                        check(L.m3d_conv3d_bwd_weight_halo(ptr(x), ptr(halo[0]), halo[1], halo[2], 1, ptr(dz),
                                                           B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD,
                                                           *geo.stride, *geo.pad, ptr(grads["kernel"]), stream()),
                              "conv3d_bwd_weight_halo")
                    elif min(Cin, Cout) < WINO_WGRAD_MIN_C:
                        check(L.m3d_conv3d_bwd_weight(ptr(x), ptr(dz), B, H, W, D, Cin, kh, kw, kd,
                                                      Cout, OH, OW, OD, *geo.stride, *geo.pad,
                                                      ptr(grads["kernel"]), stream()), "conv3d_bwd_weight")
                    elif halo is not None and ctx.u is None:
                        wsw, wswb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device)
                        check(L.m3d_conv3d_bwd_weight_wino_halo(ptr(x), ptr(halo[0]), halo[1], halo[2], ptr(dz),
                                                                B, H, W, D, Cin, Cout, ptr(grads["kernel"]),
                                                                ptr(wsw), wswb, stream()),
                              "conv3d_bwd_weight_wino_halo")
                    else:
                        wsw, wswb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device)
                        if ctx.u is not None:
                            ctx.u.record_stream(torch.cuda.current_stream())
                            check(L.m3d_conv3d_bwd_weight_wino_u(ptr(ctx.u), ptr(dz), B, H, W, D, Cin, Cout,
                                                                 OD, geo.pad[2], ptr(grads["kernel"]),
                                                                 ptr(wsw), wswb, stream()),
                                  "conv3d_bwd_weight_wino_u")
                        else:
                            check(L.m3d_conv3d_bwd_weight_wino(ptr(x), ptr(dz), B, H, W, D, Cin, Cout, OD,
                                                               geo.pad[2], ptr(grads["kernel"]), ptr(wsw),
                                                               wswb, stream()),
                                  "conv3d_bwd_weight_wino")
                    if logging:
                        exe = direct if min(Cin, Cout) < WINO_WGRAD_MIN_C else \
                            _wino_exec(B, OH, OW, OD, Cin, Cout, int(L.m3d_conv3d_wino_wgrad_tile_z()))
                        _log("wino_wgrad", direct, exe, 4.0 * (x.numel() + dz.numel() + w.numel()),
                             "bwd_weight", ctx.name, tw, "f32" if min(Cin, Cout) < WINO_WGRAD_MIN_C else "x3")
                ctx.u = None
            has_w = grads.get("kernel") is not None
            if has_w and not WGRAD_LAST:
                wgrad()
            td = _span()
            ws, wsb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device)
            dx = None
            fused_nel = 0
            if ctx.need_dx:
                dx, acc = _link_take(ctx.link, x)
                if dx is None:
                    dx = torch.empty(x.shape, device=x.device, dtype=torch.float32)
                ty = 0 if halo is not None else _dgrad_tile_y(ctx.name)
                if halo is not None:
                    dh = torch.empty_like(halo[0])
                    check(L.m3d_conv3d_bwd_data_wino_halo(ptr(dz), ptr(w), halo[1], halo[2], B, H, W, D, Cin,
                                                          Cout, ptr(dx), ptr(dh), acc, ptr(ws), wsb, stream()),
                          "conv3d_bwd_data_wino_halo")
                    slab.return_halo_grads(dx, dh)
                else:
                    vd = ctx.vd                     # the forward pre-pass's data-gradient transform (WinoVPrep)
                    if vd is not None:
                        if vd[2] != WINO_V.gen:
                            raise RuntimeError(f"{ctx.name}: conv backward after another model forward: the "
                                               "pre-transformed Winograd weights were refreshed (run each backward "
                                               "before the next forward)")
                        torch.cuda.current_stream().wait_event(vd[1])
                        v_ready = 0
                    else:
                        if ctx.wshare is not None:      # may be held across calls: not the arena
                            ws, wsb = _wino_ws(B, H, W, dext, OD, Cin, Cout, x.device, dedicated=True)
                        ws, wsb, v_ready = _shared_wino_ws(ctx.wshare, "bwd", ws, wsb, (w.data_ptr(), Cin, Cout, ty))
                    rec = ctx.fuse_in
                    if (rec is not None and rec.armed and (Cin % 256 == 0 or 256 % Cin == 0)
                            and not _per_item(B, H * W * max(D, OD), max(Cin, Cout), 0, 0)
                            and _fuse_final(ctx.link, x, acc)):
                        dres_f = torch.empty_like(x) if rec.need_res else None
                        bws, bwsb = _bn_fuse_ws(rec, B, H, W, D, Cin, x.device)
                        d = rec.descriptor(dres_f)
                        if vd is not None:
                            check(L.m3d_conv3d_bwd_data_wino_xv(ptr(dz), ptr(w), B, H, W, D, Cin, Cout, OD,
                                                                geo.pad[2], ptr(dx), acc, ptr(ws), wsb, ptr(vd[0]), ty,
                                                                ctypes.addressof(d), ptr(bws), bwsb, stream()),
                                  "conv3d_bwd_data_wino_xv(bn)")
                        else:
                            check(L.m3d_conv3d_bwd_data_wino_bny(ptr(dz), ptr(w), B, H, W, D, Cin, Cout, OD,
                                                                 geo.pad[2], ptr(dx), acc, ptr(ws), wsb, v_ready,
                                                                 ctypes.addressof(d), ptr(bws), bwsb, ty, stream()),
                                  "conv3d_bwd_data_wino_bn")
                        rec.buf, rec.dres, rec.done = dx, dres_f, True
                        fused_nel = x.numel() * (1 + (rec.z is not None) + rec.need_res)
                    elif vd is not None:
                        check(L.m3d_conv3d_bwd_data_wino_xv(ptr(dz), ptr(w), B, H, W, D, Cin, Cout, OD, geo.pad[2],
                                                            ptr(dx), acc, ptr(ws), wsb, ptr(vd[0]), ty, None, None, 0,
                                                            stream()), "conv3d_bwd_data_wino_xv")
                    else:
                        check(L.m3d_conv3d_bwd_data_wino_vy(ptr(dz), ptr(w), B, H, W, D, Cin, Cout, OD,
                                                            geo.pad[2], ptr(dx), acc, ptr(ws), wsb, v_ready, ty,
                                                            stream()), "conv3d_bwd_data_wino")
                    _shared_wino_release(ctx.wshare)
                if logging:
                    _log("wino_dgrad", direct, _wino_exec(B, OH, OW, OD, Cin, Cout, int(L.m3d_conv3d_wino_dgrad_tile_z()),
                                                          ty or int(L.m3d_conv3d_wino_dgrad_tile_y())),
                         4.0 * (dz.numel() + w.numel() + x.numel() * (1 + acc) + fused_nel), "bwd_data", ctx.name,
                         td, "x3")
                dx = _link_park(ctx.link, dx, acc)
            if has_w and WGRAD_LAST:
                wgrad()
            _grad_done(grads, side)
            ctx.halo = None
            ctx.fuse_in = None
            return (dx, (dres if need_res else None), None, None, None, None, None, None, None, None, None, None,
                    None, None, None, None)
        if halo is not None and ctx.need_dx:
            raise ValueError("the stem's halo form has no data gradient (its input is the volume)")
        strided_x3 = (WGRAD1_STRIDED_X3 and halo is None and geo.k == (1, 1, 1) and geo.stride == (2, 2, 1)
                      and geo.pad == (0, 0, 0) and (OH, OW, OD) == ((H + 1) // 2, (W + 1) // 2, D)
                      and Cin % 4 == 0 and Cout >= 65)      # (_wgrad1_x3 of the stride-1 form)

        def wgrad_d():
            with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
                tw = _span()
                if halo is not None:        # the stem on a depth slab: halo planes beside the slab
                    check(L.m3d_conv3d_bwd_weight_halo(ptr(x), ptr(halo[0]), halo[1], halo[2], halo[0].shape[3] // 2,
                                                       ptr(dz), B, H, W, D, Cin, kh, kw, kd, Cout, OH, OW, OD,
                                                       *geo.stride, *geo.pad, ptr(grads["kernel"]), stream()),
                          "conv3d_bwd_weight_halo")
                elif strided_x3:
                    # the stage-first blocks' (2,2,1)-strided 1x1x1 convs: their input rows
                    # gathered once (x[:, ::2, ::2]), then the stride-1 split-GEMM gradient
                    xs = torch.empty((B, OH, OW, OD, Cin), device=x.device, dtype=torch.float32)
                    check(L.m3d_subsample221_fwd(ptr(x), B, H, W, D, Cin, ptr(xs), stream()), "subsample221")
                    check(L.m3d_conv3d_bwd_weight(ptr(xs), ptr(dz), B, OH, OW, OD, Cin, 1, 1, 1, Cout, OH, OW, OD,
                                                  1, 1, 1, 0, 0, 0, ptr(grads["kernel"]), stream()),
                          "conv3d_bwd_weight")
                    del xs
                else:
                    check(L.m3d_conv3d_bwd_weight(ptr(x), ptr(dz), B, H, W, D, Cin, kh, kw, kd, Cout, OH,
                                                  OW, OD, *geo.stride, *geo.pad, ptr(grads["kernel"]),
                                                  stream()), "conv3d_bwd_weight")
                if logging:
                    _log(f"conv{kh}_wgrad", direct, direct, 4.0 * (x.numel() + dz.numel() + w.numel()),
                         "bwd_weight", ctx.name, tw,
                         "x3" if halo is None and (strided_x3 or _wgrad1_x3(geo, Cin, Cout, (H, W, D))) else "f32")
        has_w = grads.get("kernel") is not None
        if has_w and not WGRAD_LAST:
            wgrad_d()
        dx = None
        link = ctx.link
        acc = 0
        td = _span()
        rec = ctx.fuse_in
        fused_nel = 0
        if ctx.need_dx:
            strided = any(s != 1 for s in geo.stride)
            dx, acc = _link_take(link, x)                     # dx = parked gradient + conv^T dz
            if dx is None:
                dx = (torch.zeros if strided else torch.empty)(x.shape, device=x.device, dtype=torch.float32)
            wd, dzd, cpad = w, dz, Cout
            if Cout % 32:   # bwd-data stages 32-channel slices of dz: zero-pad the channel dim
                cpad = -(-Cout // 32) * 32
                wd = torch.zeros((kh, kw, kd, Cin, cpad), device=w.device, dtype=torch.float32)
                wd[..., :Cout] = w
                dzd = torch.zeros((B, OH, OW, OD, cpad), device=dz.device, dtype=torch.float32)
                dzd[..., :Cout] = dz
            nsk = _splitk(x.shape, geo, Cin, cpad, 1)
            dx_x3 = cpad == Cout and not acc and _conv1_x3(x.shape, geo, Cout, Cin, bwd_data=True)
            dx_x3f = (cpad == Cout and X3_BN_FUSE and rec is not None and rec.armed and (X3_BN_FUSE_ACC or not acc)
                      and _conv1_x3(x.shape, geo, Cout, Cin, bwd_data=True, fused=True))
            if dx_x3f and _fuse_final(link, x, acc):
                # the producer's BN-ReLU backward in the split GEMM's epilogue (+ the parked gradient)
                dx_x3 = True
                planes = ctx.x3_bwd if ctx.x3_bwd is not None else _x3_planes(w, Cin, Cout, False)
                dres_f = torch.empty_like(x) if rec.need_res else None
                bws, bwsb = _bn_fuse_ws(rec, B, H, W, D, Cin, x.device)
                d = rec.descriptor(dres_f)
                check(L.m3d_conv3d_bwd_data_x3_bna(ptr(dz), ptr(planes), B, H, W, D, Cin, Cout, ptr(dx), acc,
                                                   ctypes.addressof(d), ptr(bws), bwsb, stream()),
                      "conv3d_bwd_data_x3_bna")
                rec.buf, rec.dres, rec.done = dx, dres_f, True
                fused_nel = x.numel() * (1 + (rec.z is not None) + rec.need_res)
            elif dx_x3:
                planes = ctx.x3_bwd if ctx.x3_bwd is not None else _x3_planes(w, Cin, Cout, False)
                check(L.m3d_conv3d_bwd_data_x3(ptr(dz), ptr(planes), B, H, W, D, Cin, Cout, ptr(dx), stream()),
                      "conv3d_bwd_data_x3")
            elif (nsk > 1 and rec is not None and rec.armed and not strided and (OH, OW, OD) == (H, W, D)
                  and not _per_item(B, H * W * D, Cin, OH * OW * OD, cpad) and _fuse_final(link, x, acc)):
                wsk = torch.empty((nsk, M * Cin), device=x.device, dtype=torch.float32)
                dres_f = torch.empty_like(x) if rec.need_res else None
                bws, bwsb = _bn_fuse_ws(rec, B, H, W, D, Cin, x.device)
                d = rec.descriptor(dres_f)
                check(L.m3d_conv3d_bwd_data_splitk_bn(ptr(dzd), ptr(wd), B, H, W, D, Cin, cpad, ptr(dx), acc, nsk,
                                                      ptr(wsk), wsk.numel() * 4, ctypes.addressof(d), ptr(bws),
                                                      bwsb, stream()), "conv3d_bwd_data_splitk_bn")
                rec.buf, rec.dres, rec.done = dx, dres_f, True
                fused_nel = x.numel() * (1 + (rec.z is not None) + rec.need_res)
            elif nsk > 1:
                wsk = torch.empty((nsk, M * Cin), device=x.device, dtype=torch.float32)
                check(L.m3d_conv3d_bwd_data_splitk(ptr(dzd), ptr(wd), B, H, W, D, Cin, cpad, OH, OW, OD,
                                                   *geo.stride, ptr(dx), acc, nsk, ptr(wsk), wsk.numel() * 4,
                                                   stream()), "conv3d_bwd_data_splitk")
            elif (rec is not None and rec.armed and not strided and (OH, OW, OD) == (H, W, D)
                  and not _per_item(B, H * W * D, Cin, OH * OW * OD, cpad) and _fuse_final(link, x, acc)):
                dres_f = torch.empty_like(x) if rec.need_res else None
                bws, bwsb = _bn_fuse_ws(rec, B, H, W, D, Cin, x.device)
                d = rec.descriptor(dres_f)
                check(L.m3d_conv3d_bwd_data_bn(ptr(dzd), ptr(wd), B, H, W, D, Cin, kh, kw, kd, cpad, OH, OW, OD,
                                               *geo.stride, *geo.pad, ptr(dx), acc, ctypes.addressof(d), ptr(bws),
                                               bwsb, stream()), "conv3d_bwd_data_bn")
                rec.buf, rec.dres, rec.done = dx, dres_f, True
                fused_nel = x.numel() * (1 + (rec.z is not None) + rec.need_res)
            else:
                check(L.m3d_conv3d_bwd_data(ptr(dzd), ptr(wd), B, H, W, D, Cin, kh, kw, kd, cpad, OH, OW,
                                            OD, *geo.stride, *geo.pad, ptr(dx), acc, stream()),
                      "conv3d_bwd_data")
            if logging:
                _log(f"conv{kh}_dgrad", direct, direct,
                     4.0 * (dz.numel() + w.numel() + x.numel() * (1 + acc) + fused_nel),
                     "bwd_data", ctx.name, td, "x3" if dx_x3 else "f32")
            dx = _link_park(link, dx, acc)
        if has_w and WGRAD_LAST:
            wgrad_d()
        _grad_done(grads, side)
        dr = None
        if need_res:
            if ctx.res_mode == 1 and link is not None and link.mode == "res" and not trivial:
                link.buf = dres                               # consumed by the input conv's backward
            elif ctx.res_mode == 1:
                dr = dres
            else:
                rb, rh, rw, rd, rc = ctx.res_shape
                tu = _span()
                dr = torch.empty(ctx.res_shape, device=dy.device, dtype=torch.float32)
                check(L.m3d_upsample221_bwd(ptr(dres), rb, rh, rw, rd, rc, ptr(dr), 0, stream()),
                      "upsample221_bwd")
                _log("upsample_bwd", 0, 0, 4.0 * (dres.numel() + dr.numel()), "bwd_data", ctx.name, tu)
        ctx.fuse_in = None
        return dx, dr, None, None, None, None, None, None, None, None, None, None, None, None, None, None


def _stem_halo(geo, cin, cout, res_mode):
    """The one-channel 7^3 stem (core/models.py:242) in the shape whose kernel
    reads halo planes beside a depth slab (m3d_conv3d_fwd_halo)."""
    return (cin == 1 and cout == 64 and geo.k == (7, 7, 7) and geo.stride == (2, 2, 1) and res_mode == 0
            and geo.pad[2] == 3 and geo.out[2] > 0)


def _slab_extend(x, geo):
    """Under depth-slab sharding (m3d.slab.active), give a z-spanning window
    its neighbours' halo planes; z padding stays only where the volume ends."""
    if slab.current() is None or geo.k[2] == 1:
        return x, geo
    r = geo.pad[2]
    if geo.stride[2] != 1 or geo.out[2] != x.shape[3] or 2 * r != geo.k[2] - 1:
        raise ValueError("depth-slab sharding needs z-stride 1 and symmetric 'same' z padding")
    xe, nlo = slab.halo_z(x, r)
    return xe, ConvGeom(geo.k, geo.stride, (geo.pad[0], geo.pad[1], r - nlo), geo.out)


def conv_bn_act(x, layer, geo, relu, residual=None, res_mode=0, bn=None, need_dx=True, link=None,
                wshare=None, fuse=None, fuse_in=None):
    """Functional entry: ``layer`` is a Conv3D parameter group from params.py.
    ``link``: a GradLink shared by the residual conv and the input conv of an
    identity block (see GradLink).  ``wshare``: a dict shared by the calls of
    one kernel within a pass (see _shared_wino_ws).  ``fuse`` / ``fuse_in``:
    this unit's / its producer's BNFuse record (the caller guarantees this unit
    is the producer's sole consumer; see BNFuse)."""
    w = layer.kernel.data
    b = layer.bias.data if layer.bias is not None else None
    grads = layer.grad_dict(bn) if torch.is_grad_enabled() else None   # inference: no z / grads
    if grads is not None and GRAD_HOOK is not None:
        key = layer.name
        GRAD_HOOK.use(key, [t for t in grads.values() if t is not None])
        grads = dict(grads, _hook=(GRAD_HOOK, key))
    bnt = None
    if bn is not None:
        # the model forward's batched affine (ParamStore.bn_affine_refresh) when current
        st = getattr(bn, "store", None)
        aff = bn.aff if st is not None and st.bn_aff_live else None
        bnt = (bn.gamma.data, bn.beta.data, bn.moving_mean, bn.moving_variance, bn.eps, aff,
               (st, st.bn_gen) if aff is not None else None)
    if residual is not None:
        residual = residual.contiguous()
    halo = None
    if (slab.current() is not None and SLAB_HALO_PLANES and res_mode != 2
            and use_winograd(geo, x.shape[-1], w.shape[-1], tuple(x.shape[1:4]))):
        # Winograd convs read the neighbours' planes beside the slab (no extended copy);
        # the exchange overlaps the conv's weight transform and interior z tiles
        halo = (slab.halo_planes_start if SLAB_OVERLAP else slab.halo_planes)(x.contiguous(), 1)
    elif (slab.current() is not None and SLAB_HALO_PLANES and _stem_halo(geo, x.shape[-1], w.shape[-1], res_mode)
          and not (need_dx and x.requires_grad) and x.shape[3] >= geo.pad[2]):
        # the 7^3 stem reads its 3 halo planes per side beside the slab
        halo = slab.halo_planes(x.contiguous(), geo.pad[2])
    else:
        x, geo = _slab_extend(x, geo)
    # the function must see at least one tensor requiring grad to be recorded
    y = _ConvBNAct.apply(x.contiguous(), residual, w, b, bnt, geo, relu, res_mode, grads,
                         need_dx and x.requires_grad, link, halo, wshare, getattr(layer, "name", ""), fuse, fuse_in)
    if RELU_CAPTURE is not None and relu:
        RELU_CAPTURE.setdefault(getattr(layer, "name", ""), []).append((y.detach() > 0).cpu())
    return y


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, stride, pad, out):
        t0 = _span()
        B, H, W, D, C = x.shape
        y = torch.empty((B, *out, C), device=x.device, dtype=torch.float32)
        am = torch.empty((B, *out, C), device=x.device, dtype=torch.uint8)
        check(_L().m3d_maxpool3d_fwd(ptr(x), B, H, W, D, C, *k, *stride, *pad, *out, ptr(y), ptr(am),
                                     stream()), "maxpool3d_fwd")
        _log("maxpool", 0, 0, 4.0 * (x.numel() + y.numel()), "fwd", "pool1", t0)
        ctx.save_for_backward(am)
        ctx.cfg = (tuple(x.shape), k, stride, pad, out)
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        shape, k, stride, pad, out = ctx.cfg
        t0 = _span()
        dx = torch.empty(shape, device=dy.device, dtype=torch.float32)
        check(_L().m3d_maxpool3d_bwd(ptr(dy.contiguous()), ptr(am), *shape, *k, *stride, *pad, *out,
                                     ptr(dx), stream()), "maxpool3d_bwd")
        _log("maxpool_bwd", 0, 0, 4.0 * (dy.numel() + dx.numel()) + am.numel(), "bwd_data", "pool1", t0)
        return dx, None, None, None, None


class _MaxPoolHalo(torch.autograd.Function):
    """Depth-slab max-pool reading the neighbours' halo planes beside the slab
    (m3d_maxpool3d_fwd_halo): no halo-extended copy of the 64-channel C1 slab;
    the backward returns the halo planes' gradient to their owners."""

    @staticmethod
    def forward(ctx, x, halo, k, stride, pad, out):
        t0 = _span()
        hp, has_lo, has_hi = halo
        B, H, W, D, C = x.shape
        r = hp.shape[3] // 2
        y = torch.empty((B, *out, C), device=x.device, dtype=torch.float32)
        am = torch.empty((B, *out, C), device=x.device, dtype=torch.uint8)
        check(_L().m3d_maxpool3d_fwd_halo(ptr(x), ptr(hp), has_lo, has_hi, r, B, H, W, D, C, *k, *stride, *pad,
                                          *out, ptr(y), ptr(am), stream()), "maxpool3d_fwd_halo")
        _log("maxpool", 0, 0, 4.0 * (x.numel() + y.numel()), "fwd", "pool1", t0)
        ctx.save_for_backward(am)
        ctx.cfg = (tuple(x.shape), k, stride, pad, out, has_lo, has_hi, r)
        return y

    @staticmethod
    def backward(ctx, dy):
        (am,) = ctx.saved_tensors
        shape, k, stride, pad, out, has_lo, has_hi, r = ctx.cfg
        t0 = _span()
        B, H, W, D, C = shape
        dx = torch.empty(shape, device=dy.device, dtype=torch.float32)
        dh = torch.empty((B, H, W, 2 * r, C), device=dy.device, dtype=torch.float32)
        check(_L().m3d_maxpool3d_bwd_halo(ptr(dy.contiguous()), ptr(am), has_lo, has_hi, r, *shape, *k, *stride,
                                          *pad, *out, ptr(dx), ptr(dh), stream()), "maxpool3d_bwd_halo")
        _log("maxpool_bwd", 0, 0, 4.0 * (dy.numel() + dx.numel()) + am.numel(), "bwd_data", "pool1", t0)
        slab.return_halo_grads(dx, dh, r)
        return dx, None, None, None, None, None


def max_pool3d(x, k, stride, padding="same"):
    """KL.MaxPooling3D(k, strides, padding) with TF SAME semantics."""
    sp = x.shape[1:4]
    if padding == "same":
        op = [same_out_pad(n, kk, s) for n, kk, s in zip(sp, k, stride)]
        out, pad = tuple(o for o, _ in op), tuple(p for _, p in op)
    else:
        out, pad = tuple(valid_out(n, kk, s) for n, kk, s in zip(sp, k, stride)), (0, 0, 0)
    r = (k[2] - 1) // 2
    if (slab.current() is not None and SLAB_HALO_PLANES and k[2] > 1 and stride[2] == 1 and pad[2] == r
            and 2 * r + 1 == k[2] and x.shape[-1] % 4 == 0 and x.shape[3] >= r):
        # the neighbours' planes beside the slab (no extended copy of C1)
        xc = x.contiguous()
        return _MaxPoolHalo.apply(xc, slab.halo_planes(xc, r), tuple(k), tuple(stride), pad, out)
    x, geo = _slab_extend(x.contiguous(), ConvGeom(tuple(k), tuple(stride), pad, out))
    return _MaxPool.apply(x.contiguous(), tuple(k), tuple(stride), geo.pad, out)


class _Subsample221(torch.autograd.Function):
    """P6 = MaxPooling3D(pool_size=(1,1,1), strides=(2,2,1)) (core/models.py:3211)."""

    @staticmethod
    def forward(ctx, x):
        t0 = _span()
        B, H, W, D, C = x.shape
        y = torch.empty((B, (H + 1) // 2, (W + 1) // 2, D, C), device=x.device, dtype=torch.float32)
        check(_L().m3d_subsample221_fwd(ptr(x), B, H, W, D, C, ptr(y), stream()), "subsample221")
        _log("subsample", 0, 0, 4.0 * (x.numel() + y.numel()), "fwd", "fpn_p6", t0)
        ctx.shape = tuple(x.shape)
        return y

    @staticmethod
    def backward(ctx, dy):
        t0 = _span()
        dx = torch.zeros(ctx.shape, device=dy.device, dtype=torch.float32)
        check(_L().m3d_subsample221_bwd(ptr(dy.contiguous()), *ctx.shape, ptr(dx), stream()),
              "subsample221_bwd")
        _log("subsample_bwd", 0, 0, 4.0 * (dy.numel() + dx.numel()), "bwd_data", "fpn_p6", t0)
        return dx


def subsample221(x):
    return _Subsample221.apply(x.contiguous())


# False keeps the RPN class/bbox heads' weight gradient on the compute stream (A/B)
RPN_OUT_SIDE = True


def _rpn_out_wgrad(L, side, xb, dz, H, W, D, Cin, npad, grads):
    with torch.cuda.stream(side) if side is not None else contextlib.nullcontext():
        check(L.m3d_conv3d_bwd_weight(ptr(xb), ptr(dz), 1, H, W, D, Cin, 1, 1, 1, npad, H,
                                      W, D, 1, 1, 1, 0, 0, 0, ptr(grads["kernel"]),
                                      stream()), "rpn_out_wgrad")


class _RPNOut(torch.autograd.Function):
    """The RPN class/bbox 1x1x1 heads (rpn_class_raw, rpn_bbox_pred;
    core/models.py:540-556) of all pyramid levels in one function.  Each level's
    conv writes its rows straight into the level-concatenated outputs
    rpn_class_logits [B,A,2] / rpn_bbox [B,A,6] (core/models.py:3250-3263)."""

    @staticmethod
    def forward(ctx, w24, b24, grads, apl, fuses, *shared):
        """``fuses``: per level, the BNFuse of the rpn_conv_shared2 unit that
        made ``shared[level]`` (this head is its only consumer) or None."""
        t0 = _span()
        dev = shared[0].device
        B = shared[0].shape[0]
        rows = [s.shape[1] * s.shape[2] * s.shape[3] for s in shared]
        A = sum(rows) * apl
        logits = torch.empty((B, A, 2), device=dev, dtype=torch.float32)
        bbox = torch.empty((B, A, 6), device=dev, dtype=torch.float32)
        Cin = shared[0].shape[-1]
        L = _L()
        for b in range(B):
            off = 0
            for s, r in zip(shared, rows):
                xb = s[b:b + 1]
                _, H, W, D, _ = xb.shape
                check(L.m3d_conv3d_fwd(ptr(xb), 1, H, W, D, Cin, ptr(w24), 1, 1, 1, 8 * apl, H, W, D,
                                       1, 1, 1, 0, 0, 0, ptr(b24), None, None, None, 0, 0, None,
                                       logits[b].data_ptr() + off * apl * 2 * 4, 2 * apl,
                                       bbox[b].data_ptr() + off * apl * 6 * 4, 6 * apl, 2 * apl,
                                       stream()), "rpn_out_fwd")
                off += r
        if LAYER_LOG is not None:
            f = 2.0 * B * sum(rows) * Cin * 8 * apl
            _log("conv1", f, f, 4.0 * (sum(s.numel() for s in shared) + w24.numel() + logits.numel() + bbox.numel()),
                 "fwd", "rpn_class_raw+rpn_bbox_pred", t0)
        ctx.save_for_backward(w24, *shared)
        ctx.grads, ctx.rows, ctx.apl = grads, rows, apl
        ctx.bias_batch = BIAS_BATCH if grads is not None else None
        ctx.fuses = [f if (f is not None and f.armed and f.y is not None and f.y.data_ptr() == s.data_ptr()
                           and f.y.shape == s.shape) else None
                     for f, s in zip(fuses or [None] * len(shared), shared)]
        return logits, bbox

    @staticmethod
    def backward(ctx, dlogits, dbbox):
        w24, *shared = ctx.saved_tensors
        apl, rows, grads = ctx.apl, ctx.rows, ctx.grads or {}
        B = shared[0].shape[0]
        Cin = shared[0].shape[-1]
        n_out = 8 * apl
        npad = -(-n_out // 32) * 32
        dev = shared[0].device
        if dlogits is None:
            dlogits = torch.zeros((B, sum(rows) * apl, 2), device=dev)
        if dbbox is None:
            dbbox = torch.zeros((B, sum(rows) * apl, 6), device=dev)
        t0 = _span()
        w_pad = torch.nn.functional.pad(w24.reshape(Cin, n_out), (0, npad - n_out))
        dshared = [torch.empty_like(s) for s in shared]
        L = _L()
        R = sum(rows)
        fuses = ctx.fuses
        ctx.fuses = None
        fws = [None] * len(shared)
        for li, rec in enumerate(fuses):
            if rec is not None and not _per_item(1, rows[li], Cin, rows[li], npad):
                _, H, W, D, _ = shared[li].shape
                fws[li] = (torch.empty_like(shared[li]) if rec.need_res else None,
                           *_bn_fuse_ws(rec, 1, H, W, D, Cin, dev))
        for b in range(B):
            # all levels' output gradients as one [R, npad] matrix (row = voxel,
            # level-concatenated like the outputs): one cat + one pad instead of
            # a zero fill and two slice copies per level
            dz_all = torch.nn.functional.pad(
                torch.cat([dlogits[b].reshape(R, 2 * apl), dbbox[b].reshape(R, 6 * apl)], dim=1),
                (0, npad - n_out))
            if grads.get("bias") is not None:
                # all levels' rows at once (one column sum of the level-concatenated matrix)
                bias_grad(dz_all, R, npad, grads["bias"], grads,
                          ctx.bias_batch if "rpn" in BIAS_BATCH_UNITS.split("+") else None)
            off = 0
            for li, (s, r) in enumerate(zip(shared, rows)):
                xb = s[b:b + 1]
                _, H, W, D, _ = xb.shape
                dz = dz_all[off:off + r]
                side = None
                if grads.get("kernel") is not None:
                    # on the weight-gradient stream like every conv unit's (joined before the
                    # update); the data gradients below do not wait for it
                    side = _wgrad_stream(dev) if RPN_OUT_SIDE else None
                    if side is not None:
                        dz_all.record_stream(side)
                        s.record_stream(side)
                    if not WGRAD_LAST:
                        _rpn_out_wgrad(L, side, xb, dz, H, W, D, Cin, npad, grads)
                if fws[li] is not None:
                    # rpn_conv_shared2's ReLU backward (and bias sums) in this data gradient's epilogue
                    dres_f, bws, bwsb = fws[li]
                    d = fuses[li].descriptor(dres_f, b)
                    check(L.m3d_conv3d_bwd_data_bn(ptr(dz), ptr(w_pad), 1, H, W, D, Cin, 1, 1, 1, npad, H, W, D,
                                                   1, 1, 1, 0, 0, 0, dshared[li][b:b + 1].data_ptr(), 0,
                                                   ctypes.addressof(d), ptr(bws), bwsb, stream()), "rpn_out_dgrad_bn")
                else:
                    check(L.m3d_conv3d_bwd_data(ptr(dz), ptr(w_pad), 1, H, W, D, Cin, 1, 1, 1, npad, H,
                                                W, D, 1, 1, 1, 0, 0, 0, dshared[li][b:b + 1].data_ptr(),
                                                0, stream()), "rpn_out_dgrad")
                if grads.get("kernel") is not None and WGRAD_LAST:
                    _rpn_out_wgrad(L, side, xb, dz, H, W, D, Cin, npad, grads)
                off += r
        for li, rec in enumerate(fuses):
            if fws[li] is not None:
                rec.buf, rec.dres, rec.done = dshared[li], fws[li][0], True
        if LAYER_LOG is not None:
            f = 2.0 * B * R * Cin * n_out
            nx = sum(s.numel() for s in shared)
            _log("conv1_bwd", 2 * f, 2 * f, 4.0 * (2 * nx + 2 * B * R * npad + 2 * w24.numel()), "bwd_data",
                 "rpn_class_raw+rpn_bbox_pred (wgrad+dgrad)", t0)
        return (None, None, None, None, None) + tuple(dshared)
