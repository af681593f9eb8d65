"""Benchmark: volumes/sec of the RPN training step (backbone + FPN + RPN head
fwd/bwd + SGD + ProposalLayer with 3-D NMS) on synthetic 128^3 volumes
(BASELINE.json configs[1]), one process per GPU (weak scaling, data parallel
over RCCL), plus the 3-D PyramidROIAlign HBM roofline (configs[2] shapes).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--size 128]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "3d-mask-r-cnn_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "volumes/sec fwd+bwd @128³ & 256³, 1/2/4/8 MI355X; 3D ROIAlign GB/s vs HBM peak"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
F32_MFMA_PEAK_TFLOPS = 157.3   # v_mfma_f32_32x32x2_f32 dense peak (MI355X_MICROARCH.md)
# bf16 MFMA dense peak: 256 CUs x 4 SIMDs x 1024 FLOP/clk (v_mfma_f32_32x32x16_bf16,
# 32 cycles) x 2.4 GHz; the X3 kernels run 6 of them per fp32 product, so their
# fp32-FLOP ceiling is a sixth of it
BF16_MFMA_PEAK_TFLOPS = 2516.6
X3_PEAK_TFLOPS = round(BF16_MFMA_PEAK_TFLOPS / 6, 1)
# the step's largest kernel by time in the rocprof table of this tree
# (profiles/dominant_kernel_table.txt, line 1): the headline `roofline` prices
# its largest launch.  Round 5's interleaved MFMA chains (x3_mac_pair) took the
# weight-gradient GEMM below the Winograd point GEMM (profiles/r05prof2_*:
# x3_gemm256_af_kernel 6.92, x3_wgrad_tr_kernel 6.43 ms per step); the other is
# reported beside it (roofline.wgrad_gemm)
DOMINANT_KERNEL = "x3_gemm256_af_kernel"


class LegWatchdog:
    """Bounds a multi-rank leg whose collectives have no timeout of their own:
    if the leg is still running after `seconds`, rank 0 prints the result line
    gathered so far (the leg reported as timed out) and every rank leaves with
    status 3: one hung leg cannot cost the bench line of the whole run, and
    the hang stays visible to the launcher (the legs after it are missing)."""

    def __init__(self, seconds, rank, out, key):
        import threading
        self.rank, self.out, self.key = rank, out, key
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True

    def _fire(self):
        if self.rank == 0:
            self.out[self.key] = {"error": "timeout: the leg did not finish (watchdog)"}
            print(json.dumps(self.out), flush=True)
        log(f"[bench] watchdog: {self.key} timed out on rank {self.rank}, exiting with status 3")
        os._exit(3)

    def __enter__(self):
        self.timer.start()
        return self

    def __exit__(self, *exc):
        self.timer.cancel()
        return False


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------- dominant kernel
def _event_time(fn, reps):
    """Average seconds per call of fn(), HIP events on torch's current stream
    (the stream every libm3d launch of fn() is enqueued on).  The priced GEMM
    legs take 20 launches, as their rocprofv3 runs (scripts/kernels_for_pmc.py)
    do: with 5 the average sat 5-9 % above rocprof's on the same box."""
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps / 1e3


def _pmc_traffic(kernel_key):
    """HBM bytes per launch of the same launch, measured by rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes (scripts/gpu_prof.sh, gfx950 FETCH x2
    correction) and committed under profiles/; None if not measured."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        return json.load(open(path)).get(kernel_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def wgrad_gemm_shape(S):
    """The largest launch of the step's dominant kernel, x3_wgrad_tr_kernel: the
    (NY+2)*4*(NZ+2) batched Winograd weight-gradient GEMMs of rpn_conv_shared1
    (3x3x3, 256->512) on P2 [S/4, S/4, S] -- the (NY+2)*4*(NZ+2) point GEMMs of
    the weight gradient's tile (m3d_conv3d_wino_wgrad_tile_z / _tile_y; 144 for
    F(4x2x4)) on the forward's kept U, reduction over M = T tiles, K = 256,
    N = 512."""
    from m3d import _lib
    nz = int(_lib.load().m3d_conv3d_wino_wgrad_tile_z())
    ny = int(_lib.load().m3d_conv3d_wino_tile_y())
    q = S // 4
    T = ((q + ny - 1) // ny) * ((q + 1) // 2) * ((S + nz - 1) // nz)
    return (ny + 2) * 4 * (nz + 2), T, 256, 512


def wino_gemm_shape(S):
    """The largest launch of x3_gemm256_af_kernel (the step's second kernel by
    time since round 4, profiles/dominant_kernel_table.txt): the
    (NY+2)*4*(NZ+2) batched Winograd point GEMMs of rpn_conv_shared1 (3x3x3,
    256->512) on P2 [S/4, S/4, S]: M = T = 2x2xNZ output tiles, K = 256,
    N = 512 (NZ = 4 by default: 96 GEMMs)."""
    from m3d import _lib
    nz = int(_lib.load().m3d_conv3d_wino_tile_z())
    ny = int(_lib.load().m3d_conv3d_wino_tile_y())
    q = S // 4
    T = ((q + ny - 1) // ny) * ((q + 1) // 2) * ((S + nz - 1) // nz)
    return (ny + 2) * 4 * (nz + 2), T, 256, 512


def time_wino_gemm(S, reps=20):
    """The Winograd point GEMMs of rpn_conv_shared1 on P2 in the form the step
    runs them (M3D_GEMM_X3 bit 4): U in fp32 split inside x3_gemm256_af_kernel,
    the weight planes split once, untimed, as the weight transform does in the
    step (m3d_gemm_x3_af)."""
    from m3d import _lib
    L = _lib.load()
    nb, T, K, N = wino_gemm_shape(S)
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn((nb, T, K), device="cuda", generator=g)
    Bt = torch.randn((nb, N, K), device="cuda", generator=g) * 0.05
    B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device="cuda")
    _lib.check(L.m3d_split3_f32(Bt.data_ptr(), Bt.numel(), B3.data_ptr(), _lib.stream()), "split3")
    del Bt
    C = torch.empty((nb, T, N), device="cuda")

    def launch():
        _lib.check(L.m3d_gemm_x3_af(A.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, T, K, N, _lib.stream()),
                   "gemm_x3_af")
    t = _event_time(launch, reps)
    flops = 2.0 * nb * T * K * N
    key = f"wino_gemm_x3af_rpn_shared1_S{S}"
    return {"bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": X3_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(flops / t / 1e12 / X3_PEAK_TFLOPS, 4),
            "traffic": _pmc_traffic(key),
            "kernel": f"x3_gemm256_af_kernel (fp32 GEMM as 6 bf16 MFMAs per product on the exact 3-way split, "
                      f"A in fp32 split in registers): "
                      f"{nb} batched Winograd point GEMMs of rpn_conv_shared1 on P2, M={T} K={K} N={N}",
            "peak_note": "bf16 MFMA dense peak 2516.6 TFLOP/s / 6; achieved counts fp32 FLOPs 2*M*K*N",
            "f32_mfma_peak_frac": round(flops / t / 1e12 / F32_MFMA_PEAK_TFLOPS, 4),
            "flop_per_launch": flops, "avg_launch_ms": round(t * 1e3, 4),
            "algorithmic_bytes_per_launch": nb * (4.0 * T * K + 6.0 * N * K + 4.0 * T * N),
            "direct_conv_equivalent_tflops": round(2.0 * (S // 4) ** 2 * S * 27 * K * N / t / 1e12, 2)}


def time_wgrad_gemm(S, reps=20):
    """The Winograd weight-gradient GEMMs of rpn_conv_shared1 on P2 through
    m3d_gemm_wgrad_f32 (x3_wgrad_tr_kernel by default)."""
    from m3d import _lib
    L = _lib.load()
    nb, T, K, N = wgrad_gemm_shape(S)
    g = torch.Generator(device="cuda").manual_seed(5)
    A = torch.randn((nb, T, K), device="cuda", generator=g)
    Bm = torch.randn((nb, T, N), device="cuda", generator=g) * 0.05
    C = torch.zeros((nb, K, N), device="cuda")

    def launch():
        _lib.check(L.m3d_gemm_wgrad_f32(A.data_ptr(), Bm.data_ptr(), C.data_ptr(), nb, T, K, N,
                                        _lib.stream()), "gemm_wgrad")
    t = _event_time(launch, reps)
    flops = 2.0 * nb * T * K * N
    return {"bound": "mfma", "achieved": round(flops / t / 1e12, 2), "peak": X3_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": round(flops / t / 1e12 / X3_PEAK_TFLOPS, 4),
            "traffic": _pmc_traffic(f"wino_wgrad_gemm_rpn_shared1_S{S}"),
            "traffic_note": "HBM bytes per launch from rocprofv3 FETCH_SIZE x2 + WRITE_SIZE passes "
                            "(scripts/gpu_prof.sh -> profiles/traffic.json)",
            "kernel": f"x3_wgrad_tr_kernel (fp32 GEMM as 6 bf16 MFMAs per product, 256x256 tiles, operands "
                      f"split in the LDS store): {nb} batched Winograd weight-gradient GEMMs of rpn_conv_shared1 on P2, "
                      f"C[K][N] += A[M][K]^T B[M][N], M={T} K={K} N={N}",
            "peak_note": "bf16 MFMA dense peak 2516.6 TFLOP/s / 6; achieved counts fp32 FLOPs 2*M*K*N",
            "f32_mfma_peak_frac": round(flops / t / 1e12 / F32_MFMA_PEAK_TFLOPS, 4),
            "flop_per_launch": flops, "avg_launch_ms": round(t * 1e3, 4),
            "algorithmic_bytes_per_launch": nb * (4.0 * T * (K + N) + 4.0 * K * N),
            "shape": f"{nb} x (M={T}) K={K} N={N}"}


def time_wino_fwd(S, reps=5):
    """rpn_conv_shared1 (3x3x3, 256->512) on P2 as the whole F(2x2x4) Winograd
    forward (weight + input transforms, 96 point GEMMs on the exact bf16 split
    (x3_gemm_kernel), output transform): time and direct-conv-equivalent rate."""
    from m3d import _lib
    L = _lib.load()
    B, H, W, D, Cin, Cout = 1, S // 4, S // 4, S, 256, 512
    g = torch.Generator(device="cuda").manual_seed(6)
    x = torch.randn((B, H, W, D, Cin), device="cuda", generator=g)
    w = torch.randn((3, 3, 3, Cin, Cout), device="cuda", generator=g) / (27 * Cin) ** 0.5
    y = torch.empty((B, H, W, D, Cout), device="cuda")
    nb = L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, Cin, Cout)
    ws = torch.empty(nb // 4 + 64, device="cuda")

    def launch():
        _lib.check(L.m3d_conv3d_fwd_wino(x.data_ptr(), B, H, W, D, Cin, w.data_ptr(), Cout, D, 1, None, None,
                                         None, None, 0, None, y.data_ptr(), ws.data_ptr(), nb, _lib.stream()),
                   "wino fwd")
    t = _event_time(launch, reps)
    nz = int(L.m3d_conv3d_wino_tile_z())
    ny = int(L.m3d_conv3d_wino_tile_y())
    T = ((H + ny - 1) // ny) * ((W + 1) // 2) * ((D + nz - 1) // nz)
    return {"ms": round(t * 1e3, 4),
            "gemm_tflops": round(2.0 * (ny + 2) * 4 * (nz + 2) * T * Cin * Cout / t / 1e12, 2),
            "direct_conv_equivalent_tflops": round(2.0 * H * W * D * 27 * Cin * Cout / t / 1e12, 2)}


def time_direct_conv(model, fmaps, reps=5):
    """rpn_conv_shared1 (3x3x3, 256->512) on P2 as the direct implicit GEMM."""
    from m3d import _lib
    from m3d.nn import conv_geom
    L = _lib.load()
    p2 = fmaps[0].detach().contiguous()
    B, H, W, D, C = p2.shape
    layer = model.rpn.shared1
    geo = conv_geom((H, W, D), (3, 3, 3), (1, 1, 1), "same")
    y = torch.empty((B, H, W, D, 512), device=p2.device)

    def launch():
        _lib.check(L.m3d_conv3d_fwd(p2.data_ptr(), B, H, W, D, C, layer.kernel.data.data_ptr(), 3, 3, 3,
                                    512, H, W, D, 1, 1, 1, *geo.pad, layer.bias.data.data_ptr(), None,
                                    None, None, 0, 1, None, y.data_ptr(), 512, None, 0, 0,
                                    _lib.stream()), "conv")
    t = _event_time(launch, reps)
    flops = 2.0 * B * H * W * D * 27 * C * 512
    return {"achieved": round(flops / t / 1e12, 2), "unit": "TFLOP/s",
            "frac": round(flops / t / 1e12 / F32_MFMA_PEAK_TFLOPS, 4), "avg_launch_ms": round(t * 1e3, 4),
            "traffic": _pmc_traffic(f"direct_conv_rpn_shared1_S{model.config.IMAGE_SHAPE[0]}")}


# ---------------------------------------------------------------- ROIAlign roofline
def roi_boxes(n, S, seed=3, hi=128):
    """n ROIs with log-uniform cube-root pixel volume in [24, hi]."""
    rng = np.random.default_rng(seed)
    side = np.exp(rng.uniform(np.log(24), np.log(hi), n))
    asp = np.exp(rng.uniform(-0.3, 0.3, (n, 3)))
    ext = side[:, None] * asp / S
    ext = np.minimum(ext, 0.95)
    lo = rng.uniform(0, 1, (n, 3)) * (1 - ext)
    return np.concatenate([lo, lo + ext], 1).astype(np.float32)[None]


def unique_voxels(boxes, fshapes, pool, S):
    """|U|: distinct input voxels touched by all 8-corner samples (host, exact float32 maths)."""
    from oracle import ops_ref as R
    bx, lvl = R.roi_prepare(boxes[0], (S, S, S))
    keys, off = [], 0
    for li in range(4):
        sel = np.nonzero(lvl == li + 2)[0]
        H, W, D = fshapes[li]
        base, off = off, off + H * W * D
        for b in bx[sel]:
            coords = []
            for ax, (n, Sz) in enumerate(zip(pool, (H, W, D))):
                b1, b2 = np.float32(b[ax]), np.float32(b[ax + 3])
                sc = np.float32((b2 - b1) * np.float32(Sz - 1)) / np.float32(n - 1)
                c = np.float32(b1 * np.float32(Sz - 1)) + np.arange(n, dtype=np.float32) * sc
                coords.append(np.unique(np.concatenate([np.floor(c), np.ceil(c)]).astype(np.int64)))
            g = np.meshgrid(*coords, indexing="ij")
            keys.append(base + ((g[0] * W + g[1]) * D + g[2]).ravel())
    return int(np.unique(np.concatenate(keys)).size) if keys else 0


def time_roi_align(fmaps, S, n_rois=128, reps=10, pools=(7, 14), hi=128):
    from m3d import layers
    maps = [f.detach().contiguous() for f in fmaps[:4]]
    C = maps[0].shape[-1]
    boxes = torch.from_numpy(roi_boxes(n_rois, S, hi=hi)).to(maps[0].device)
    meta = torch.zeros((1, 18), device=maps[0].device)
    meta[0, 5:8] = S
    res = {}
    fshapes = [tuple(m.shape[1:4]) for m in maps]
    for p in pools:
        layer = layers.PyramidROIAlign((p, p, p))
        layer([boxes, meta] + maps)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            layer([boxes, meta] + maps)
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / reps / 1e3
        bnp = boxes.cpu().numpy()
        u = unique_voxels(bnp, fshapes, (p, p, p), S)
        alg = 4.0 * n_rois * p ** 3 * C + 4.0 * C * u
        # per-ROI bound: sum over ROIs of each ROI's own unique voxels (what any
        # kernel that does not share rows between different ROIs must read)
        u_roi = sum(unique_voxels(bnp[:, i:i + 1], fshapes, (p, p, p), S) for i in range(n_rois))
        per_roi = 4.0 * n_rois * p ** 3 * C + 4.0 * C * u_roi
        res[f"pool{p}"] = {"ms": round(t * 1e3, 4), "algorithmic_bytes": alg,
                           "gather_bytes": 8 * 4.0 * n_rois * p ** 3 * C,
                           "GBps": round(alg / t / 1e9, 1), "frac_hbm": round(alg / t / 1e9 / HBM_PEAK_GBS, 4),
                           "per_roi_bytes": per_roi,
                           "frac_hbm_per_roi": round(per_roi / t / 1e9 / HBM_PEAK_GBS, 4),
                           "traffic": _pmc_traffic(f"pyramid_fwd_pool{p}_S{S}_N{n_rois}")}
    return res


def time_roi_align_bwd(fmaps, S, n_rois=128, reps=5, pools=(7, 14), hi=128):
    """CropAndResize3DGradImage through PyramidROIAlign's backward (SURVEY.md 8d:
    HBM / atomics): bytes = 4|grads| (read) + 32|grads| (8 corner atomic RMW)
    + 4|P2..P5| (zero fill of the image gradients)."""
    from m3d import _lib, ops
    L = _lib.load()
    maps = [f.detach().contiguous() for f in fmaps[:4]]
    C = maps[0].shape[-1]
    boxes = torch.from_numpy(roi_boxes(n_rois, S, hi=hi)).to(maps[0].device)
    meta = torch.zeros((1, 18), device=maps[0].device)
    meta[0, 5:8] = S
    gm = [torch.empty_like(m) for m in maps]
    gptrs = (_lib.c_p * 4)(*[g.data_ptr() for g in gm])
    fshape = ((_lib.c_i64 * 3) * 4)(*[(_lib.c_i64 * 3)(*m.shape[1:4]) for m in maps])
    img = sum(m.numel() for m in maps)
    res = {}
    for p in pools:
        _, badj, lev = ops.pyramid_roi_align(boxes, meta, maps, (p, p, p), return_levels=True)
        grad = torch.randn((1, n_rois, p, p, p, C), device=maps[0].device)

        def launch():
            _lib.check(L.m3d_pyramid_roi_align3d_bwd(grad.data_ptr(), badj.data_ptr(), lev.data_ptr(), 1, n_rois,
                                                     p, p, p, gptrs, fshape, C, _lib.stream()), "roi bwd")
        t = _event_time(launch, reps)
        nb = 4.0 * grad.numel() * (1 + 8) + 4.0 * img
        rows = touched_voxel_rows(badj.cpu().numpy().reshape(-1, 6), lev.cpu().numpy().reshape(-1),
                                  [m.shape[1:4] for m in maps], p)
        # minimal traffic of the backward: read the gradient once, zero-fill the
        # image gradients once, read-modify-write each touched voxel row once
        # per ROI (8 B per channel)
        nmin = 4.0 * grad.numel() + 4.0 * img + 8.0 * C * rows
        res[f"pool{p}"] = {"ms": round(t * 1e3, 4), "bytes": nmin, "GBps": round(nmin / t / 1e9, 1),
                           "frac_hbm": round(nmin / t / 1e9 / HBM_PEAK_GBS, 4),
                           "touched_voxel_rows": int(rows),
                           "scatter_bytes": nb, "scatter_frac_hbm": round(nb / t / 1e9 / HBM_PEAK_GBS, 4),
                           "note": "bytes = 4|grads| + 4|P2..P5| + 8*C*touched voxel rows (per ROI); "
                                   "scatter_bytes = the per-sample 8-corner atomic form (4|grads| + 32|grads| "
                                   "+ 4|P2..P5|)"}
        # CropAndResize3DGradImage itself (the op the TF binding calls) on P2 with
        # all the ROIs: fast (atomic) mode vs deterministic mode 1 (destination-
        # owned sums in the reference's order, bit-identical to the wheel)
        g0 = grad[0].contiguous()
        bi = torch.zeros(n_rois, dtype=torch.int32, device=g0.device)
        bx = badj.reshape(-1, 6).contiguous()
        shape2 = tuple(maps[0].shape)
        tf = _event_time(lambda: ops.crop_and_resize_3d_grad_image(g0, bx, bi, shape2, deterministic=0), reps)
        td = _event_time(lambda: ops.crop_and_resize_3d_grad_image(g0, bx, bi, shape2, deterministic=1), reps)
        res[f"pool{p}"]["crop_grad_image_P2"] = {
            "fast_atomic_ms": round(tf * 1e3, 4), "deterministic_ms": round(td * 1e3, 4),
            "note": f"CropAndResize3DGradImage of {n_rois} ROIs x {p}^3 x C={C} into P2 {list(shape2)}; "
                    "deterministic = mode 1 (bit-identical to the reference's sequential scatter)"}
    return res


def touched_voxel_rows(boxes, levels, shapes, p):
    """Sum over ROIs of the distinct feature-map voxels the trilinear backward
    of a p^3 crop touches (per axis the floor/ceil corners of the in-bounds
    samples, the float32 coordinate maths of SURVEY.md A.1; a box's voxel set
    is the product of its three axis sets)."""
    total = 0
    f32 = np.float32
    for b, lv in zip(boxes.astype(np.float32), levels):
        H, W, D = shapes[int(lv) - 2]
        n = 1
        for ax, S in enumerate((H, W, D)):
            b1, b2 = f32(b[ax]), f32(b[ax + 3])
            i = np.arange(p, dtype=np.float32)
            if p > 1:
                sc = f32(f32(f32(b2 - b1) * f32(S - 1)) / f32(p - 1))
                coord = f32(b1 * f32(S - 1)) + i * sc
            else:
                coord = np.full(1, f32(0.5 * float(f32(b1 + b2)) * (S - 1)), np.float32)
            ok = (coord >= 0) & (coord <= S - 1)
            vox = set(np.floor(coord[ok]).astype(int)) | set(np.ceil(coord[ok]).astype(int))
            n *= len(vox)
        total += n
    return total


def time_nms(dev, k=15000, max_out=6000, thr=0.7, reps=5, seed=4):
    """NonMaxSuppression3D at the ProposalLayer's training shape (k = PRE_NMS_LIMIT
    boxes -> POST_NMS_ROIS_TRAINING): latency-bound, reported as ms and IoU
    pairs/s (k(k-1)/2 pairs)."""
    from m3d import ops
    rng = np.random.default_rng(seed)
    c = rng.uniform(0.05, 0.95, (k, 3))
    ext = np.exp(rng.uniform(np.log(0.02), np.log(0.3), (k, 3))) / 2
    boxes = torch.from_numpy(np.concatenate([c - ext, c + ext], 1).astype(np.float32)).to(dev)
    scores = torch.from_numpy(np.sort(rng.uniform(size=k))[::-1].astype(np.float32).copy()).to(dev)
    keep, num = ops.non_max_suppression_3d_padded(boxes, scores, max_out, thr)
    t = _event_time(lambda: ops.non_max_suppression_3d_padded(boxes, scores, max_out, thr), reps)
    pairs = k * (k - 1) / 2
    return {"k": k, "max_output_size": max_out, "iou_threshold": thr, "kept": int(num.item()),
            "ms": round(t * 1e3, 4), "pairs_per_s": round(pairs / t, 1)}


def time_allreduce(flat, world, reps=3):
    """Bucketed gradient all-reduce alone (RCCL over xGMI): ms and bus bandwidth
    2(n-1)/n * bytes / t."""
    from m3d.parallel import allreduce_mean_
    buf = flat.clone()
    dist.barrier()
    t = _event_time(lambda: allreduce_mean_(buf, world), reps)
    nb = buf.numel() * buf.element_size()
    t_max = torch.tensor([t], device=flat.device, dtype=torch.float64)
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    t = float(t_max.item())
    return {"bytes": nb, "ms": round(t * 1e3, 3), "bus_GBps": round(2 * (world - 1) / world * nb / t / 1e9, 1)}


# ---------------------------------------------------------------- depth-slab leg
def targets_in_step_leg(model, image, steps, warmup, dev, n_gt=8, seed=11):
    """The configs[1] step with its RPN targets built on the GPU every
    iteration (core/data_generators.py:986 calls build_rpn_targets per volume):
    m3d.targets.RPNTargetBuilder (ATSS labels, balancing, deltas; stream-ordered,
    no host round trip) from seeded GT boxes, then the same training step.
    Reports the step time, the builder alone, and the positives it found."""
    from m3d.targets import RPNTargetBuilder
    S = image.shape[1]
    rng = np.random.default_rng(seed)
    side = rng.uniform(12, 40, (n_gt, 3)) / S
    lo = rng.uniform(0, 1, (n_gt, 3)) * (1 - side)
    gt = torch.from_numpy(np.concatenate([lo, lo + side], 1).astype(np.float32)).to(dev)
    builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), model.config, max_gt=n_gt)
    for i in range(warmup):
        model.train_step(image, builder(gt, seed=i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        r = model.train_step(image, builder(gt, seed=1000 + i))
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / steps
    el, r = _graphed_targets_steps(model, image, builder, gt, steps, warmup, 1000)
    tb = _event_time(lambda: builder(gt, seed=7), 5)
    cnt = builder.counts.cpu().tolist()
    return {"workload": f"configs[1] step with GPU-built RPN targets ({n_gt} GT boxes, ATSS), {S}^3; "
                        f"builder launched before each replay of the step's HIP graph",
            "ms_per_step": round(el * 1e3, 2), "volumes_per_s": round(1.0 / el, 4),
            "eager_ms_per_step": round(eager * 1e3, 2),
            "builder_ms": round(tb * 1e3, 3), "positives": cnt[0], "negatives": cnt[1],
            "loss": round(float(r["loss"]), 5)}


def _graphed_targets_steps(model, image, builder, gt, steps, warmup, seed0):
    """The training step replayed from a HIP graph with the RPN targets built
    on the GPU right before every replay: the builder (RPNTargetBuilder, ~40
    stream-ordered launches, a new host seed each step) writes its persistent
    rpn_match / rpn_bbox buffers in place, and the graph was captured reading
    those buffers (DeviceRPNTargets).  Seconds per step, last result."""
    targets = builder(gt, seed=seed0 - 1)
    step = model.graphed_train_step(image, targets, warmup=max(warmup, 1))
    for i in range(warmup):
        builder(gt, seed=seed0 - 100 + i)
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        builder(gt, seed=seed0 + i)
        r = step()
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / steps
    model._graph = None
    return el, r


def configs0_leg(dev, steps, warmup, seed=5, S=64):
    """BASELINE configs[0]: RPN training on one synthetic 64^3 toy-shapes
    volume (generate_data.py, restated seeded in m3d.toydata), GT boxes ->
    RPN targets built on the GPU each step (RPNTargetBuilder) -> the training
    step; beside it the same step through the CPU oracle port (targets from
    the numpy restatement oracle/heads_ref.build_rpn_targets)."""
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN
    from m3d.targets import RPNTargetBuilder
    from m3d.toydata import network_input, toy_volume
    from oracle import heads_ref as HR
    v = toy_volume(S, seed=seed)
    cfg = synthetic_rpn_config(S)
    model = RPN(cfg, device=dev, seed=1)
    image = torch.from_numpy(network_input(v["image"])).to(dev)
    gt = (v["boxes"] / np.float32(S)).astype(np.float32)
    builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), cfg, max_gt=32)
    gtd = torch.from_numpy(gt).to(dev)
    for i in range(warmup):
        model.train_step(image, builder(gtd, seed=i))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        r = model.train_step(image, builder(gtd, seed=100 + i))
    torch.cuda.synchronize()
    eager = (time.perf_counter() - t0) / steps
    el, r = _graphed_targets_steps(model, image, builder, gtd, steps, warmup, 100)
    res = {"workload": f"configs[0]: RPN training step on one {S}^3 toy-shapes volume ({len(gt)} objects), "
                       f"GPU-built ATSS targets; builder then the step's HIP-graph replay", "ms_per_step": round(el * 1e3, 2),
           "volumes_per_s": round(1.0 / el, 3), "eager_ms_per_step": round(eager * 1e3, 2),
           "loss": round(float(r["loss"]), 5), "positives": int(builder.counts[0])}
    try:
        anchors = model.anchors.reshape(-1, 6).cpu().numpy()
        rm, rb = HR.build_rpn_targets(anchors, gt, float(cfg.RPN_POSITIVE_IOU), float(cfg.RPN_NEGATIVE_IOU),
                                      int(cfg.RPN_TRAIN_ANCHORS_PER_IMAGE), float(getattr(cfg, "RPN_POSITIVE_RATIO", 0.5)),
                                      int(cfg.ATSS_TOPK), int(cfg.ATSS_MIN_POS_PER_GT), cfg.RPN_BBOX_STD_DEV, 7)
        res["cpu_baseline"] = cpu_baseline(model, S, (rm.reshape(1, -1, 1), rb[None]))
    except Exception as e:  # report, never hide
        res["cpu_baseline"] = {"error": repr(e)}
    del model
    torch.cuda.empty_cache()
    return res


def depth_slab_leg(S, steps, warmup, rank, world, dev, proposals=True):
    """BASELINE configs[4]: ONE S^3 volume per step, split into depth slabs over
    all ranks (halo exchange + SUM gradient all-reduce over RCCL, merged
    proposals); strong scaling -- the total work is fixed as N grows."""
    from m3d import slab
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_rpn_targets, synthetic_volume
    from m3d.parallel import SlabRPN
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)      # peak_mem_gb is this leg's own
    cfg = synthetic_rpn_config(S)
    model = RPN(cfg, device=dev, seed=1)
    sg = slab.SlabGroup(S, rank, world)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=2)
    srpn = SlabRPN(model, sg, match, bbox)
    vol = synthetic_volume(S, seed=100)
    image = srpn.slice(vol).to(dev)
    validation = None
    if world > 1:
        validation = validate_slab(srpn, image, vol, cfg, match, bbox, rank, dev, proposals)
    del vol
    for _ in range(warmup):
        r = srpn.train_step(image, proposals=proposals)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        r = srpn.train_step(image, proposals=proposals)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    out = {"workload": f"configs[4]: RPN training step on ONE {S}^3 volume depth-slab sharded over "
                       f"{world} GPU(s) ({sg.Dl} planes/rank), halo exchange + grad all-reduce over RCCL",
           "size": S, "n_gpus": world, "steps": steps, "ms_per_step": round(el / steps * 1e3, 2),
           "volumes_per_s": round(steps / el, 4), "scaling": "strong",
           "loss": round(float(r["loss"]), 6),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)}
    if validation is not None:
        from m3d.parallel import validate_replicas
        after = validate_replicas({"weights": model.store.flat})
        validation["weights_after_steps_identical"] = after["ok"]
        validation["ok"] = bool(validation["ok"] and after["ok"])
        out["validation"] = validation
        log(f"[bench] depth_slab validation: {json.dumps(validation)}")
    if world == 1:
        try:
            out["step_roofline"] = step_roofline(model, lambda: srpn.train_step(image, proposals=proposals),
                                                 el / steps * 1e3, os.environ.get("M3D_STEP_ROOFLINE_TABLE_256"))
        except Exception as e:  # report, never hide
            out["step_roofline"] = {"error": repr(e)}
    del model, srpn, image
    from m3d import nn as mnn
    mnn.release_wino_arena()
    torch.cuda.empty_cache()
    return out


def validate_slab(srpn, image, vol, cfg, match, bbox, rank, dev, proposals):
    """First multi-rank depth-slab step, checked before timing (nothing in it
    is timed): one sharded forward + backward without the optimizer; every
    rank must hold bit-identical merged proposals and all-reduced loss, and
    rank 0 reruns the UNSHARDED forward + loss of the same volume on its GPU
    (the N = 1 path): the proposals must be bit-identical (the slab forward is
    exact: same Winograd tiles, halo planes beside the slab) and the loss equal
    within the fp32 summation-order tolerance 1e-5 (per-slab partial sums)."""
    from m3d.model import RPN, RPNTargets
    from m3d.parallel import rel_close, validate_replicas
    r = srpn.train_step(image, proposals=proposals, apply=False)
    torch.cuda.synchronize()
    named = {"loss": r["loss"]}
    if proposals:
        named["rpn_rois"] = r["rpn_rois"]
    v = validate_replicas(named)
    v["loss"] = float(r["loss"])
    if rank == 0:
        ref = RPN(cfg, device=dev, seed=1)
        with torch.no_grad():
            o = ref.forward(vol.to(dev), proposals=proposals)
            tot, _, _ = ref.loss_total(o, RPNTargets(match, bbox, dev))
        v["loss_n1"] = float(tot)
        v["loss_matches_n1"] = rel_close(v["loss"], v["loss_n1"], 1e-5)
        if proposals:
            v["rois_match_n1"] = bool(torch.equal(o["rpn_rois"], r["rpn_rois"]))
        v["ok"] = bool(v["ok"] and v["loss_matches_n1"] and v.get("rois_match_n1", True))
        del ref, o
        torch.cuda.empty_cache()
    flag = torch.tensor([1 if v["ok"] else 0], device=dev, dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    v["ok"] = bool(int(flag.item()))
    return v


def validate_dp(model, world):
    """Data-parallel run (weak scaling): after the timed steps the weights --
    each rank's own update from the averaged gradient -- must be bit-identical
    on every rank."""
    from m3d.parallel import validate_replicas
    v = validate_replicas({"weights": model.store.flat, "sgd_moments": model.store.moments})
    v["world"] = world
    return v


# ---------------------------------------------------------------- forward roofline
def _peak_flops(engine):
    """FLOP/s ceiling of the kernel that ran a logged launch group: the x3
    kernels (fp32 as six bf16 MFMAs) at bf16 peak / 6, the rest at the f32 MFMA peak."""
    return (X3_PEAK_TFLOPS if engine == "x3" else F32_MFMA_PEAK_TFLOPS) * 1e12


def _roof_s(rec_row, f32_only=False):
    eng = "f32" if f32_only else (rec_row[8] if len(rec_row) > 8 else "f32")
    return max(rec_row[2] / _peak_flops(eng), rec_row[3] / (HBM_PEAK_GBS * 1e9))


def _host_ahead(seconds=0.5):
    """Let the host run ahead of the GPU before an instrumented pass: a spin
    kernel on the current stream holds the GPU while the host enqueues the pass,
    so the HIP events around each launch group time the GPU's work, not the
    host's enqueue gaps (the brackets of a GPU waiting for the host measured
    e.g. conv1 fwd 2.2 ms vs its 0.32 ms kernel)."""
    torch.cuda._sleep(int(seconds * 2.0e9))
def fwd_roofline(model, image, reps=3):
    """Per-stage forward roofline: every conv / pool of the
    backbone, FPN and RPN head is logged once (m3d.nn.LAYER_LOG) with its
    direct-conv FLOPs, the MFMA FLOPs the chosen algorithm executes (Winograd
    GEMMs for the 3^3 layers) and its compulsory HBM bytes (in + w + residual
    + out).  t_roof = sum_l max(F_exec_l / P_mfma, B_l / P_hbm); frac =
    t_roof / t_measured (HIP events, no_grad forward of that stage).  The SURVEY
    form with direct FLOPs is reported too (it exceeds 1 where Winograd beats
    the direct-conv bound)."""
    from m3d import nn as mnn
    stages = {}

    def run(name, fn):
        mnn.LAYER_LOG = []
        with torch.no_grad():
            r = fn()
        torch.cuda.synchronize()
        rec, mnn.LAYER_LOG = mnn.LAYER_LOG, None
        with torch.no_grad():
            t = _event_time(fn, reps)
        t_exec = sum(_roof_s(r_) for r_ in rec)
        t_exec32 = sum(_roof_s(r_, f32_only=True) for r_ in rec)
        t_dir = sum(max(r_[1] / (F32_MFMA_PEAK_TFLOPS * 1e12), r_[3] / (HBM_PEAK_GBS * 1e9)) for r_ in rec)
        nb = sum(r_[3] for r_ in rec)
        stages[name] = {"ms": round(t * 1e3, 3), "layers": len(rec),
                        "direct_tflop": round(sum(r_[1] for r_ in rec) / 1e12, 4),
                        "executed_tflop": round(sum(r_[2] for r_ in rec) / 1e12, 4),
                        "compulsory_gb": round(nb / 1e9, 3),
                        "roofline_ms": round(t_exec * 1e3, 3), "frac_roofline": round(t_exec / t, 4),
                        "frac_roofline_f32_priced": round(t_exec32 / t, 4),
                        "frac_roofline_direct_flops": round(t_dir / t, 4),
                        "hbm_frac": round(nb / t / (HBM_PEAK_GBS * 1e9), 4)}
        return r

    _, C2, C3, C4, C5 = run("backbone", lambda: model.backbone(image))
    fm = run("fpn", lambda: model.fpn(C2, C3, C4, C5))
    run("rpn_head", lambda: model.rpn(fm)[:2])
    tot_ms = sum(v["ms"] for v in stages.values())
    roof = sum(v["roofline_ms"] for v in stages.values())
    stages["total"] = {"ms": round(tot_ms, 3), "roofline_ms": round(roof, 3),
                       "frac_roofline": round(roof / tot_ms, 4),
                       "compulsory_gb": round(sum(v["compulsory_gb"] for v in stages.values()), 3)}
    return stages


def step_roofline(model, run_step, ms_per_step, table_path=None):
    """Roofline of the whole headline step (forward + backward + optimizer;
    SURVEY.md 8d per-layer form): one extra instrumented step logs every
    launch group (m3d.nn.LAYER_LOG with LAYER_TIMING: conv forward, BN/ReLU
    backward, data gradient, weight gradient, pooling / resampling, the fused
    RPN output heads, the optimizer) with its executed MFMA FLOPs, compulsory
    HBM bytes and the MFMA form it ran on, bracketed by HIP events on the
    stream it runs on.  t_roof = sum_l max(F_l / P_l, B_l / P_hbm) with P_l the
    ceiling of the kernel that ran group l (x3 kernels: bf16 peak / 6 = 419.4
    TFLOP/s; f32 MFMA kernels: 157.3); frac = t_roof / ms_per_step (the timed
    headline step); frac_f32_priced prices every group at the f32 MFMA peak
    (the looser bound of round 3).  The host is put ahead of the GPU first
    (_host_ahead), so each group's event bracket is GPU time -- its own kernels,
    slowed by whatever the side streams run beside them -- not enqueue gaps.
    'top_gaps' lists the five largest measured - roofline differences (weight
    gradients run on a side stream concurrently with the data-gradient chain,
    so measured times overlap and their sum exceeds the step).  The loss, the
    ProposalLayer (side stream, latency-bound) and the gradient zero-fill are
    not logged: the roofline is a lower bound."""
    from m3d import nn as mnn
    run_step()                         # an eager, un-logged step first (allocator / caches warm)
    torch.cuda.synchronize()
    mnn.LAYER_LOG, mnn.LAYER_TIMING = [], True
    try:
        _host_ahead()
        run_step()
        torch.cuda.synchronize()
        rec = mnn.LAYER_LOG
    finally:
        mnn.LAYER_LOG, mnn.LAYER_TIMING = None, False
    if not rec:
        return {"error": "no launch group logged (a graph replay is not instrumented)"}
    pb = HBM_PEAK_GBS * 1e9
    rows, phases = [], {}
    for r_ in rec:
        kind, fd, fe, nb, phase, name, e0, e1 = r_[:8]
        eng = r_[8] if len(r_) > 8 else "f32"
        pf = _peak_flops(eng)
        tr = max(fe / pf, nb / pb)
        tr32 = _roof_s(r_, f32_only=True)
        tm = e0.elapsed_time(e1) / 1e3 if e0 is not None else None
        rows.append({"layer": name, "kind": kind, "phase": phase, "engine": eng, "flop": fe, "bytes": nb,
                     "bound": "mfma" if fe / pf >= nb / pb else "hbm",
                     "roof_us": round(tr * 1e6, 2), "roof_f32_us": round(tr32 * 1e6, 2),
                     "meas_us": None if tm is None else round(tm * 1e6, 2)})
        ph = phases.setdefault(phase, {"launch_groups": 0, "roof_ms": 0.0, "roof_f32_ms": 0.0, "meas_ms": 0.0,
                                       "tflop": 0.0, "gb": 0.0})
        ph["launch_groups"] += 1
        ph["roof_ms"] += tr * 1e3
        ph["roof_f32_ms"] += tr32 * 1e3
        ph["meas_ms"] += (tm or 0.0) * 1e3
        ph["tflop"] += fe / 1e12
        ph["gb"] += nb / 1e9
    for ph in phases.values():
        for k in ("roof_ms", "roof_f32_ms", "meas_ms", "tflop", "gb"):
            ph[k] = round(ph[k], 3)
    roof = sum(r["roof_us"] for r in rows) / 1e3
    roof32 = sum(r["roof_f32_us"] for r in rows) / 1e3
    gaps = sorted((r for r in rows if r["meas_us"] is not None), key=lambda r: r["meas_us"] - r["roof_us"],
                  reverse=True)[:5]
    if table_path:
        with open(table_path, "w") as f:
            json.dump({"ms_per_step": ms_per_step, "step_roofline_ms": roof, "step_roofline_f32_priced_ms": roof32,
                       "rows": rows}, f, indent=0)
    return {"step_roofline_ms": round(roof, 3), "ms_per_step": round(ms_per_step, 3),
            "frac": round(roof / ms_per_step, 4),
            "step_roofline_f32_priced_ms": round(roof32, 3), "frac_f32_priced": round(roof32 / ms_per_step, 4),
            "launch_groups": len(rows), "phases": phases,
            "top_gaps": [{k: r[k] for k in ("layer", "kind", "phase", "engine", "bound", "roof_us", "meas_us")}
                         for r in gaps],
            "peaks": {"x3_tflops": X3_PEAK_TFLOPS, "f32_mfma_tflops": F32_MFMA_PEAK_TFLOPS, "hbm_gbs": HBM_PEAK_GBS},
            "note": "sum over launch groups of max(executed MFMA FLOPs / the ceiling of the kernel that ran them, "
                    "compulsory bytes / HBM peak) / ms_per_step; Winograd layers priced at their executed GEMM FLOPs; "
                    "meas_us = HIP events around the group with the host enqueued ahead (GPU time)"}


def roi_leg_large(S, dev, n_rois=512):
    """configs[3] shapes: PyramidROIAlign 7^3 and 14^3 of 512 proposals on the
    P2..P5 maps of a frozen S^3 forward (boxes log-uniform in [24, S] px, so
    levels 2-4 are hit at 256^3)."""
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    model = RPN(synthetic_rpn_config(S), device=dev, seed=1)
    image = synthetic_volume(S).to(dev)
    with torch.no_grad():
        fmaps = model.features(image)
    r = time_roi_align(fmaps, S, n_rois=n_rois, hi=S)
    try:
        r["bwd"] = time_roi_align_bwd(fmaps, S, n_rois=n_rois, hi=S)
    except Exception as e:  # report, never hide
        r["bwd"] = {"error": repr(e)}
    r["config"] = f"{n_rois} ROIs on P2..P5 of a {S}^3 volume, C=256"
    del fmaps
    torch.cuda.empty_cache()
    try:
        r["fwd_roofline"] = fwd_roofline(model, image)
    except Exception as e:  # report, never hide
        r["fwd_roofline"] = {"error": repr(e)}
    del model, image
    return r


def inference_roofline(model, image, meta, reps=3):
    """Per-stage roofline of MaskRCNN.detect (BASELINE configs[3],
    core/models.py:5473-5754): every stage of the inference pass timed alone
    with HIP events (the host enqueued ahead), and priced at
    max(executed MFMA FLOPs / the ceiling of the kernel that ran them,
    compulsory HBM bytes / HBM peak):
      backbone / fpn / rpn_head / mask_head convs: m3d.nn.LAYER_LOG (Winograd
        layers at their point-GEMM FLOPs), plus the mask head's dilated conv3b,
        transposed conv and sigmoid conv counted here;
      roi_align7 / roi_align14: output + 4*C*|unique voxels| (HBM);
      classifier: mrcnn_class_conv1 (a pool^3 x C GEMM, f32 MFMA), conv2 and the
        dense heads, weights + activations (whichever bound);
      proposal_layer (top-k + 3-D NMS) and detection (2-D NMS): latency-bound by
        definition (the serial greedy reduction), reported without a roof.
    frac = sum of the roofs / sum of the measured stage times."""
    from m3d import nn as mnn
    P = HBM_PEAK_GBS * 1e9
    stages = {}

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        _host_ahead(0.2)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            r = fn()
        e1.record()
        torch.cuda.synchronize()
        return r, e0.elapsed_time(e1) / reps / 1e3

    def logged(name, fn, extra_flop=0.0, extra_bytes=0.0, engine="f32"):
        mnn.LAYER_LOG = []
        try:
            r = fn()
            torch.cuda.synchronize()
            rec = mnn.LAYER_LOG
        finally:
            mnn.LAYER_LOG = None
        r, t = timed(fn)
        roof = sum(_roof_s(x) for x in rec) + max(extra_flop / _peak_flops(engine), extra_bytes / P)
        stages[name] = {"ms": round(t * 1e3, 3), "roofline_ms": round(roof * 1e3, 3),
                        "frac_roofline": round(roof / t, 4), "layers": len(rec)}
        return r

    def priced(name, fn, flop, nbytes, engine="f32"):
        r, t = timed(fn)
        roof = max(flop / _peak_flops(engine), nbytes / P)
        stages[name] = {"ms": round(t * 1e3, 3), "roofline_ms": round(roof * 1e3, 3),
                        "frac_roofline": round(roof / t, 4), "bound": "mfma" if flop / _peak_flops(engine) >=
                        nbytes / P else "hbm", "tflop": round(flop / 1e12, 4), "gb": round(nbytes / 1e9, 4)}
        return r

    def latency(name, fn):
        r, t = timed(fn)
        stages[name] = {"ms": round(t * 1e3, 3), "roofline_ms": None, "bound": "latency"}
        return r

    with torch.no_grad():
        _, C2, C3, C4, C5 = logged("backbone", lambda: model.backbone(image))
        fmaps = logged("fpn", lambda: model.fpn(C2, C3, C4, C5))
        _, rpn_probs, rpn_bbox = logged("rpn_head", lambda: model.rpn(fmaps))
        rois = latency("proposal_layer", lambda: model.proposal_layer([rpn_probs, rpn_bbox, model.anchors]))
        maps4 = fmaps[:4]
        fshapes = [tuple(f.shape[1:4]) for f in maps4]
        C = int(maps4[0].shape[-1])
        S = int(image.shape[1])
        cfg = model.config

        def roi_bytes(boxes, pool):
            n = int(boxes.shape[1])
            u = unique_voxels(boxes[:1].detach().float().cpu().numpy(), fshapes, (pool,) * 3, S)
            return 4.0 * (n * pool ** 3 * C + C * u)
        p7 = int(cfg.POOL_SIZE)
        pooled = priced("roi_align7", lambda: model.roi_align_classifier([rois, meta] + maps4), 0.0,
                        roi_bytes(rois, p7))
        M = int(pooled.shape[0] * pooled.shape[1])
        K, fc, ncls = p7 ** 3 * C, model.classifier.fc, model.classifier.C
        f_cls = 2.0 * M * (K * fc + fc * fc + fc * 7 * ncls)
        b_cls = 4.0 * (M * K + K * fc + fc * fc + fc * 7 * ncls + 2 * M * fc + M * 8 * ncls)
        _, mclass, mbbox = priced("classifier", lambda: model.classifier(pooled), f_cls, b_cls)
        det = latency("detection", lambda: model.detection([rois, mclass, mbbox, meta]))
        dboxes = det[..., :6].contiguous()
        p14 = int(cfg.MASK_POOL_SIZE)
        mpooled = priced("roi_align14", lambda: model.roi_align_mask([dboxes, meta] + maps4), 0.0,
                         roi_bytes(dboxes, p14))
        Mm = int(mpooled.shape[0] * mpooled.shape[1])
        ch = model.mask_head.ch
        v = Mm * p14 ** 3
        f_extra = 2.0 * v * 27 * ch * ch + 2.0 * v * 8 * ch * ch + 2.0 * 8 * v * ch * ncls
        b_extra = 4.0 * (3 * v * ch + 27 * ch * ch + v * ch + 8 * ch * ch + 8 * v * ch + 8 * v * ch + 8 * v * ncls)
        logged("mask_head", lambda: model.mask_head(mpooled), f_extra, b_extra)
    tot = sum(v["ms"] for v in stages.values())
    roof = sum(v["roofline_ms"] or 0.0 for v in stages.values())
    return {"stages": stages, "ms": round(tot, 3), "roofline_ms": round(roof, 3), "frac": round(roof / tot, 4),
            "note": "sum over stages timed alone of max(MFMA FLOPs / ceiling, compulsory bytes / HBM peak) / "
                    "sum of stage times; NMS stages are latency-bound and carry no roof (lower bound)"}


def mrcnn_inference_leg(S, steps, warmup, dev):
    """BASELINE configs[3]: full Mask R-CNN inference on one S^3 volume --
    backbone + FPN + RPN forward, ProposalLayer (3-D NMS, 512 proposals),
    PyramidROIAlign 7^3 -> classifier head -> DetectionLayer (2-D NMS) ->
    PyramidROIAlign 14^3 -> mask head.  Random-init weights: the detection
    count is whatever the synthetic volume yields (reported).  `roofline`:
    inference_roofline (per stage); its rocprof kernel table is
    profiles/r05*_infer_kernels*.txt (scripts/infer_prof.py)."""
    from m3d.config import synthetic_mrcnn_config
    from m3d.heads import MaskRCNN
    from m3d.model import compose_image_meta, synthetic_volume
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)      # peak_mem_gb is this leg's own
    cfg = synthetic_mrcnn_config(S)
    model = MaskRCNN(cfg, device=dev, seed=1)
    image = synthetic_volume(S, seed=100).to(dev)
    meta = torch.from_numpy(compose_image_meta(0, [S, S, S, 1], [S, S, S, 1], [0, 0, 0, S, S, S], 1.0,
                                               [0, 1])[None]).to(dev)
    for _ in range(warmup):
        out = model.detect(image, meta)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = model.detect(image, meta)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    n_det = int((out["detections"][0, :, 7] > 0).sum())
    res = {"workload": f"configs[3]: MaskRCNN inference, one {S}^3 volume, {cfg.POST_NMS_ROIS_INFERENCE} "
                       f"proposals, ROIAlign 7^3/14^3, classifier + DetectionLayer + mask head",
           "size": S, "ms_per_volume": round(el / steps * 1e3, 2), "volumes_per_s": round(steps / el, 4),
           "detections": n_det, "max_instances": int(cfg.DETECTION_MAX_INSTANCES),
           "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 1)}
    del out
    try:
        res["roofline"] = inference_roofline(model, image, meta)
    except Exception as e:  # report, never hide
        res["roofline"] = {"error": repr(e)}
    del model
    torch.cuda.empty_cache()
    return res


def _host_cpus():
    """The box's CPUs beside the thread count the baseline used: os.cpu_count()
    (the whole machine), the CPUs this process may run on (its affinity / the
    box's CPU share, which OMP_NUM_THREADS mirrors) and the lscpu model name."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    return {"os_cpu_count": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads": os.environ.get("OMP_NUM_THREADS"), "model": model}


def _usable_cpus(default):
    """CPUs this process can actually run on: its affinity set, capped by the
    cgroup CPU quota (cpu.max) when one is set -- threads beyond the quota only
    time-slice against each other."""
    try:
        n = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return default
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                n = min(n, max(1, int(int(q) / int(per))))
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            n = min(n, max(1, q // per))
    except (OSError, ValueError):
        pass
    return max(1, min(n, 256))


def cpu_baseline(model, S, targets_np, depth_slab=0, threads=None):
    """The oracle restatement timed on the host for the SAME step as the GPU
    leg: oracle/model_ref.py forward (torch-CPU fp32) -> the RPN losses of
    core/models.py:1589-1673 with the compiled weights (1.0 / 1.5,
    core/models.py:3366-3369) on the same synthetic targets -> backward ->
    the Keras SGD update of every weight (oracle/optim_ref.py: L2 term,
    clipnorm, momentum) -> the ProposalLayer (oracle/ops_ref.py: top-k,
    decode, the C NMS restatement 15000 -> 6000).  With depth_slab the
    network runs on an S x S x depth_slab slab and its time is scaled to the
    whole volume (work is linear in depth); the ProposalLayer and SGD always
    run at full size."""
    from oracle import model_ref as MR
    from oracle import ops_ref as R
    from oracle import optim_ref as OR
    depth_slab = depth_slab or S
    if threads:
        torch.set_num_threads(threads)
    cfg = model.config
    params = model.store.state_dict()
    ref = MR.RefRPN(params, dtype=torch.float32)
    trainable = [k for k in ref.p if not k.endswith(("moving_mean:0", "moving_variance:0"))]
    for k in trainable:
        ref.p[k].requires_grad_(True)
    match, bbox = targets_np
    x = torch.tanh(0.5 * torch.randn((1, S, S, depth_slab, 1), generator=torch.Generator().manual_seed(0)))
    t0 = time.perf_counter()
    o = ref.forward(x)
    if depth_slab == S:
        m = torch.from_numpy(match.astype(np.int64))
        loss = MR.rpn_class_loss(m, o["rpn_class_logits"]) * 1.0 + \
            MR.rpn_bbox_loss(torch.from_numpy(bbox), m, o["rpn_bbox"]) * 1.5
    else:   # slab: the anchors differ from the targets' -- same reduction work, synthetic objective
        loss = o["rpn_class_logits"].square().mean() + o["rpn_bbox"].square().mean()
    loss.backward()
    t_net = time.perf_counter() - t0
    t1 = time.perf_counter()
    opt = model.optimizer
    lr, mom, clip = float(opt.current_lr()), float(opt.params.get("momentum", 0.0)), opt.clipnorm
    state = {}
    for k in trainable:
        p = model.store.by_name.get(k)
        l2 = cfg.WEIGHT_DECAY / ref.p[k].numel() if (p is not None and p.l2) else 0.0
        OR.step("SGD", ref.p[k].detach().numpy(), ref.p[k].grad.numpy(), state.setdefault(k, {}), 0, lr,
                clipnorm=clip, l2coef=l2, momentum=mom)
    probs = o["rpn_class"].detach().numpy()
    deltas = o["rpn_bbox"].detach().numpy()
    if depth_slab == S:
        anchors = model.anchors.cpu().numpy()
        R.proposal_layer(probs, deltas, anchors, cfg.POST_NMS_ROIS_TRAINING, cfg.RPN_NMS_THRESHOLD,
                         cfg.PRE_NMS_LIMIT, np.asarray(cfg.RPN_BBOX_STD_DEV, np.float32), float(cfg.IMAGE_DEPTH))
    t_rest = time.perf_counter() - t1
    t = t_net * (S / depth_slab) + t_rest
    return {"value": 1.0 / t, "unit": "volumes/s", "cores": torch.get_num_threads(), "kind": "port",
            "host": _host_cpus(),
            "sample": f"one RPN training step (the GPU step's work) on the host: oracle/model_ref.py torch-CPU fp32 fwd + RPN "
                      f"losses + bwd on a {S}x{S}x{depth_slab} volume ({t_net:.1f} s"
                      + (f", scaled x{S // depth_slab}" if depth_slab != S else "")
                      + f"), oracle SGD update of all weights + ProposalLayer (C NMS) {t_rest:.1f} s"}


def cpu_ops_leg(fmaps, S, dev, n_rois=128, pools=(7, 14)):
    """the reference's native ops are single-threaded CPU
    OpKernels (CropAndResize3D @0x4370, its GradImage @0x3a80,
    NonMaxSuppression3D @0xe4e0: no Shard), so each is timed here as the
    oracle's C restatement (oracle/oracle.c, gcc -O2, ONE thread) beside the
    HIP kernel on the same inputs: NMS 15000 -> 6000 at IoU 0.7 (the
    ProposalLayer's training shape) and CropAndResize3D fwd / GradImage of 128
    ROIs at 7^3 and 14^3 on P2 of the 128^3 forward (C = 256)."""
    from m3d import ops
    from oracle import ops_ref as R
    res = {"threads": 1, "kind": "port"}
    # NMS at the time_nms shape and seed
    rng = np.random.default_rng(4)
    k = 15000
    c = rng.uniform(0.05, 0.95, (k, 3))
    ext = np.exp(rng.uniform(np.log(0.02), np.log(0.3), (k, 3))) / 2
    bnp = np.concatenate([c - ext, c + ext], 1).astype(np.float32)
    snp = np.sort(rng.uniform(size=k))[::-1].astype(np.float32).copy()
    t0 = time.perf_counter()
    keep_c = R.non_max_suppression_3d(bnp, snp, 6000, 0.7)
    t_c = time.perf_counter() - t0
    bt, st_ = torch.from_numpy(bnp).to(dev), torch.from_numpy(snp).to(dev)
    keep_g = ops.non_max_suppression_3d(bt, st_, 6000, 0.7)
    t_g = _event_time(lambda: ops.non_max_suppression_3d_padded(bt, st_, 6000, 0.7), 5)
    res["nms_15000_6000"] = {"cpu_ms": round(t_c * 1e3, 2), "gpu_ms": round(t_g * 1e3, 4),
                             "speedup": round(t_c / t_g, 1),
                             "identical": bool(np.array_equal(keep_g.cpu().numpy(), keep_c))}
    p2 = fmaps[0].detach().contiguous()
    img = p2.cpu().numpy()
    boxes = roi_boxes(n_rois, S)[0]
    bi = np.zeros(n_rois, np.int32)
    bt = torch.from_numpy(boxes).to(dev)
    bit = torch.from_numpy(bi).to(dev)
    for p in pools:
        t0 = time.perf_counter()
        crop_c = R.crop_and_resize_3d(img, boxes, bi, (p, p, p))
        t_fc = time.perf_counter() - t0
        crop_g = ops.crop_and_resize_3d(p2, bt, bit, (p, p, p), validate=False)
        t_fg = _event_time(lambda: ops.crop_and_resize_3d(p2, bt, bit, (p, p, p), validate=False), 5)
        g = np.random.default_rng(p).normal(size=crop_c.shape).astype(np.float32)
        t0 = time.perf_counter()
        gi_c = R.crop_and_resize_3d_grad_image(g, boxes, bi, img.shape)
        t_bc = time.perf_counter() - t0
        gt = torch.from_numpy(g).to(dev)
        t_ba = _event_time(lambda: ops.crop_and_resize_3d_grad_image(gt, bt, bit, img.shape, deterministic=0), 5)
        gi_d = ops.crop_and_resize_3d_grad_image(gt, bt, bit, img.shape, deterministic=1)
        t_bd = _event_time(lambda: ops.crop_and_resize_3d_grad_image(gt, bt, bit, img.shape, deterministic=1), 5)
        res[f"crop_{p}"] = {"cpu_fwd_ms": round(t_fc * 1e3, 2), "gpu_fwd_ms": round(t_fg * 1e3, 4),
                            "fwd_speedup": round(t_fc / t_fg, 1),
                            "fwd_identical": bool(np.array_equal(crop_g.cpu().numpy(), crop_c)),
                            "cpu_grad_image_ms": round(t_bc * 1e3, 2),
                            "gpu_grad_image_atomic_ms": round(t_ba * 1e3, 4),
                            "gpu_grad_image_deterministic_ms": round(t_bd * 1e3, 4),
                            "grad_speedup_deterministic": round(t_bc / t_bd, 1),
                            "grad_deterministic_identical": bool(np.array_equal(gi_d.cpu().numpy(), gi_c))}
        del crop_c, gi_c, gi_d, crop_g
    res["note"] = (f"single-thread C restatement vs the HIP kernel, same inputs; crops: {n_rois} ROIs on P2 "
                   f"{list(p2.shape)}")
    return res


# ---------------------------------------------------------------- main
def deterministic_leg(step, steps, warmup):
    """The same N=1 training step in deterministic mode (m3d.set_deterministic:
    weight-gradient m-splits and clip norms summed in a fixed order through a
    scratch buffer, no fp32 atomics): ms/step, and whether two runs of the
    weights' update agree bit for bit is covered by tests/test_gpu_determinism."""
    from m3d import _lib
    _lib.set_deterministic(True)
    try:
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
    finally:
        _lib.set_deterministic(False)
    return {"ms_per_step": round(el / steps * 1e3, 2), "steps": steps, "scratch_mb": 256}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--size", type=int, default=128)
    ap.add_argument("--no-proposals", action="store_true")
    ap.add_argument("--slab-size", type=int, default=256,
                    help="depth-slab leg volume size (configs[4]); 0 disables the leg")
    ap.add_argument("--no-extras", action="store_true", help="skip roofline / ROIAlign / CPU legs")
    ap.add_argument("--roi-size", type=int, default=256, help="large-volume ROIAlign leg (0: off)")
    ap.add_argument("--infer-size", type=int, default=256, help="MaskRCNN inference leg size (0: off)")
    ap.add_argument("--cpu-slab", type=int, default=0, help="CPU-baseline depth slab (0: whole volume)")
    ap.add_argument("--graph", action="store_true", help="(default at N=1) HIP-graph replay of the step")
    ap.add_argument("--eager", action="store_true", help="N=1: eager launches instead of the HIP-graph replay")
    ap.add_argument("--wgrad-inline", action="store_true",
                    help="weight gradients on the compute stream (serialized kernel traces)")
    args = ap.parse_args()
    if args.wgrad_inline:
        from m3d import nn as mnn
        mnn.WGRAD_STREAM = False

    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume
    from m3d.parallel import data_parallel_train_step, init_from_env

    rank, world = init_from_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    S = args.size
    cfg = synthetic_rpn_config(S)
    model = RPN(cfg, device=dev, seed=1)          # same init on every rank
    image = synthetic_volume(S, seed=100 + rank).to(dev)
    match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE,
                                        seed=200 + rank)
    targets = RPNTargets(match, bbox, dev)
    props = not args.no_proposals

    def eager_step():
        return data_parallel_train_step(model, image, targets, world, proposals=props)

    graph_error = None
    use_graph = world == 1 and not args.eager
    if use_graph:
        # N=1: the forward + backward (+ ProposalLayer) captured once as a HIP graph
        # (m3d.model.RPN.graphed_train_step) and replayed, the optimizer eager
        # after it.  128^3: 26.04 vs 26.23 ms eager, host 6.6 vs 16.5 ms per step
        # (DESIGN.md 5, round 5).  N>1 stays eager: the gradient buckets'
        # all-reduces are enqueued as the backward produces them.
        try:
            step = model.graphed_train_step(image, targets, proposals=props)
        except Exception as e:  # report, never hide: the line then says hip_graph false
            graph_error = repr(e)
            use_graph = False
            torch.cuda.synchronize()
    if not use_graph:
        step = eager_step

    log(f"[bench] rank {rank}/{world} size {S}^3, warmup {args.warmup}")
    for _ in range(args.warmup):
        r = step()
    torch.cuda.synchronize()
    log(f"[bench] warmup done, loss {float(r['loss']):.4f}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        r = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el / args.steps * 1e3
    value = world * args.steps / el
    log(f"[bench] {ms:.1f} ms/step, {value:.3f} volumes/s, loss {float(r['loss']):.4f}")

    out = {"metric": METRIC, "value": round(value, 4), "unit": "volumes/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 2),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic (tanh(0.5*N(0,1)) volumes, seeded RPN targets; random-init weights)",
           "config": {"workload": f"configs[1]: RPN training step, ResNet50-3D+FPN+RPN fwd+bwd+SGD"
                                  f"{' + ProposalLayer(3D NMS 15000->6000)' if props else ''}, "
                                  f"{S}^3 x1 volume per GPU",
                      "size": S, "batch_per_gpu": 1, "parallelism": f"dp{world}",
                      "anchors": int(model.anchors.shape[1]),
                      "hip_graph": use_graph}}
    if graph_error is not None:
        out["config"]["hip_graph_error"] = graph_error
    if use_graph:
        # the same step launched eagerly, timed the same way (for comparison only)
        for _ in range(2):
            eager_step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            eager_step()
        torch.cuda.synchronize()
        out["eager_ms_per_step"] = round((time.perf_counter() - t0) / args.steps * 1e3, 2)
        model._graph = step = None              # release the replay's private pool before the legs
    if world == 1 and not args.no_extras:
        try:
            out["step_roofline"] = step_roofline(model, eager_step, ms, os.environ.get("M3D_STEP_ROOFLINE_TABLE"))
        except Exception as e:  # report, never hide
            out["step_roofline"] = {"error": repr(e)}
    if world > 1:
        v = validate_dp(model, world)
        out.setdefault("validation", {})["dp"] = v
        log(f"[bench] dp validation: {json.dumps(v)}")
    if world > 1 and not args.no_extras:
        try:
            ar = time_allreduce(model.store.grad_flat, world)
        except Exception as e:  # report, never hide
            ar = {"error": repr(e)}
        if rank == 0:
            out["allreduce"] = ar
            out["validation"]["dp"]["allreduce_bus_GBps"] = ar.get("bus_GBps")
    if args.slab_size and not args.no_extras:
        log(f"[bench] leg depth_slab {args.slab_size}^3 ({time.strftime('%H:%M:%S')})")
        del r
        torch.cuda.empty_cache()
        try:
            # N > 1: the halo exchanges and merged proposals run over RCCL P2P /
            # all-gathers that have no timeout of their own
            with LegWatchdog(float(os.environ.get("M3D_SLAB_LEG_TIMEOUT", "300")), rank, out, "depth_slab") \
                    if world > 1 else contextlib.nullcontext():
                out["depth_slab"] = depth_slab_leg(args.slab_size, args.steps, args.warmup, rank, world, dev,
                                                   proposals=props)
                if "validation" in out["depth_slab"]:
                    out.setdefault("validation", {})["depth_slab"] = out["depth_slab"]["validation"]
        except Exception as e:  # report, never hide
            out["depth_slab"] = {"error": repr(e)}
    if world == 1 and not args.no_extras:
        try:
            log(f"[bench] leg configs0 ({time.strftime('%H:%M:%S')})")
            out["configs0"] = configs0_leg(dev, max(3, args.steps // 2), 2)
        except Exception as e:  # report, never hide
            out["configs0"] = {"error": repr(e)}
        try:
            log(f"[bench] leg targets_in_step ({time.strftime('%H:%M:%S')})")
            out["targets_in_step"] = targets_in_step_leg(model, image, max(3, args.steps // 2), 2, dev)
        except Exception as e:  # report, never hide
            out["targets_in_step"] = {"error": repr(e)}
        try:
            log(f"[bench] leg deterministic ({time.strftime('%H:%M:%S')})")
            out["deterministic"] = deterministic_leg(eager_step, max(3, args.steps // 2), 2)
        except Exception as e:  # report, never hide
            out["deterministic"] = {"error": repr(e)}
    if rank == 0 and not args.no_extras:
        with torch.no_grad():
            fmaps = model.features(image)
        try:
            # the headline roofline prices the step's dominant kernel, DOMINANT_KERNEL
            # (line 1 of the committed rocprof table of the same tree,
            # profiles/dominant_kernel_table.txt; tests/test_bench_contract.py checks
            # the two agree); the other point-GEMM kernel is a sub-leg
            log(f"[bench] leg roofline ({time.strftime('%H:%M:%S')})")
            legs = {"x3_wgrad_tr_kernel": lambda: time_wgrad_gemm(S), "x3_gemm256_af_kernel": lambda: time_wino_gemm(S)}
            out["roofline"] = legs[DOMINANT_KERNEL]()
            for k, f in legs.items():
                if k != DOMINANT_KERNEL:
                    out["roofline"]["wino_gemm" if k == "x3_gemm256_af_kernel" else "wgrad_gemm"] = f()
            out["roofline"]["dominant_kernel_table"] = "profiles/dominant_kernel_table.txt"
            out["roofline"]["direct_conv"] = time_direct_conv(model, fmaps)
            out["roofline"]["wino_fwd_conv"] = time_wino_fwd(S)
        except Exception as e:  # report, never hide
            out["roofline"] = {"error": repr(e)}
        try:
            log(f"[bench] leg roi_align ({time.strftime('%H:%M:%S')})")
            out["roi_align"] = time_roi_align(fmaps, S)
        except Exception as e:
            out["roi_align"] = {"error": repr(e)}
        try:
            log(f"[bench] leg roi_align_bwd ({time.strftime('%H:%M:%S')})")
            out["roi_align_bwd"] = time_roi_align_bwd(fmaps, S)
        except Exception as e:
            out["roi_align_bwd"] = {"error": repr(e)}
        del fmaps
        try:
            log(f"[bench] leg nms ({time.strftime('%H:%M:%S')})")
            out["nms"] = time_nms(dev)
        except Exception as e:
            out["nms"] = {"error": repr(e)}
        try:
            log(f"[bench] leg fwd_roofline ({time.strftime('%H:%M:%S')})")
            out["fwd_roofline"] = fwd_roofline(model, image)
        except Exception as e:
            out["fwd_roofline"] = {"error": repr(e)}
        torch.cuda.empty_cache()
        if args.roi_size:
            try:
                log(f"[bench] leg roi_align_256 ({time.strftime('%H:%M:%S')})")
                out["roi_align_256"] = roi_leg_large(args.roi_size, dev)
            except Exception as e:
                out["roi_align_256"] = {"error": repr(e)}
            torch.cuda.empty_cache()
        if args.infer_size:
            try:
                log(f"[bench] leg mrcnn_inference ({time.strftime('%H:%M:%S')})")
                out["mrcnn_inference"] = mrcnn_inference_leg(args.infer_size, max(3, args.steps // 2),
                                                             1, dev)
            except Exception as e:
                out["mrcnn_inference"] = {"error": repr(e)}
        if world == 1:
            try:
                with torch.no_grad():
                    fm2 = model.features(image)
                log(f"[bench] leg cpu_ops ({time.strftime('%H:%M:%S')})")
                out["cpu_ops"] = cpu_ops_leg(fm2, S, dev)
                del fm2
            except Exception as e:
                out["cpu_ops"] = {"error": repr(e)}
            try:
                # the box's CPU share (OMP_NUM_THREADS) and every CPU of its affinity;
                # the faster one is the reported baseline, both are kept
                n_share = torch.get_num_threads()
                n_aff = _usable_cpus(n_share)
                log(f"[bench] leg cpu_baseline: {n_share} and {n_aff} threads")
                runs = [cpu_baseline(model, S, (match, bbox), args.cpu_slab, threads=n_share)]
                if n_aff > n_share:
                    runs.append(cpu_baseline(model, S, (match, bbox), args.cpu_slab, threads=n_aff))
                torch.set_num_threads(n_share)
                best = dict(max(runs, key=lambda r: r["value"]))
                best["runs"] = [{"cores": r["cores"], "value": round(r["value"], 4)} for r in runs]
                out["cpu_baseline"] = best
            except Exception as e:
                out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        out["summary"] = summary(out)     # last key: survives a truncated tail of the line
        print(json.dumps(out), flush=True)
    failed = [k for k, v in out.get("validation", {}).items() if isinstance(v, dict) and v.get("ok") is False]
    if world > 1:
        dist.destroy_process_group()
    if failed:
        log(f"[bench] VALIDATION FAILED: {failed}")
        sys.exit(4)


def summary(out):
    """Compact trailer of the JSON line: the headline numbers of every config."""
    def g(*path):
        d = out
        for k in path:
            if not isinstance(d, dict) or k not in d:
                return None
            d = d[k]
        return d
    return {"volumes_per_s_128": out.get("value"), "ms_per_step_128": out.get("ms_per_step"),
            "depth_slab_ms_per_step_256": g("depth_slab", "ms_per_step"),
            "depth_slab_volumes_per_s_256": g("depth_slab", "volumes_per_s"),
            "depth_slab_n_gpus": g("depth_slab", "n_gpus"),
            "step_roofline_frac_128": g("step_roofline", "frac"),
            "step_roofline_frac_256": g("depth_slab", "step_roofline", "frac"),
            "dominant_kernel_frac": g("roofline", "frac"),
            "roi14_256_frac_hbm": g("roi_align_256", "pool14", "frac_hbm"),
            "mrcnn_inference_256_ms": g("mrcnn_inference", "ms_per_volume"),
            "mrcnn_inference_256_roofline_frac": g("mrcnn_inference", "roofline", "frac"),
            "validation_ok": all(v.get("ok", True) for v in out.get("validation", {}).values()
                                 if isinstance(v, dict))}


if __name__ == "__main__":
    main()
