"""A/B of x3_gemm256_af_kernel builds: the priced launch (bench.py
time_wino_gemm: 96 batched Winograd point GEMMs of rpn_conv_shared1 on P2,
M=T, K=256, N=512 at 128^3; and the 256^3 shape) timed for libm3d.so and each
make-ab library named on the command line, interleaved over rounds in ONE
process (cdna_hip_programming.md 5.4 rule 24).  Outputs must be bit-identical.
Usage: python scripts/x3_ab.py libm3d_x3p1.so libm3d_x3p2.so ..."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402

names = ["libm3d.so"] + sys.argv[1:]
libs = []
for n in names:
    L = ctypes.CDLL(os.path.join(ROOT, "3d-mask-r-cnn_amd", "m3d", n))
    L.m3d_gemm_x3_af.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int64] * 4 + [ctypes.c_void_p]
    L.m3d_split3_f32.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    libs.append(L)
dev = torch.device("cuda:0")
res = {}
SHAPES = [("P2_128", 8192, 256, 512), ("P2_256", 65536, 256, 512), ("res2_128", 8192, 64, 64),
          ("res3_128", 2048, 128, 128), ("res4_128", 512, 256, 256), ("res5_128", 128, 512, 512),
          ("res4_256", 4096, 256, 256)]
for S, T, K, N in SHAPES:
    nb = 96
    g = torch.Generator(device=dev).manual_seed(5)
    A = torch.randn((nb, T, K), device=dev, generator=g)
    Bt = torch.randn((nb, N, K), device=dev, generator=g) * 0.05
    B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device=dev)
    libs[0].m3d_split3_f32(Bt.data_ptr(), Bt.numel(), B3.data_ptr(), torch.cuda.current_stream().cuda_stream)
    del Bt
    outs = [torch.empty((nb, T, N), device=dev) for _ in libs]
    st = torch.cuda.current_stream().cuda_stream
    times = {n: [] for n in names}
    for rnd in range(6):
        for L, n, C in zip(libs, names, outs):
            L.m3d_gemm_x3_af(A.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, T, K, N, st)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                L.m3d_gemm_x3_af(A.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, T, K, N, st)
            e1.record()
            torch.cuda.synchronize()
            times[n].append(e0.elapsed_time(e1) / 5)
    flops = 2.0 * nb * T * K * N
    for n, C in zip(names, outs):
        med = statistics.median(times[n])
        res[f"S{S}:{n}"] = {"ms_median": round(med, 4), "ms_min": round(min(times[n]), 4),
                            "frac": round(flops / (med * 1e-3) / 1e12 / 419.4, 4),
                            "identical": bool(torch.equal(C, outs[0]))}
        print(S, n, res[f"S{S}:{n}"], flush=True)
    del A, B3, outs
    torch.cuda.empty_cache()
print(json.dumps(res))
