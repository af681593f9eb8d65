"""Clock stamps of x3_gemm256_af_kernel (libm3d_stamp.so, M3D_X3AF_STAMP=1) on
the priced launch (bench.wino_gemm_shape): per workgroup the shader-clock
cycles of the prologue, each k step (barrier to barrier, wave 0), the epilogue,
and the effective clock (s_memtime / s_memrealtime at 100 MHz)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d import _lib  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
L = _lib.load()
nb, T, K, N = bench.wino_gemm_shape(S)
g = torch.Generator(device="cuda").manual_seed(5)
A = torch.randn((nb, T, K), device="cuda", generator=g)
Bt = torch.randn((nb, N, K), device="cuda", generator=g) * 0.05
B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device="cuda")
_lib.check(L.m3d_split3_f32(Bt.data_ptr(), Bt.numel(), B3.data_ptr(), _lib.stream()), "split3")
C = torch.empty((nb, T, N), device="cuda")
for _ in range(5):
    _lib.check(L.m3d_gemm_x3_af(A.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, T, K, N, _lib.stream()), "x3af")
torch.cuda.synchronize()
Cv = C.view(torch.int32).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
rows = []
for b in range(nb):
    for mt in range((T + 255) // 256):
        for nt in range(N // 256):
            rows.append(Cv[b, mt * 256, nt * 256:nt * 256 + 64])
R = np.array(rows)
nk = int(R[0, 6])
w = lambda a, b: (b - a) & 0xFFFFFFFF  # noqa: E731
t0, t1, t2, t3, r0, r3 = (R[:, i] for i in range(6))
cyc = w(t0, t3).astype(float)
real = w(r0, r3).astype(float) / 100e6
print(f"S={S} tiles={len(R)} nk={nk}")
print("clock GHz median", np.median(cyc / real / 1e9).round(3))
pro = w(t0, t1)
steps = np.stack([w(R[:, 8 + k], R[:, 9 + k]) for k in range(nk - 1)], 1)
last = w(R[:, 8 + nk - 1], t2)
epi = w(t2, t3)
print("prologue cycles  median %.0f  p90 %.0f" % (np.median(pro), np.percentile(pro, 90)))
print("first barrier (t1 -> step0) median %.0f" % np.median(w(t1, R[:, 8])))
print("step cycles      median %.0f  mean %.0f  p10 %.0f p90 %.0f  (MFMA-bound: 3072 per step at 2 waves/SIMD)"
      % (np.median(steps), steps.mean(), np.percentile(steps, 10), np.percentile(steps, 90)))
print("per-step median by k:", [int(np.median(steps[:, k])) for k in range(nk - 1)])
print("last step + drain median %.0f" % np.median(last))
print("epilogue cycles  median %.0f  p90 %.0f" % (np.median(epi), np.percentile(epi, 90)))
print("workgroup total  median %.0f  mean %.0f" % (np.median(cyc), cyc.mean()))
tot = w(t0.min(), t3.max()) if False else None
# launch span from the stamps (shader clocks are per XCD: use realtime)
span = (r3.max() - r0.min()) / 100e6
print("launch span (realtime) %.1f us; sum of WG times / (256 CUs) %.1f us" % (span * 1e6, real.sum() / 256 * 1e6))
