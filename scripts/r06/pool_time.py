"""The stem pool at 256^3 (C1 [1,128,128,256,64] -> [1,64,64,256,64]): the
specialised maxpool_fwd333 / bwd333 kernels (m3d_maxpool3d_fwd/bwd) against
the general z-run kernels (the slab form with no neighbours), event-timed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d import _lib  # noqa: E402

L = _lib.load()
S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
B, H, W, D, C = 1, S // 2, S // 2, S, 64
OH, OW = H // 2, W // 2
x = torch.randn((B, H, W, D, C), device="cuda")
halo = torch.zeros((B, H, W, 2, C), device="cuda")
y = torch.empty((B, OH, OW, D, C), device="cuda")
am = torch.empty((B, OH, OW, D, C), device="cuda", dtype=torch.uint8)
dy = torch.randn_like(y)
dx = torch.empty_like(x)
dh = torch.zeros_like(halo)
st = _lib.stream()
args = (3, 3, 3, 2, 2, 1, 0, 0, 1, OH, OW, D)
f_new = lambda: L.m3d_maxpool3d_fwd(x.data_ptr(), B, H, W, D, C, *args, y.data_ptr(), am.data_ptr(), st)  # noqa
f_old = lambda: L.m3d_maxpool3d_fwd_halo(x.data_ptr(), halo.data_ptr(), 0, 0, 1, B, H, W, D, C, *args,  # noqa
                                         y.data_ptr(), am.data_ptr(), st)
b_new = lambda: L.m3d_maxpool3d_bwd(dy.data_ptr(), am.data_ptr(), B, H, W, D, C, *args, dx.data_ptr(), st)  # noqa
b_old = lambda: L.m3d_maxpool3d_bwd_halo(dy.data_ptr(), am.data_ptr(), 0, 0, 1, B, H, W, D, C, *args,  # noqa
                                         dx.data_ptr(), dh.data_ptr(), st)
byf = 4 * x.numel() + 5 * y.numel()
byb = 5 * y.numel() + 4 * x.numel()
for name, fn, by in (("fwd333", f_new, byf), ("fwd4z", f_old, byf), ("bwd333", b_new, byb), ("bwd4z", b_old, byb),
                     ("fwd333", f_new, byf), ("fwd4z", f_old, byf), ("bwd333", b_new, byb), ("bwd4z", b_old, byb)):
    t = bench._event_time(fn, 10)
    print(f"{name} {t * 1e3:.3f} ms  {by / t / 1e12:.2f} TB/s")
