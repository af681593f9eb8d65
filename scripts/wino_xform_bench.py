"""Winograd forward + data gradient of one 3x3x3 conv shape, repeated, for a
rocprofv3 --kernel-trace --stats view of the input / output transform kernels
(wino_input_kernel, wino_output_kernel) against their algorithmic bytes.
SHAPE=H,W,D,Cin,Cout (default 32,32,32,256,512), REPS (20)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402

H, W, D, Cin, Cout = (int(v) for v in os.environ.get("SHAPE", "32,32,32,256,512").split(","))
REPS = int(os.environ.get("REPS", "20"))
L = _lib.load()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn((1, H, W, D, Cin), device=dev, generator=g)
w = torch.randn((3, 3, 3, Cin, Cout), device=dev, generator=g) * 0.05
dy = torch.randn((1, H, W, D, Cout), device=dev, generator=g)
y = torch.empty((1, H, W, D, Cout), device=dev)
dx = torch.empty((1, H, W, D, Cin), device=dev)
wsb = int(L.m3d_conv3d_wino_workspace_bytes(1, H, W, D, D, Cin, Cout))
ws = torch.empty(wsb, device=dev, dtype=torch.uint8)
p = _lib.ptr
s = _lib.stream()
for _ in range(REPS):
    _lib.check(L.m3d_conv3d_fwd_wino(p(x), 1, H, W, D, Cin, p(w), Cout, D, 1, None, None, None, None, 0,
                                     None, p(y), p(ws), wsb, s), "fwd_wino")
    _lib.check(L.m3d_conv3d_bwd_data_wino(p(dy), p(w), 1, H, W, D, Cin, Cout, D, 1, p(dx), 0, p(ws), wsb, s),
               "bwd_data_wino")
torch.cuda.synchronize()
T = ((H + 1) // 2) * ((W + 1) // 2) * ((D + 3) // 4)
print(f"shape {H}x{W}x{D} {Cin}->{Cout}: tiles {T}; fwd input transform algorithmic "
      f"{(H * W * D * Cin + 96 * T * Cin) * 4 / 1e6:.1f} MB, dgrad {(H * W * D * Cout + 96 * T * Cout) * 4 / 1e6:.1f} MB; "
      f"output transform fwd {(96 * T * Cout + H * W * D * Cout) * 4 / 1e6:.1f} MB, dgrad {(96 * T * Cin + H * W * D * Cin) * 4 / 1e6:.1f} MB")
