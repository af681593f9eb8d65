"""1x1x1 conv weight gradients of the 128^3 step's shapes, alone (no side
stream, no concurrent work), for a rocprofv3 --kernel-trace --stats view:
which kernel runs each shape and at what rate.  SHAPES=H,W,D,Cin,Cout;...
(default: the res2..res5 / FPN / RPN 1^3 shapes at 128^3), REPS (10)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402

DEF = ("32,32,128,64,64;32,32,128,256,64;32,32,128,64,256;16,16,128,512,128;16,16,128,128,512;"
       "8,8,128,1024,256;8,8,128,256,1024;4,4,128,2048,512;4,4,128,512,2048;32,32,128,256,256;32,32,128,512,512")
shapes = [tuple(int(v) for v in s.split(",")) for s in os.environ.get("SHAPES", DEF).split(";")]
REPS = int(os.environ.get("REPS", "10"))
L = _lib.load()
dev = torch.device("cuda:0")
p = _lib.ptr
ev = []
for (H, W, D, Cin, Cout) in shapes:
    x = torch.randn((1, H, W, D, Cin), device=dev)
    dz = torch.randn((1, H, W, D, Cout), device=dev)
    dw = torch.zeros((1, 1, 1, Cin, Cout), device=dev)
    for _ in range(2):
        _lib.check(L.m3d_conv3d_bwd_weight(p(x), p(dz), 1, H, W, D, Cin, 1, 1, 1, Cout, H, W, D, 1, 1, 1, 0, 0, 0,
                                           p(dw), _lib.stream()), "bwd_weight")
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(REPS):
        _lib.check(L.m3d_conv3d_bwd_weight(p(x), p(dz), 1, H, W, D, Cin, 1, 1, 1, Cout, H, W, D, 1, 1, 1, 0, 0, 0,
                                           p(dw), _lib.stream()), "bwd_weight")
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / REPS
    M = H * W * D
    fl = 2.0 * M * Cin * Cout
    by = 4.0 * M * (Cin + Cout)
    print(f"M={M:7d} Cin={Cin:5d} Cout={Cout:5d}: {ms * 1e3:7.1f} us  {fl / ms / 1e9:6.1f} TFLOP/s  {by / ms / 1e9:6.2f} TB/s")
