"""fp32 GEMM accuracy and speed of the current GEMM mode (M3D_GEMM_X3=0 f32 MFMA,
=2 the same split3 arithmetic as the Winograd x3_gemm_kernel, in the conv kernel):
m3d_gemm_f32 against a float64 matmul (max |err| / max |ref|, rms err / rms ref)
for K up to the direct 3^3 conv depth, and the time of the bench's priced
launch shape (96 batched 8192x256x512 GEMMs)."""
import json
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d import _lib  # noqa: E402

L = _lib.load()
dev = torch.device("cuda")
out = {"x3": os.environ.get("M3D_GEMM_X3", "0")}
for nb, M, K, N in [(4, 1024, 256, 512), (2, 1024, 6912, 256), (1, 2048, 1728, 64)]:
    g = torch.Generator().manual_seed(K)
    A = torch.randn((nb, M, K), generator=g)
    B = torch.randn((nb, K, N), generator=g) / K ** 0.5
    ref = torch.bmm(A.double(), B.double())
    Ad, Bd = A.to(dev), B.to(dev)
    C = torch.zeros((nb, M, N), device=dev)
    _lib.check(L.m3d_gemm_f32(Ad.data_ptr(), Bd.data_ptr(), C.data_ptr(), nb, M, K, N, None, 0, 0,
                              _lib.stream()), "gemm")
    got = C.double().cpu()
    # the fp32 rounding of the exact result: the floor any fp32 GEMM reaches
    e = (got - ref)
    out[f"{nb}x{M}x{K}x{N}"] = {"max_rel": float(e.abs().max() / ref.abs().max()),
                                "rms_rel": float(e.pow(2).mean().sqrt() / ref.pow(2).mean().sqrt())}
nb, M, K, N = 96, 8192, 256, 512
A = torch.randn((nb, M, K), device=dev)
B = torch.randn((nb, K, N), device=dev)
C = torch.empty((nb, M, N), device=dev)
s = torch.cuda.current_stream()
for _ in range(3):
    L.m3d_gemm_f32(A.data_ptr(), B.data_ptr(), C.data_ptr(), nb, M, K, N, None, 0, 0, _lib.stream())
t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0.record(s)
for _ in range(10):
    L.m3d_gemm_f32(A.data_ptr(), B.data_ptr(), C.data_ptr(), nb, M, K, N, None, 0, 0, _lib.stream())
t1.record(s)
torch.cuda.synchronize()
ms = t0.elapsed_time(t1) / 10
out["priced_gemm_ms"] = round(ms, 3)
out["priced_gemm_tflops"] = round(2 * nb * M * K * N / ms / 1e9, 1)
print(json.dumps(out))
