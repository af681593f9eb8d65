"""Which outputs of m3d_gemm_x3 differ from float64 (debug probe)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch
from m3d import _lib
L = _lib.load()
for nb, M, K, N in [(1, 256, 32, 256), (1, 256, 64, 256), (2, 300, 64, 256), (1, 512, 256, 512)]:
    g = torch.Generator().manual_seed(13)
    A = torch.randn((nb, M, K), generator=g)
    Bt = torch.randn((nb, N, K), generator=g)
    Ad, Bd = A.cuda(), Bt.cuda()
    A3 = torch.empty(3 * A.numel(), dtype=torch.int16, device="cuda")
    B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device="cuda")
    _lib.check(L.m3d_split3_f32(Ad.data_ptr(), A.numel(), A3.data_ptr(), _lib.stream()), "split3")
    _lib.check(L.m3d_split3_f32(Bd.data_ptr(), Bt.numel(), B3.data_ptr(), _lib.stream()), "split3")
    C = torch.full((nb, M, N), 7.0, device="cuda")
    _lib.check(L.m3d_gemm_x3(A3.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, M, K, N, _lib.stream()), "gemm_x3")
    torch.cuda.synchronize()
    ref = torch.bmm(A.double(), Bt.double().transpose(1, 2))
    bad = (C.cpu().double() - ref).abs() > 1e-3 * ref.abs().max()
    print(nb, M, K, N, "bad", int(bad.sum()), "of", bad.numel())
    if bad.any():
        idx = bad.nonzero()
        print("  rows", sorted(set(idx[:, 1].tolist()))[:40])
        print("  cols", sorted(set(idx[:, 2].tolist()))[:40])
        b0 = idx[0].tolist()
        print("  first", b0, float(C[tuple(b0)]), float(ref[tuple(b0)]))
        # is it a k-permutation? compare against A with k-chunks swapped
        for name, perm in [("swap8", torch.arange(K).view(-1, 2, 8).flip(1).reshape(-1))]:
            r2 = torch.bmm(A.double()[:, :, perm], Bt.double().transpose(1, 2))
            print("  ", name, float((C.cpu().double() - r2).abs().max()))
