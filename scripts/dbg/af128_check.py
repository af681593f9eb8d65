"""m3d_gemm_x3_af on fixed random operands (the priced Winograd shape and a
ragged one); writes C to OUT.npy so two library configurations (M3D_X3_AF128)
can be compared bit for bit."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import numpy as np
import torch
from m3d import _lib
L = _lib.load()
outs = []
for (nb, T, K, N) in [(96, 8192, 256, 512), (5, 1000, 96, 256), (3, 300, 512, 128)]:
    g = torch.Generator(device="cuda").manual_seed(7)
    A = torch.randn((nb, T, K), device="cuda", generator=g)
    Bt = torch.randn((nb, N, K), device="cuda", generator=g) * 0.05
    B3 = torch.empty(3 * Bt.numel(), dtype=torch.int16, device="cuda")
    _lib.check(L.m3d_split3_f32(Bt.data_ptr(), Bt.numel(), B3.data_ptr(), _lib.stream()), "split3")
    C = torch.full((nb, T, N), 7.0, device="cuda")
    _lib.check(L.m3d_gemm_x3_af(A.data_ptr(), B3.data_ptr(), C.data_ptr(), nb, T, K, N, _lib.stream()), "af")
    ref = torch.bmm(A.double(), Bt.double().transpose(1, 2))
    err = float((C.double() - ref).abs().max() / ref.abs().max())
    print(nb, T, K, N, "rel err vs fp64", err, flush=True)
    assert err < 1e-5
    outs.append(C.cpu().numpy().ravel())
np.save(sys.argv[1], np.concatenate(outs))
