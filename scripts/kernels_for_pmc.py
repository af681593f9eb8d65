"""Runs ONE priced launch of bench.py a few times for the rocprofv3 --pmc
passes of scripts/gpu_prof.sh:  kernels_for_pmc.py LEG [S]
  gemm    the Winograd point GEMM launch of rpn_conv_shared1 (x3_gemm256_af_kernel)
  wgrad   the dominant kernel's largest launch: batched Winograd weight-gradient GEMM of rpn_conv_shared1 (x3_wgrad_kernel)
  direct  rpn_conv_shared1 as a direct implicit-GEMM conv on P2
  roi7 / roi14  PyramidROIAlign 7^3 / 14^3 at configs[2] shapes
  infer   MaskRCNN inference (configs[3]) x3 after one warm-up
The priced kernel's dispatches are the LAST ones of its name in the trace."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

leg = sys.argv[1]
S = int(sys.argv[2]) if len(sys.argv) > 2 else 128
NR = 128 if S == 128 else 512          # configs[2] / configs[3] ROI counts (bench.py)
if leg == "gemm":
    print(bench.time_wino_gemm(S, reps=20))      # 20: the cold first launch moves the average < 2 %
elif leg == "wgrad":
    print(bench.time_wgrad_gemm(S, reps=20))
elif leg == "winofwd":
    # rpn_conv_shared1 on P2 as a Winograd conv through the C-ABI (M3D_GEMM_X3 picks the GEMM)
    from m3d import _lib
    L = _lib.load()
    B, H, W, D, Cin, Cout = 1, S // 4, S // 4, S, 256, 512
    x = torch.randn((B, H, W, D, Cin), device="cuda")
    w = torch.randn((3, 3, 3, Cin, Cout), device="cuda") / (27 * Cin) ** 0.5
    y = torch.empty((B, H, W, D, Cout), device="cuda")
    nb = L.m3d_conv3d_wino_workspace_bytes(B, H, W, D, D, Cin, Cout)
    ws = torch.empty(nb // 4 + 64, device="cuda")
    for _ in range(3):
        _lib.check(L.m3d_conv3d_fwd_wino(x.data_ptr(), B, H, W, D, Cin, w.data_ptr(), Cout, D, 1, None, None,
                                         None, None, 0, None, y.data_ptr(), ws.data_ptr(), nb, _lib.stream()),
                   "wino")
    torch.cuda.synchronize()
elif leg == "infer":
    print(bench.mrcnn_inference_leg(S, 3, 1, torch.device("cuda")))
else:
    from m3d.config import synthetic_rpn_config
    from m3d.model import RPN, synthetic_volume
    model = RPN(synthetic_rpn_config(S), device=torch.device("cuda"), seed=1)
    with torch.no_grad():
        fmaps = model.features(synthetic_volume(S).to("cuda"))
    torch.cuda.synchronize()
    if leg.startswith("roibwd"):
        print(bench.time_roi_align_bwd(fmaps, S, n_rois=NR, reps=5, pools=(int(leg[6:]),),
                                       hi=128 if S == 128 else S))
    elif leg == "direct":
        print(bench.time_direct_conv(model, fmaps, reps=3))
    else:
        print(bench.time_roi_align(fmaps, S, n_rois=NR, reps=3, pools=(int(leg[3:]),),
                                   hi=128 if S == 128 else S))
