"""Runs the dominant conv kernel (rpn_conv_shared1 fwd on P2 @128^3) and the
PyramidROIAlign 14^3 / 7^3 kernels a few times each, for rocprofv3 --pmc passes."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch
import bench
from m3d.config import synthetic_rpn_config
from m3d.model import RPN, synthetic_volume

dev = torch.device("cuda")
S = 128
model = RPN(synthetic_rpn_config(S), device=dev, seed=1)
with torch.no_grad():
    fmaps = model.features(synthetic_volume(S).to(dev))
print(bench.time_dominant_conv(model, fmaps, reps=3))
print(bench.time_roi_align(fmaps, S, reps=3))
