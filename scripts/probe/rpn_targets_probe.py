"""Per-kernel time of the in-step RPN target builder at 128^3 (rocprofv3 probe)."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import numpy as np
import torch
from m3d.anchors import get_anchors
from m3d.config import synthetic_rpn_config
from m3d.targets import RPNTargetBuilder
S = int(sys.argv[1]) if len(sys.argv) > 1 else 128
cfg = synthetic_rpn_config(S)
anchors = torch.from_numpy(get_anchors(cfg)).cuda()
rng = np.random.default_rng(11)
side = rng.uniform(12, 40, (8, 3)) / S
lo = rng.uniform(0, 1, (8, 3)) * (1 - side)
gt = torch.from_numpy(np.concatenate([lo, lo + side], 1).astype(np.float32)).cuda()
b = RPNTargetBuilder(anchors, cfg, max_gt=8)
for i in range(6):
    b(gt, seed=i)
torch.cuda.synchronize()
print("A", anchors.shape[0], "counts", b.counts.tolist())
