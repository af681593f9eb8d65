"""Same-box A/B of nn.X3_BN_FUSE (the BN-ReLU backward in the bf16-split 1x1x1
data gradient's epilogue): the 256^3 depth-slab step (N = 1) with the flag off
and on, twice.  python scripts/r06/fuse_ab.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d import nn as mnn  # noqa: E402

bench.step_roofline = lambda *a, **k: None
dev = torch.device("cuda")
for rep in range(2):
    for on in (False, True):
        mnn.X3_BN_FUSE = on
        r = bench.depth_slab_leg(256, 5, 2, 0, 1, dev)
        print(json.dumps({"x3_bn_fuse": on, "ms_per_step": r["ms_per_step"], "peak_mem_gb": r["peak_mem_gb"]}),
              flush=True)
