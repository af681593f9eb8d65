"""Same-box A/B of the 256^3 depth-slab step (N = 1) under data-gradient tile
policies (nn.WINO_DGRAD_Y4): slab_ab.py POLICY [POLICY ...]; '-' = default."""
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
pols = sys.argv[1:] or ["-"]
for rep in range(2):
    for pol in pols:
        mnn.WINO_DGRAD_Y4 = "" if pol == "-" else pol
        r = bench.depth_slab_leg(256, 5, 2, 0, 1, dev)
        print(json.dumps({"policy": pol, "ms_per_step": r["ms_per_step"], "peak_mem_gb": r["peak_mem_gb"]}),
              flush=True)
