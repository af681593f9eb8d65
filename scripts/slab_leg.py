"""bench.depth_slab_leg alone at N = 1 (the 256^3 step of BASELINE configs[4]),
with module switches applied first:
    python scripts/slab_leg.py 256 [nn.X=1,...]   -> one JSON line"""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
for item in filter(None, (sys.argv[2] if len(sys.argv) > 2 else "").split(",")):
    key, val = item.split("=")
    mod, attr = key.rsplit(".", 1)
    m = importlib.import_module("m3d." + mod)
    old = getattr(m, attr)
    setattr(m, attr, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
torch.zeros(1, device="cuda:0")                     # initialise the device first
r = bench.depth_slab_leg(S, 5, 2, 0, 1, torch.device("cuda:0"), proposals=True)
print(json.dumps({k: r.get(k) for k in ("ms_per_step", "peak_mem_gb")}))
