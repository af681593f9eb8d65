"""bench.fwd_roofline alone at 256^3 (python scripts/fwd_roofline_256.py [S] [nn.X=1,...]) (the roi_align_256 leg's backbone / FPN /
RPN-head forward roofline) -- one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, synthetic_volume  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 256
if len(sys.argv) > 2:                       # module switches, as scripts/bench_ab.py takes them
    import importlib
    for item in filter(None, sys.argv[2].split(",")):
        key, val = item.split("=")
        mod, attr = key.rsplit(".", 1)
        m = importlib.import_module("m3d." + mod)
        old = getattr(m, attr)
        setattr(m, attr, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
dev = torch.device("cuda:0")
model = RPN(synthetic_rpn_config(S), device=dev, seed=1)
image = synthetic_volume(S).to(dev)
with torch.no_grad():
    model.features(image)
torch.cuda.synchronize()
print(json.dumps(bench.fwd_roofline(model, image)))
