"""Same-box A/B of m3d module constants on the 256^3 depth-slab step (N = 1):
mod_ab.py SPEC [SPEC ...], SPEC = "nn.NAME=VALUE,..." or "-" (defaults); each
spec twice, interleaved."""
import importlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

bench.step_roofline = lambda *a, **k: None
dev = torch.device("cuda")
specs = sys.argv[1:] or ["-"]
saved = {}
for spec in specs:
    for item in filter(None, spec.split(",")) if spec != "-" else []:
        key = item.split("=")[0]
        mod, attr = key.rsplit(".", 1)
        m = importlib.import_module("m3d." + mod)
        saved[key] = (m, attr, getattr(m, attr))
for rep in range(2):
    for spec in specs:
        for m, attr, v in saved.values():
            setattr(m, attr, v)
        for item in filter(None, spec.split(",")) if spec != "-" else []:
            key, val = item.split("=")
            m, attr, old = saved[key]
            setattr(m, attr, type(old)(int(val)) if isinstance(old, (bool, int)) else type(old)(val))
        r = bench.depth_slab_leg(256, 5, 2, 0, 1, dev)
        print(json.dumps({"spec": spec, "ms_per_step": r["ms_per_step"], "peak_mem_gb": r["peak_mem_gb"]}), flush=True)
