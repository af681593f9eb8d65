"""bench.py's configs[0] and targets_in_step legs alone (graph + eager)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, synthetic_volume  # noqa: E402

dev = torch.device("cuda")
bench.cpu_baseline = lambda *a, **k: {"skipped": True}
print(json.dumps({"configs0": bench.configs0_leg(dev, 20, 3)}), flush=True)
model = RPN(synthetic_rpn_config(128), device=dev, seed=1)
image = synthetic_volume(128).to(dev)
print(json.dumps({"targets_in_step": bench.targets_in_step_leg(model, image, 20, 3, dev)}), flush=True)
