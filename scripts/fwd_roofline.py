"""Forward roofline legs of bench.py (backbone / FPN / RPN head) at the given sizes."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, synthetic_volume  # noqa: E402

dev = torch.device("cuda")
for S in [int(v) for v in (sys.argv[1:] or ["128", "256"])]:
    model = RPN(synthetic_rpn_config(S), device=dev, seed=1)
    print(S, json.dumps(bench.fwd_roofline(model, synthetic_volume(S).to(dev))), flush=True)
    del model
    torch.cuda.empty_cache()
