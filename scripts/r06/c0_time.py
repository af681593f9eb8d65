"""Where configs[0]'s graphed step goes: host time of the builder launch, the
replay call and the optimizer, against the GPU time of one replay (events)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN  # noqa: E402
from m3d.targets import RPNTargetBuilder  # noqa: E402
from m3d.toydata import network_input, toy_volume  # noqa: E402

dev = torch.device("cuda")
S = 64
v = toy_volume(S, seed=5)
cfg = synthetic_rpn_config(S)
model = RPN(cfg, device=dev, seed=1)
image = torch.from_numpy(network_input(v["image"])).to(dev)
gt = torch.from_numpy((v["boxes"] / np.float32(S)).astype(np.float32)).to(dev)
builder = RPNTargetBuilder(model.anchors.reshape(-1, 6), cfg, max_gt=32)
t = builder(gt, seed=0)
step = model.graphed_train_step(image, t, warmup=2)
graph = model._graph
for i in range(3):
    builder(gt, seed=i)
    step()
torch.cuda.synchronize()
hb, hr, ho, gpu = [], [], [], []
for i in range(20):
    a = time.perf_counter()
    builder(gt, seed=10 + i)
    b = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    c = time.perf_counter()
    model.sgd_step()
    d = time.perf_counter()
    hb.append(b - a); hr.append(c - b); ho.append(d - c)
    torch.cuda.synchronize()
    gpu.append(e0.elapsed_time(e1) / 1e3)
med = lambda x: round(float(np.median(x)) * 1e3, 3)  # noqa: E731
print({"host_builder_ms": med(hb), "host_replay_ms": med(hr), "host_optimizer_ms": med(ho),
       "gpu_replay_ms": med(gpu), "graph_nodes": None})
# back-to-back wall
torch.cuda.synchronize()
a = time.perf_counter()
for i in range(20):
    builder(gt, seed=50 + i)
    step()
torch.cuda.synchronize()
print({"wall_ms_per_step": round((time.perf_counter() - a) / 20 * 1e3, 3)})
