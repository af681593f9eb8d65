"""Host-side cost of the 128^3 training step: CPU time to enqueue N steps
without a sync (if it matches the GPU time per step the host bounds the step),
the GPU time per step, and every synchronising call inside a step
(torch.cuda.set_sync_debug_mode "warn").  python scripts/host_overhead.py"""
import os
import sys
import time
import warnings

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]
import torch  # noqa: E402

from m3d.config import synthetic_rpn_config  # noqa: E402
from m3d.model import RPN, RPNTargets, synthetic_rpn_targets, synthetic_volume  # noqa: E402

import m3d.nn as nn  # noqa: E402

GRAPH = "--graph" in sys.argv             # also time the HIP-graph replay's host and GPU cost
NO_PROFILE = "--no-profile" in sys.argv
if "--wgrad-last" in sys.argv:
    nn.WGRAD_LAST = True
dev = torch.device("cuda:0")
S = int(os.environ.get("S", "128"))
cfg = synthetic_rpn_config(S)
model = RPN(cfg, device=dev, seed=1)
image = synthetic_volume(S, seed=100).to(dev)
match, bbox = synthetic_rpn_targets(model.anchors.shape[1], cfg.RPN_TRAIN_ANCHORS_PER_IMAGE, seed=200)
targets = RPNTargets(match, bbox, dev)
for _ in range(3):
    model.train_step(image, targets)
torch.cuda.synchronize()
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    torch.cuda.set_sync_debug_mode("warn")
    model.train_step(image, targets)
    torch.cuda.set_sync_debug_mode(0)
    syncs = [str(x.message).split("\n")[0][:160] for x in w
             if "prototype feature" not in str(x.message)]        # the mode's own notice
torch.cuda.synchronize()
print(f"synchronising calls in one step: {len(syncs)}")
for s in syncs[:12]:
    print("  ", s)
N = 10
t0 = time.perf_counter()
for _ in range(N):
    model.train_step(image, targets)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host enqueue {(t1 - t0) / N * 1e3:.2f} ms/step, wall {(t2 - t0) / N * 1e3:.2f} ms/step")
if GRAPH:
    step = model.graphed_train_step(image, targets, proposals=True)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(N):
        model._graph.replay()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph replay (WGRAD_LAST={nn.WGRAD_LAST}): host {(t1 - t0) / N * 1e3:.2f} ms/replay, "
          f"wall {(t2 - t0) / N * 1e3:.2f} ms/replay")
    t0 = time.perf_counter()
    for _ in range(N):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"graph step (replay + optimizer): host {(t1 - t0) / N * 1e3:.2f} ms/step, wall {(t2 - t0) / N * 1e3:.2f} ms/step")
if NO_PROFILE:
    sys.exit(0)
# where the host's enqueue time goes: cProfile over N more steps (the GPU queue
# stays full, so the profile sees the host's own work, plus any blocking call)
import cProfile  # noqa: E402
import io  # noqa: E402
import pstats  # noqa: E402

pr = cProfile.Profile()
pr.enable()
for _ in range(N):
    model.train_step(image, targets)
pr.disable()
torch.cuda.synchronize()
for key in ("tottime", "cumulative"):
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats(key).print_stats(35)
    print(f"--- cProfile over {N} steps, by {key} (seconds are for all {N} steps)")
    print("\n".join(l for l in buf.getvalue().splitlines() if l.strip())[:9000])
