"""Kernel table of the configs[3] MaskRCNN inference pass:
MaskRCNN.detect on one S^3 synthetic volume, `--reps` timed passes after a
warm-up, meant to run under rocprofv3 --stats so the summary holds the
inference kernels only (divide by --reps for per-volume figures):

    rocprofv3 --stats --kernel-trace -d gpurun_out/inf -o run -- python3 scripts/infer_prof.py --size 256 --reps 5
    python scripts/prof_summary.py gpurun_out/inf/run_kernel_stats.csv 5 40
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "3d-mask-r-cnn_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from m3d.config import synthetic_mrcnn_config
    from m3d.heads import MaskRCNN
    from m3d.model import compose_image_meta, synthetic_volume
    S = a.size
    dev = torch.device("cuda", 0)
    model = MaskRCNN(synthetic_mrcnn_config(S), device=dev, seed=1)
    image = synthetic_volume(S, seed=100).to(dev)
    meta = torch.from_numpy(compose_image_meta(0, [S, S, S, 1], [S, S, S, 1], [0, 0, 0, S, S, S], 1.0,
                                               [0, 1])[None]).to(dev)
    model.detect(image, meta)                  # warm-up (outside the per-volume figures: divide by reps + 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        out = model.detect(image, meta)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(f"infer {S}^3: {el / a.reps * 1e3:.2f} ms/volume over {a.reps} passes, "
          f"{int((out['detections'][0, :, 7] > 0).sum())} detections", flush=True)


if __name__ == "__main__":
    main()
