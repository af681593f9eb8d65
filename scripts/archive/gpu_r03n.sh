#!/bin/bash
# 256^3 depth-slab leg (N=1) with the kept-U weight gradient: time and peak memory, both tile choices
set -o pipefail
OUT=gpurun_out/r03n
mkdir -p $OUT
export TMPDIR=/tmp
for nz in 4 2; do
  M3D_WINO_WGRAD_NZ=$nz timeout -k 10 400 python -u - > $OUT/s$nz.json 2> $OUT/s$nz.err <<'PY' || { tail -20 $OUT/s$nz.err; exit 1; }
import json, sys
sys.path[:0] = [".", "3d-mask-r-cnn_amd"]
import torch
import bench
r = bench.depth_slab_leg(256, 5, 2, 0, 1, torch.device("cuda:0"))
print(json.dumps({k: r[k] for k in ("ms_per_step", "volumes_per_s", "loss", "peak_mem_gb")}))
PY
  echo "NZ=$nz $(tail -n 1 $OUT/s$nz.json)"
done
bash scripts/gpu_step_ab.sh r03n/ab "M3D_WINO_WGRAD_MIN_C=128" "M3D_WINO_WGRAD_MIN_C=64" || true
