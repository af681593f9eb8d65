#!/bin/bash
# 256^3 depth-slab leg (N=1, standalone): allocator behaviour per configuration, each twice
set -o pipefail
OUT=gpurun_out/r03r
mkdir -p $OUT
export TMPDIR=/tmp
for rep in 1; do
for e in "M3D_WGRAD_THROTTLE_EVERY=4" "M3D_WGRAD_THROTTLE_EVERY=2" "M3D_WGRAD_THROTTLE_EVERY=8" "M3D_WGRAD_THROTTLE=0.4"; do
  env $e timeout -k 10 400 python -u - > $OUT/s.json 2> $OUT/s.err <<'PY' || { tail -20 $OUT/s.err; exit 1; }
import json, sys, time
sys.path[:0] = [".", "3d-mask-r-cnn_amd"]
import torch
import bench
dev = torch.device("cuda:0")
r = bench.depth_slab_leg(256, 5, 2, 0, 1, dev)
st = torch.cuda.memory_stats(dev)
print(json.dumps({"ms": r["ms_per_step"], "peak_alloc_gb": r["peak_mem_gb"],
                  "peak_reserved_gb": round(st["reserved_bytes.all.peak"] / 1e9, 1),
                  "device_allocs": st.get("num_device_alloc"), "device_frees": st.get("num_device_free")}))
PY
  echo "$e $(tail -n 1 $OUT/s.json)"
done
done
