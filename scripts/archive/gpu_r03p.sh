#!/bin/bash
# 256^3 depth-slab leg (N=1): time + allocator statistics per configuration
set -o pipefail
OUT=gpurun_out/r03p
mkdir -p $OUT
export TMPDIR=/tmp
for e in "M3D_WINO_WGRAD_NZ=4" "M3D_WINO_WGRAD_NZ=4 PYTORCH_CUDA_ALLOC_CONF=expandable_segments:True" "M3D_WINO_WGRAD_NZ=2"; do
  env $e timeout -k 10 400 python -u - > $OUT/s.json 2> $OUT/s.err <<'PY' || { tail -20 $OUT/s.err; exit 1; }
import json, sys, time
sys.path[:0] = [".", "3d-mask-r-cnn_amd"]
import torch
import bench
dev = torch.device("cuda:0")
free, total = torch.cuda.mem_get_info(dev)
r = bench.depth_slab_leg(256, 5, 2, 0, 1, dev)
st = torch.cuda.memory_stats(dev)
print(json.dumps({"ms": r["ms_per_step"], "peak_alloc_gb": r["peak_mem_gb"],
                  "peak_reserved_gb": round(st["reserved_bytes.all.peak"] / 1e9, 1),
                  "alloc_retries": st["num_alloc_retries"], "device_allocs": st.get("num_device_alloc"),
                  "device_frees": st.get("num_device_free"), "free_gb_at_start": round(free / 1e9, 1),
                  "total_gb": round(total / 1e9, 1)}))
PY
  echo "$e $(tail -n 1 $OUT/s.json)"
done
