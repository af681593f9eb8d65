#!/bin/bash
# Winograd workspace arena: model / determinism (HIP graph) / slab tests, then the 256^3
# depth-slab leg with and without the arena, allocator statistics
set -o pipefail
OUT=gpurun_out/r03q
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_slab.py tests/test_gpu_dp.py -m gpu > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for e in "M3D_WINO_ARENA=1" "M3D_WINO_ARENA=0" "M3D_WINO_ARENA=1"; do
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
