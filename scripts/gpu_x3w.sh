#!/bin/bash
# X3 weight-gradient GEMM: GPU tests, the priced wgrad GEMM (bench roofline
# leg) f32 vs X3, bench ms/step alternating (3x).
set -o pipefail
O=gpurun_out/x3w; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for v in "M3D_GEMM_X3=1" "M3D_GEMM_X3=5"; do
  env $v timeout -k 10 120 python3 -c "
import sys; sys.path[:0]=['.','3d-mask-r-cnn_amd']
import bench, json
r=bench.time_dominant_kernel(128)
print(json.dumps({k: r[k] for k in ('achieved','frac','avg_launch_ms')}))" > $O/g 2>&1 || { tail -5 $O/g; exit 1; }
  echo "$v $(tail -1 $O/g)"
done
for i in 1 2 3; do for v in "M3D_GEMM_X3=1" "M3D_GEMM_X3=5"; do
  env $v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b 2>&1 || { tail -5 $O/b; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b)"
done; done
