#!/bin/bash
# Winograd U in fp32 + split in x3_gemm_kernel (M3D_GEMM_X3 bit 4) vs pre-split planes:
# GPU tests under the variant, Winograd fwd time, ms/step alternating.
set -o pipefail
O=gpurun_out/af32; mkdir -p $O
M3D_GEMM_X3=29 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
echo "bit4 tests: $(tail -1 $O/tests.txt)"
for v in 13 29; do
  M3D_GEMM_X3=$v timeout -k 10 120 python3 -c "
import sys; sys.path[:0]=['.','3d-mask-r-cnn_amd']
import bench; print(bench.time_wino_fwd(128, reps=10), bench.time_wino_fwd(256, reps=3))" > $O/w$v.txt 2>&1 || { tail -5 $O/w$v.txt; exit 1; }
  echo "X3=$v wino fwd: $(tail -1 $O/w$v.txt)"
done
for i in 1 2; do for v in 13 29; do
  M3D_GEMM_X3=$v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b$v 2>&1 || { tail -5 $O/b$v; exit 1; }
  echo "X3=$v $(grep -o '"ms_per_step": [0-9.]*' $O/b$v)"
done; done
for v in 13 29; do
  M3D_GEMM_X3=$v timeout -k 10 300 python3 bench.py --steps 4 --warmup 2 --no-extras --size 256 > $O/c$v 2>&1 || { tail -5 $O/c$v; exit 1; }
  echo "X3=$v 256: $(grep -o '"ms_per_step": [0-9.]*' $O/c$v)"
done
