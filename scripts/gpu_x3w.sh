#!/bin/bash
# X3 weight-gradient variants: GPU tests, bench ms/step alternating (3x).
set -o pipefail
O=gpurun_out/x3w; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_slab.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
for i in 1 2 3; do for v in ${VARIANTS:-"M3D_GEMM_X3=5" "M3D_GEMM_X3=13"}; do
  env $v timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b 2>&1 || { tail -5 $O/b; exit 1; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/b)"
done; done
