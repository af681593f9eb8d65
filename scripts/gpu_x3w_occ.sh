#!/bin/bash
# x3_wgrad_kernel at 2 vs 3 blocks/CU (M3D_X3W_OCC): parity, priced launch, ms/step.
set -o pipefail
O=gpurun_out/x3wocc; mkdir -p $O
M3D_X3W_OCC=3 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/t.txt 2>&1 || { tail -20 $O/t.txt; exit 1; }
echo "OCC=3 tests: $(tail -1 $O/t.txt)"
for i in 1 2; do for o in 2 3; do
  M3D_X3W_OCC=$o timeout -k 10 120 python3 scripts/kernels_for_pmc.py wgrad 128 > $O/k$o.txt 2>&1 || { tail -5 $O/k$o.txt; exit 1; }
  echo "OCC=$o $(tail -1 $O/k$o.txt | cut -c1-200)"
done; done
for i in 1 2; do for o in 2 3; do
  M3D_X3W_OCC=$o timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b$o 2>&1 || { tail -5 $O/b$o; exit 1; }
  echo "OCC=$o $(grep -o '"ms_per_step": [0-9.]*' $O/b$o)"
done; done
for o in 2 3; do
  M3D_X3W_OCC=$o timeout -k 10 300 python3 bench.py --steps 6 --warmup 3 --no-extras --size 256 > $O/c$o 2>&1 || { tail -5 $O/c$o; exit 1; }
  echo "OCC=$o 256: $(grep -o '"ms_per_step": [0-9.]*' $O/c$o)"
done
