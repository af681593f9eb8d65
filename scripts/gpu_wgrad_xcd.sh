#!/bin/bash
# wgrad XCD remap check: GPU conv tests, priced wgrad GEMM time + HBM traffic
# (FETCH/WRITE passes), bench ms/step.
set -o pipefail
O=gpurun_out/wx; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1 || { tail -20 $O/tests.txt; exit 1; }
tail -1 $O/tests.txt
LEGS="gemm:conv_wgrad_kernel:wino_wgrad_gemm_rpn_shared1_S128" bash scripts/gpu_prof.sh r01q 128 > $O/prof.txt 2>&1 || { tail -20 $O/prof.txt; exit 1; }
tail -14 $O/prof.txt
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-extras > $O/b 2>&1 || exit 1
grep -o '"ms_per_step": [0-9.]*' $O/b
